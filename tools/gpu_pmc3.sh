#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc3; export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --latency-iters 0"
i=0
for grp in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VALU SQ_WAVES" \
           "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc3/p$i -o run -- $B > gpurun_out/pmc3/p$i.out 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -2 gpurun_out/pmc3/p$i.out
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
mkdir -p gpurun_out/pmc3/all; for j in $(seq 1 $i); do cp gpurun_out/pmc3/p$j/run_counter_collection.csv gpurun_out/pmc3/all/pass$j.csv 2>/dev/null; done
python3 tools/pmc_summary.py gpurun_out/pmc3/all 1048576 2.2

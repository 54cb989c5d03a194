#!/bin/bash
# Quick PMC on the current build: instruction count, issue rate, waits (comb + finish kernels)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc2; export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --latency-iters 0"
i=0
for grp in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM" "FETCH_SIZE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc2/p$i -o run -- $B > gpurun_out/pmc2/p$i.out 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
mkdir -p gpurun_out/pmc2/all; for j in $(seq 1 $i); do cp gpurun_out/pmc2/p$j/run_counter_collection.csv gpurun_out/pmc2/all/pass$j.csv 2>/dev/null; done
python3 tools/pmc_summary.py gpurun_out/pmc2/all 1048576 ${MS:-2.35}

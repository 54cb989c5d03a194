#!/bin/bash
# PMC passes on the current build (one counter group per rocprofv3 run, --pmc only, no tracing domains).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; D=gpurun_out/pmc_cur; rm -rf $D; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $D/counters_list.txt 2>&1 || true
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras"
i=0
for grp in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "VALUBusy VALUUtilization" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $D/p$i -o run -- $B > $D/p$i.out 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $D/p$i.out; if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then exit $rc; fi; fi
done
mkdir -p $D/all; for j in $(seq 1 $i); do cp $D/p$j/run_counter_collection.csv $D/all/pass$j.csv 2>/dev/null; done
echo "== comb_kernel"; KERNEL=comb_kernel python3 tools/pmc_summary.py $D/all 1048576
echo "== finish_kernel"; KERNEL=finish_kernel python3 tools/pmc_summary.py $D/all 1048576

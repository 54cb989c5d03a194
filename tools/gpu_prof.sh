#!/bin/bash
# Profiles of the bench launch pair (2^20 round): one rocprofv3 --kernel-trace --stats run, then the PMC passes
# (one counter group per rocprofv3 run, --pmc only, no tracing domains), each step under its own time limit;
# tools/pmc_derive.py turns them into derived.json (VALU instructions per signature, VALUBusy, HBM bytes with the
# gfx950 FETCH_SIZE x2 correction).   usage: [SIGS=n] tools/gpu_prof.sh TAG [extra bench args]
# (SIGS: signatures per launch for the derivation, default 1048576; e.g. SIGS=131072 ... --seqs 256 = the 8-GPU shard)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-run}; shift; D=gpurun_out/prof_$TAG; rm -rf $D; mkdir -p $D; export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 3 --no-cpu --no-extras $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $B > $D/trace.out 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 $D/trace.out; exit $rc; }
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras $*"
i=0
for grp in "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "VALUBusy VALUUtilization" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d $D/p$i -o run -- $B > $D/p$i.out 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $D/p$i.out; exit $rc; fi
done
mkdir -p $D/all; for j in $(seq 1 $i); do cp $D/p$j/run_counter_collection.csv $D/all/pass$j.csv; done
find $D/trace -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \;
python3 tools/pmc_derive.py $D/all 10 13 ${SIGS:-1048576} $D/kernel_stats.csv > $D/derive.out 2>&1; echo "derive rc=$?"
rm -rf $D/p*/ $D/trace/*/*/*results.db 2>/dev/null; true

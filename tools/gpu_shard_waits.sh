#!/bin/bash
# where do the 131k shard's comb waves wait?  (1) the stamped diagnostic build's per-wave phases
# at 131k and 2^20 (tools/comb_stamps.py), (2) SQ wait-state counters of the bench's launch pair at both sizes, one
# rocprofv3 --pmc pass each (8 SQ counters), each step under its own limit.   usage: tools/gpu_shard_waits.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}; D=gpurun_out/waits_$TAG; rm -rf $D; mkdir -p $D
timeout -k 10 240 python -u tools/comb_stamps.py build/ab/libpbft_stamps.so 131072 1048576 > $D/stamps.txt 2>&1 || { tail -5 $D/stamps.txt; exit 1; }
cat $D/stamps.txt
G="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for sz in 256 2048; do
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d $D/p$sz -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras --seqs $sz > $D/p$sz.out 2>&1
  rc=$?; echo "pmc seqs=$sz rc=$rc"; [ $rc -ne 0 ] && { tail -3 $D/p$sz.out; exit $rc; }
  find $D/p$sz -name "*counter_collection.csv" -exec cp {} $D/pmc_seqs$sz.csv \;
done
python3 tools/pmc_waits.py $D/pmc_seqs256.csv $D/pmc_seqs2048.csv | tee $D/waits.txt
rm -rf $D/p256 $D/p2048

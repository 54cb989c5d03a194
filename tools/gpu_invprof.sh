#!/bin/bash
# rocprofv3 kernel durations of the old / new inversion at the 131k shard and at 2^20 (one library per run;
# build/abx is gpurun-ignored after r06, see tools/gpu_inv.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
D=gpurun_out/r06_invprof; mkdir -p $D
for L in invold invbat; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/$L -o $L -- python3 tools/ab.py build/abx/libpbft_$L.so --replicas 16 --seqs 32768 --sizes 131072,1048576 --rounds 8 --iters 20 > $D/$L.txt 2>&1 || exit 1
  rm -f $D/$L/*kernel_trace.csv
done

#!/bin/bash
# Comb placement (PBFT_OPT_COMB_SPREAD): stamped build's per-SIMD placement and phases off / on, then the interleaved
# timing A/B of the product library, each step under its own limit.   usage: tools/gpu_spread.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}; D=gpurun_out/spread_$TAG; mkdir -p $D
for sp in 0 1; do
  PBFT_COMB_SPREAD=$sp timeout -k 10 240 python -u tools/comb_stamps.py build/ab/libpbft_stamps.so 131072 65536 1048576 > $D/stamps_spread$sp.txt 2>&1 || { tail -5 $D/stamps_spread$sp.txt; exit 1; }
done
timeout -k 10 300 python -u tools/opt_ab.py 12 0 1 --sizes 131072,65536,98304,196608,262144,1048576 > $D/ab.txt 2>&1 || { tail -5 $D/ab.txt; exit 1; }
grep -E "==|placement|shared by|lifetime|end us" $D/stamps_spread*.txt; cat $D/ab.txt

#!/bin/bash
# round 4: finish width / waves per SIMD at 2^20 and 2^19 with the row-wise product tree (options 2 = width,
# 8 = waves per SIMD), one process, interleaved, 16-position plan.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=pbft_amd/libpbft_verify.so
timeout -k 10 400 python -u tools/ab.py $L@3=20000 $L@3=20000,2=8,8=1 $L@3=20000,2=4,8=2 $L@3=20000,2=4,8=1 --sizes 1048576,524288 --rounds 10 > gpurun_out/ab_finw.txt 2>&1; rc=$?
grep -v "^W2026" gpurun_out/ab_finw.txt
[ $rc -ne 0 ] && exit $rc
# the 131k shard (one GPU of 8 at config #4): kernel trace + PMC passes of the bench headline at --seqs 256
SIGS=131072 bash tools/gpu_prof.sh shard --seqs 256; rc=$?
cat gpurun_out/prof_shard/derive.out | head -30; exit $rc

#!/bin/bash
# r04: finish configurations on the 131k shard (option 2 = signatures per finish lane, 8 = waves per SIMD compiled
# for, 4 = tree levels), one process, interleaved (tools/ab.py), 16 keys (six contexts: 64 keys each would not fit the HBM)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=pbft_amd/libpbft_verify.so
timeout -k 10 400 python -u tools/ab.py $L $L@2=1 $L@2=1,8=2 $L@2=2,8=2 $L@2=4 $L@2=1,4=0 --replicas 16 --seqs 4096 \
  --sizes 131072,65536 --rounds 10 --iters 10 > gpurun_out/ab_fin_shard.txt 2>&1; rc=$?
cut -c1-100 gpurun_out/ab_fin_shard.txt
exit $rc

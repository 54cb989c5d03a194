#!/bin/bash
# r04: the single-wave comb compiled for 2 waves per SIMD (no 128-VGPR cap; chain and column multiplies) against the
# default build on the 131k shard and 2^16, one process, interleaved (tools/ab.py), 16 keys
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=pbft_amd/libpbft_verify.so
timeout -k 10 400 python -u tools/ab.py $L@10=0 $L build/ab/libpbft_w2.so@10=0 build/ab/libpbft_w2col.so@10=0 \
  --replicas 16 --seqs 4096 --sizes 131072,65536 --rounds 10 --iters 10 > gpurun_out/ab_occ_shard.txt 2>&1; rc=$?
cut -c1-100 gpurun_out/ab_occ_shard.txt
exit $rc

#!/bin/bash
# r04 pair-kernel A/B: comb_pair_kernel (option 10 = 1; a variant with an earlier role-1 barrier) against comb_kernel
# (option 10 = 0), one process, interleaved (tools/ab.py), 64 keys
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=pbft_amd/libpbft_verify.so
timeout -k 10 500 python -u tools/ab.py $L@10=0 $L@10=1 build/ab/libpbft_b6.so@10=1 --replicas 64 --seqs 2048 \
  --sizes ${SIZES:-32768,65536,131072,196608,262144} --rounds 8 --iters 10 > gpurun_out/ab_pair3.txt 2>&1; rc=$?
cut -c1-100 gpurun_out/ab_pair3.txt
exit $rc

#!/bin/bash
# r04: small batches -- the latency kernel (default below 12,288) against comb_pair_kernel forced for every size
# (option 1 = 0: no latency mode; option 10 = 1: pair comb) and the single-wave comb, back-to-back launches and
# single synchronized launches (p50 wall), one process, interleaved (tools/ab.py), 64 keys
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=pbft_amd/libpbft_verify.so
S=4096,8192,12288,16384,24576,32768
timeout -k 10 300 python -u tools/ab.py $L $L@1=0,10=1 $L@1=0,10=0 --replicas 64 --seqs 256 --sizes $S --rounds 8 \
  --iters 10 > gpurun_out/ab_pair_small.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab.py $L $L@1=0,10=1 --replicas 64 --seqs 256 --sizes $S --rounds 8 --latency \
  >> gpurun_out/ab_pair_small.txt 2>&1; rc=$?
cut -c1-100 gpurun_out/ab_pair_small.txt
exit $rc

#!/bin/bash
# r06 inversion rewrite: GPU parity of the new divstep lookup chain, then an interleaved A/B of the old / new
# finish (plain and stamped builds) at the 131k shard, at 2^20 and on the latency kernel.
# (build/abx/libpbft_{invold,invpin,invbat}[_st].so: tools/build_variant.sh-style builds of the three source states;
# ./build/abx is gpurun-ignored after r06 -- drop that line from .gpurunignore to run this again)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
D=gpurun_out/r06_inv; mkdir -p $D
B=build/abx
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify.py -x -v --timeout 300 --timeout-method thread > $D/verify_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab.py $B/libpbft_invold.so $B/libpbft_invpin.so $B/libpbft_invbat.so --replicas 16 --seqs 32768 --sizes 131072,1048576 --rounds 16 --iters 20 > $D/ab.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab.py $B/libpbft_invold_st.so $B/libpbft_invpin_st.so $B/libpbft_invbat_st.so --replicas 16 --seqs 32768 --sizes 131072 --rounds 6 --iters 10 > $D/ab_stamps.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab.py $B/libpbft_invold.so $B/libpbft_invbat.so --replicas 16 --seqs 32768 --sizes 4096,8192 --rounds 8 --latency > $D/ab_latency.txt 2>&1

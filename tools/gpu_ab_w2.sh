#!/bin/bash
# r03 A/B: pipelined wave inversion; finish width / tree / waves per SIMD by runtime options (ab.py lib@opt=v)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=build/ab
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 500 python tools/ab.py $B/libpbft_base.so $B/libpbft_w2.so "$B/libpbft_w2.so@2=1" "$B/libpbft_w2.so@2=2" "$B/libpbft_w2.so@2=2,8=2" "$B/libpbft_w2.so@2=4,4=6,8=2" "$B/libpbft_w2.so@2=8,4=6,8=2" --sizes 131072,262144,1048576 --rounds 10 > gpurun_out/ab_w2.log 2>&1; rc=$?
grep -E "N=|Error|error" gpurun_out/ab_w2.log; [ $rc -ne 0 ] && exit $rc
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 300 python tools/ab.py $B/libpbft_base.so $B/libpbft_w2.so --sizes 1024,4096,8192 --rounds 8 --latency > gpurun_out/ab_w2_lat.log 2>&1; rc=$?
grep -E "N=|Error|error" gpurun_out/ab_w2_lat.log; [ $rc -ne 0 ] && exit $rc
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 300 python tools/ab.py $B/libpbft_w2st.so "$B/libpbft_w2st.so@2=2" "$B/libpbft_w2st.so@2=4,4=6,8=2" --sizes 131072,1048576 --rounds 4 > gpurun_out/ab_w2_st.log 2>&1; rc=$?
grep -E "N=|stamps|Error|error" gpurun_out/ab_w2_st.log; exit $rc

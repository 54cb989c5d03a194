#!/bin/bash
# r03 A/B: divstep lookups on the SALU (readfirstlane) vs the VALU (row broadcast); throughput, latency, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=build/ab
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 300 python tools/ab.py $B/libpbft_sl.so $B/libpbft_vl.so --sizes 131072,1048576 --rounds 12 > gpurun_out/ab_vl.log 2>&1; rc=$?
grep -E "N=" gpurun_out/ab_vl.log | sed "s/\[pbft.*//"; [ $rc -ne 0 ] && exit $rc
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 300 python tools/ab.py $B/libpbft_sl.so $B/libpbft_vl.so --sizes 1024,4096,8192 --rounds 8 --latency > gpurun_out/ab_vl_lat.log 2>&1; rc=$?
grep -E "N=" gpurun_out/ab_vl_lat.log; [ $rc -ne 0 ] && exit $rc
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 200 python tools/ab.py $B/libpbft_vlst.so --sizes 131072 --rounds 4 > gpurun_out/ab_vl_st.log 2>&1; rc=$?
grep -E "stamps" gpurun_out/ab_vl_st.log; exit $rc

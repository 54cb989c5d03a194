#!/bin/bash
# r03 A/B: lane-parallel wave inversion (fe_invert_wave) vs table divsteps vs r03 base; throughput, latency, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=build/ab
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 400 python tools/ab.py $B/libpbft_base.so $B/libpbft_tab.so $B/libpbft_wave.so $B/libpbft_wave16.so $B/libpbft_wavefm2.so --sizes 131072,262144,1048576 --rounds 10 > gpurun_out/ab_wave.log 2>&1; rc=$?
grep -E "N=|Error|error" gpurun_out/ab_wave.log; [ $rc -ne 0 ] && exit $rc
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 300 python tools/ab.py $B/libpbft_base.so $B/libpbft_tab.so $B/libpbft_wave.so --sizes 1024,4096,8192 --rounds 8 --latency > gpurun_out/ab_wave_lat.log 2>&1; rc=$?
grep -E "N=|Error|error" gpurun_out/ab_wave_lat.log; [ $rc -ne 0 ] && exit $rc
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 300 python tools/ab.py $B/libpbft_wavest.so --sizes 131072,262144 --rounds 4 > gpurun_out/ab_wave_st.log 2>&1; rc=$?
grep -E "N=|stamps|Error|error" gpurun_out/ab_wave_st.log; exit $rc

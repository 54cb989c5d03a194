#!/bin/bash
# r03 A/B: table-driven divsteps in the finish tree / latency kernel (build/ab variants), throughput then latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L="build/ab/libpbft_base.so build/ab/libpbft_tab.so build/ab/libpbft_tab16.so build/ab/libpbft_tabfm2.so"
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 400 python tools/ab.py $L --sizes 131072,262144,1048576 --rounds 10 > gpurun_out/ab_tab.log 2>&1; rc=$?
grep -E "N=|Error|error" gpurun_out/ab_tab.log; [ $rc -ne 0 ] && exit $rc
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 300 python tools/ab.py build/ab/libpbft_base.so build/ab/libpbft_tab.so --sizes 1024,4096,8192 --rounds 8 --latency > gpurun_out/ab_tab_lat.log 2>&1; rc=$?
grep -E "N=|Error|error" gpurun_out/ab_tab_lat.log; exit $rc

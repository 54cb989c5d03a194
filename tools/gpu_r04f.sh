#!/bin/bash
# round 4: rekey parity, which HIP call of a votes chunk launch blocks the host (PBFT_LAUNCH_TRACE), the finish
# product tree over 16-lane rows (PBFT_FIN_LV=4) vs the wave (6): interleaved A/B, phase stamps, kernel split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py -x -v -m gpu -k "rekey or progressive" --timeout 200 --timeout-method thread > gpurun_out/pt_r04f.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04f.log | tail -5
[ $rc -ne 0 ] && exit $rc
PBFT_LAUNCH_TRACE=1 timeout -k 10 200 python -u tools/replica_probe.py 8 > gpurun_out/probe_lt.json 2> gpurun_out/probe_lt.err; rc=$?
grep -E "launch-stall" gpurun_out/probe_lt.err | head -40; cat gpurun_out/probe_lt.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab.py build/ab/libpbft_base.so@3=20000 build/ab/libpbft_lv4.so@3=20000 --sizes 131072,262144,1048576 --rounds 10 > gpurun_out/ab_lv4.txt 2>&1; rc=$?
cat gpurun_out/ab_lv4.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab.py build/ab/libpbft_st6.so@3=20000 build/ab/libpbft_st4.so@3=20000 --sizes 131072,1048576 --rounds 4 > gpurun_out/ab_st.txt 2>&1; rc=$?
cat gpurun_out/ab_st.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_shard -o shard -- python -u tools/ab.py build/ab/libpbft_base.so --sizes 131072 --rounds 6 > gpurun_out/prof_shard.log 2>&1; rc=$?
tail -3 gpurun_out/prof_shard.log; exit $rc

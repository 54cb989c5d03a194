#!/bin/bash
# round 4: copy/compute overlap probe, the -m gpu suite, replica timeline (launch-stall trace on), bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench/alloc_h2d 64 overlap > gpurun_out/overlap.txt 2>&1; rc=$?
cat gpurun_out/overlap.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_r04g.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04g.log | tail -5
[ $rc -ne 0 ] && exit $rc
PBFT_LAUNCH_TRACE=1 timeout -k 10 200 python -u tools/replica_probe.py 8 > gpurun_out/probe_r04g.json 2> gpurun_out/probe_r04g.err; rc=$?
grep -E "launch-stall" gpurun_out/probe_r04g.err | head -20; cat gpurun_out/probe_r04g.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04g.json 2> gpurun_out/bench_r04g.err; rc=$?
tail -c 300 gpurun_out/bench_r04g.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab.py pbft_amd/libpbft_verify.so@3=20000 build/ab/libpbft_latrows.so@3=20000 --latency --sizes 4096,8192 --rounds 8 > gpurun_out/ab_latrows.txt 2>&1; rc=$?
grep -v "^W2026" gpurun_out/ab_latrows.txt; exit $rc

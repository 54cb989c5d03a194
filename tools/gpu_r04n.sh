#!/bin/bash
# round 4: end-anchored chunk schedule -- parity suite, staged 2^20 pipeline, replica timeline, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_r04n.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04n.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/zc_probe.py 8 0 > gpurun_out/zc_n.json 2>/dev/null; rc=$?
cat gpurun_out/zc_n.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/replica_probe.py 8 > gpurun_out/probe_r04n.json 2> gpurun_out/probe_r04n.err; rc=$?
cat gpurun_out/probe_r04n.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04n.json 2> gpurun_out/bench_r04n.err; rc=$?
tail -c 300 gpurun_out/bench_r04n.err
exit $rc

#!/bin/bash
# round 4: zero-copy votes rows -- parity suite, interleaved A/B (tools/zc_probe.py), replica timeline, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_r04h.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04h.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/zc_probe.py 8 > gpurun_out/zc_probe.json 2> gpurun_out/zc_probe.err; rc=$?
cat gpurun_out/zc_probe.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/zc_probe.err; exit $rc; }
PBFT_LAUNCH_TRACE=1 timeout -k 10 200 python -u tools/replica_probe.py 8 > gpurun_out/probe_r04h.json 2> gpurun_out/probe_r04h.err; rc=$?
grep -E "launch-stall" gpurun_out/probe_r04h.err | head -20; cat gpurun_out/probe_r04h.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04h.json 2> gpurun_out/bench_r04h.err; rc=$?
tail -c 300 gpurun_out/bench_r04h.err
exit $rc

#!/bin/bash
# round 4: envelope table imported by a kernel -- parity suite, replica timeline (stall trace at 30 us), bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_r04o.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04o.log | tail -5
[ $rc -ne 0 ] && exit $rc
PBFT_LAUNCH_TRACE=30 timeout -k 10 200 python -u tools/replica_probe.py 8 > gpurun_out/probe_r04o.json 2> gpurun_out/probe_r04o.err; rc=$?
grep -E "launch-stall" gpurun_out/probe_r04o.err | awk '{print $2}' | sort | uniq -c | sort -rn | head; cat gpurun_out/probe_r04o.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/zc_probe.py 8 0 > gpurun_out/zc_o.json 2>/dev/null; rc=$?
cat gpurun_out/zc_o.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04o.json 2> gpurun_out/bench_r04o.err; rc=$?
tail -c 300 gpurun_out/bench_r04o.err
exit $rc

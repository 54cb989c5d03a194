#!/bin/bash
# round 4: votes chunks on two compute streams -- parity suite, staged pipeline one stream vs two (separate
# processes, env PBFT_VOTES_TWO_STREAMS), the copy/kernel trace with two, replica timeline, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_r04k.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04k.log | tail -5
[ $rc -ne 0 ] && exit $rc
for t in 0 1 0 1; do
  PBFT_VOTES_TWO_STREAMS=$t timeout -k 10 200 python -u tools/zc_probe.py 8 0 > gpurun_out/zc_t$t.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/zc_t$t.json')); print('two_streams=$t', {k: round(v['median'],4) for k, v in d.items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_votes3 -o votes -- python -u tools/zc_probe.py 3 0 > /dev/null 2>&1; rc=$?
echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
PBFT_LAUNCH_TRACE=1 timeout -k 10 200 python -u tools/replica_probe.py 8 > gpurun_out/probe_r04k.json 2> gpurun_out/probe_r04k.err; rc=$?
grep -E "launch-stall" gpurun_out/probe_r04k.err | head -20; cat gpurun_out/probe_r04k.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04k.json 2> gpurun_out/bench_r04k.err; rc=$?
tail -c 300 gpurun_out/bench_r04k.err
exit $rc

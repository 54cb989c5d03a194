#!/bin/bash
# round 4: 72-byte staged votes rows (one copy per chunk) -- parity suite, staged/pageable pipeline (with the copy
# trace), replica timeline, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_r04j.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04j.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_votes2 -o votes -- python -u tools/zc_probe.py 6 0,1 > gpurun_out/zc_probe2.json 2> gpurun_out/zc_probe2.err; rc=$?
cat gpurun_out/zc_probe2.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/zc_probe2.err; exit $rc; }
PBFT_LAUNCH_TRACE=1 timeout -k 10 200 python -u tools/replica_probe.py 8 > gpurun_out/probe_r04j.json 2> gpurun_out/probe_r04j.err; rc=$?
grep -E "launch-stall" gpurun_out/probe_r04j.err | head -20; cat gpurun_out/probe_r04j.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04j.json 2> gpurun_out/bench_r04j.err; rc=$?
tail -c 300 gpurun_out/bench_r04j.err
exit $rc

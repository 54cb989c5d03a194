#!/bin/bash
# round 3 re-entry: GPU parity suite, full bench line, then the rocprofv3 trace + PMC passes (tools/gpu_prof_r03.sh)
# each step under its own time limit, chained: the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt.log | tail -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -1 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -c 600 gpurun_out/bench.err
[ $rc -ne 0 ] && exit $rc
[ "${1:-}" = "noprof" ] && exit 0
bash tools/gpu_prof_r03.sh

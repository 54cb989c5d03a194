#!/bin/bash
# One GPU call of a round: the -m gpu parity suite, smoke(), the full bench line, then (unless "noprof") the
# rocprofv3 trace + PMC passes of the bench's launch pair (tools/gpu_prof.sh).  Each step under its own time
# limit, chained: the first failure ends the call.   usage: tools/gpu_round.sh TAG [noprof]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_$TAG.log | tail -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$?
tail -1 gpurun_out/smoke_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
tail -c 600 gpurun_out/bench_$TAG.err
[ $rc -ne 0 ] && exit $rc
[ "${2:-}" = "noprof" ] && exit 0
bash tools/gpu_prof.sh "$TAG"

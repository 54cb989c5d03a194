#!/bin/bash
# One bench line (optionally with the -m gpu suite first): usage tools/gpu_bench.sh TAG [tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
if [ "${2:-}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1; rc=$?
  grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_$TAG.log | tail -5
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
tail -c 400 gpurun_out/bench_$TAG.err
exit $rc

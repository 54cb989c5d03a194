#!/bin/bash
# round 3: GPU parity suite, then the clock-aware VALU microbenchmark (each step time-limited, chained)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|replica 2\^20|passed|failed" gpurun_out/pt.log | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 ./tools/microbench/valu_clock > gpurun_out/valu_clock.txt 2>&1; rc=$?
cat gpurun_out/valu_clock.txt
exit $rc

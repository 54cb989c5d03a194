#!/bin/bash
# GPU parity suite of the current build (round 3), each step under its own time limit
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|replica 2\^20|passed|failed" gpurun_out/pt.log | tail -40
exit $rc

#!/bin/bash
# The -m gpu suite, then the replica leg with the arena handed over vs the staging fill, alternating by round.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt_ab.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_ab.log | tail -5
[ $rc -ne 0 ] && exit $rc
SPECS="${SPECS:-PBFT_REPLICA_DIRECT=1,0}" bash tools/gpu_push_ab.sh

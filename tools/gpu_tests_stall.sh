#!/bin/bash
# GPU call: the -m gpu suite, then the config-#5 back-to-back stall probe with the library's HIP-call trace
# (PBFT_LAUNCH_TRACE=1000: calls > 1 ms), each step under its own limit, chained.   usage: tools/gpu_tests_stall.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -s --timeout 400 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_$TAG.log | tail -10
[ $rc -ne 0 ] && exit $rc
PBFT_LAUNCH_TRACE=1000 timeout -k 10 240 python -u tools/stall_probe.py 4 1.0 1 > gpurun_out/stall_$TAG.log 2>&1; rc=$?
tail -40 gpurun_out/stall_$TAG.log
exit $rc

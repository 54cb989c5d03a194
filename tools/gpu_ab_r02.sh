#!/bin/bash
# correctness of the current build on the GPU, then an in-process A/B of two builds (args: lib_a lib_b [sizes])
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log
[ $rc -ne 0 ] && exit $rc
PBFT_KEY_TABLE_BUDGET_MB=${AB_BUDGET_MB:-90000} timeout -k 10 400 python tools/ab.py "$1" "$2" --sizes "${3:-131072,1048576}" --rounds 8 > gpurun_out/ab.log 2>&1; rc=$?; grep -E "N=|Error|error" gpurun_out/ab.log; exit $rc

#!/bin/bash
# in-process A/B of variant builds (args: "lib1 lib2 ..." sizes budget_mb), each group time-limited
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PBFT_KEY_TABLE_BUDGET_MB=${3:-40000} timeout -k 10 500 python tools/ab.py $1 --sizes "${2:-131072,1048576}" --rounds 10 > gpurun_out/ab.log 2>&1; rc=$?
grep -E "N=|Error|error" gpurun_out/ab.log; exit $rc

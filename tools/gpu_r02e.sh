#!/bin/bash
# GPU parity of the current build, then in-process A/B pairs of variant libraries (args: pairs "a.so,b.so")
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log
[ $rc -ne 0 ] && exit $rc
SIZES=${SIZES:-4096,131072,262144}
i=0
for pair in "$@"; do
  i=$((i+1))
  PBFT_KEY_TABLE_BUDGET_MB=90000 timeout -k 10 300 python tools/ab.py ${pair/,/ } --sizes "$SIZES" --rounds 8 $ABARGS > gpurun_out/ab$i.log 2>&1; rc=$?
  grep -E "N=|Error|error" gpurun_out/ab$i.log | cut -c1-110
  [ $rc -ne 0 ] && exit $rc
done
exit 0

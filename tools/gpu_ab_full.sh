#!/bin/bash
# same-box A/B at the bench's key plan (default budget -> PA=13, one library per process, ABAB order)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=build/ab
: > gpurun_out/ab_full.log
for rep in 1 2; do
  for spec in ${SPECS:-$B/libpbft_base.so $B/libpbft_new.so}; do
    timeout -k 10 300 python tools/ab.py "$spec" --sizes ${1:-1048576,131072} --rounds 12 >> gpurun_out/ab_full.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_full.log; exit $rc; }
  done
done
grep -E "N=|Error|error" gpurun_out/ab_full.log | sed 's/\[pbft_verify.*//'

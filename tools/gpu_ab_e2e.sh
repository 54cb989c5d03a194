#!/bin/bash
# PCIe-inclusive A/B of the host-pipeline chunk sizes (tools/ab_e2e.py, one library per process, ABC ABC)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/ab_e2e.log
for rep in 1 2; do
  for lib in ${LIBS:-build/ab/libpbft_c18.so build/ab/libpbft_c17.so build/ab/libpbft_c16.so}; do
    PBFT_VERIFY_LIB=$lib timeout -k 10 300 python tools/ab_e2e.py >> gpurun_out/ab_e2e.log 2>> gpurun_out/ab_e2e.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/ab_e2e.err; exit $rc; }
  done
done
cat gpurun_out/ab_e2e.log

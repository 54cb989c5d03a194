#!/bin/bash
# round 4: the votes pipeline under rocprofv3 (kernels + memory copies), chunked copies only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_votes -o votes -- python -u tools/zc_probe.py 3 0 > gpurun_out/prof_votes.log 2>&1; rc=$?
grep -v "^W2026" gpurun_out/prof_votes.log | tail -12; exit $rc

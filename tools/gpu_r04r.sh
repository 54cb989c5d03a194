#!/bin/bash
# round 4: the replica round under rocprofv3 (kernels + copies of one probe run), and the -m gpu suite once more.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_replica -o rep -- python -u tools/replica_probe.py 4 > gpurun_out/prof_replica.log 2>&1; rc=$?
echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_replica.log; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt_r04r.log 2>&1; rc=$?
tail -3 gpurun_out/pt_r04r.log; exit $rc

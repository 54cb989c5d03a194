#!/bin/bash
# round 4: launch gaps, eager launches vs a HIP graph of the same launches (tools/graph_probe.py), with the trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/graph_probe.py 20 > gpurun_out/graph_probe.json 2> gpurun_out/graph_probe.err; rc=$?
cat gpurun_out/graph_probe.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/graph_probe.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_graph -o g -- python -u tools/graph_probe.py 10 > /dev/null 2>&1; rc=$?
echo "trace rc=$rc"; exit $rc

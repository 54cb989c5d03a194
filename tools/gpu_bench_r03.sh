#!/bin/bash
# round 3: the full bench line (default arguments), time-limited
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -c 3000 gpurun_out/bench.err
exit $rc

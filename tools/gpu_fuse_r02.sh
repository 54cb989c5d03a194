#!/bin/bash
# GPU parity (incl. the fused finish), then the fused-vs-separate finish probe across batch sizes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/size_probe.py --sizes 16384,65536,131072,262144,524288,1048576 --widths 0 --trees 7 --fuse 0,1099511627776 > gpurun_out/fuse.json 2>gpurun_out/fuse.err || { echo "probe failed"; tail -20 gpurun_out/fuse.err; exit 1; }
cat gpurun_out/fuse.json

#!/bin/bash
# GPU parity of the current build, then finish width x cross-lane tree sweep (kernel split by rocprofv3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin -o run -- python3 tools/size_probe.py --sizes 131072,262144,1048576 --widths 1,2,4,8,16 --trees 0,6 > gpurun_out/fin_probe.json 2>gpurun_out/fin_probe.err; rc=$?
cat gpurun_out/fin_probe.json; exit $rc

#!/bin/bash
# finish width x cross-lane tree sweep only (kernel split by rocprofv3); args: sizes widths trees
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin -o run -- python3 tools/size_probe.py --sizes ${1:-131072,262144,1048576} --widths ${2:-1,2,4,8,16} --trees ${3:-0,6} > gpurun_out/fin_probe.json 2>gpurun_out/fin_probe.err; rc=$?
cat gpurun_out/fin_probe.json; exit $rc

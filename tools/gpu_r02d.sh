#!/bin/bash
# GPU parity of the current build, in-process A/B of a variant (arg 1) vs the product library at small
# (latency-mode) sizes, then the finish width/tree probe across batch sizes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log
[ $rc -ne 0 ] && exit $rc
PBFT_KEY_TABLE_BUDGET_MB=90000 timeout -k 10 400 python tools/ab.py "$1" pbft_amd/libpbft_verify.so --sizes "${2:-2048,4096,8192,12000}" --rounds 8 > gpurun_out/ab.log 2>&1; rc=$?; grep -E "N=|Error|error" gpurun_out/ab.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/size_probe.py --sizes ${3:-16384,32768,65536,262144,524288} --widths 1,4,16 --trees 0,6 > gpurun_out/tree2.json 2>gpurun_out/tree2.err || { echo "probe failed"; tail -20 gpurun_out/tree2.err; exit 1; }
cat gpurun_out/tree2.json

#!/bin/bash
# r05 comb variants: the parity test of fuse/prio/spread, then interleaved timing A/Bs (fuse off/on) at the shard
# and round sizes, each step under its own limit.   usage: tools/gpu_fuse.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}; D=gpurun_out/fuse_$TAG; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py -x -v -m gpu -k "fuse_and_prio" --timeout 240 --timeout-method thread > $D/pt.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" $D/pt.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/opt_ab.py 15 0 1 --sizes 131072,120000,100000 --rounds 10 > $D/ab.txt 2>&1 || { tail -5 $D/ab.txt; exit 1; }
cat $D/ab.txt

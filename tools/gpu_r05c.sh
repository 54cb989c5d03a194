#!/bin/bash
# r05: comb variants (stagger) + multi-context replica: parity tests, then the stagger timing A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}; D=gpurun_out/r05c_$TAG; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_replica.py -x -v -s -m gpu -k "fuse_and_prio or 2p20_round" --timeout 300 --timeout-method thread > $D/pt.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|Error|replica 2\^20" $D/pt.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/opt_ab.py 15 0 1 --sizes 131072,120000,100000 --rounds 10 > $D/ab.txt 2>&1 || { tail -5 $D/ab.txt; exit 1; }
cat $D/ab.txt

#!/bin/bash
# PBFT_OPT_COMB_PRIO: stamped build's per-wave phases with paired priorities, then the interleaved timing A/B of the
# product library, each step under its own limit.   usage: tools/gpu_prio.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}; D=gpurun_out/prio_$TAG; mkdir -p $D
PBFT_COMB_PRIO=1 timeout -k 10 240 python -u tools/comb_stamps.py build/ab/libpbft_stamps.so 131072 1048576 > $D/stamps_prio1.txt 2>&1 || { tail -5 $D/stamps_prio1.txt; exit 1; }
grep -E "==|placement|shared by|lifetime|end us|live" $D/stamps_prio1.txt
timeout -k 10 300 python -u tools/opt_ab.py 13 0 1 --sizes 131072,196608,262144,524288,1048576 > $D/ab.txt 2>&1 || { tail -5 $D/ab.txt; exit 1; }
cat $D/ab.txt

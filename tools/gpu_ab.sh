#!/bin/bash
# In-process A/B of library variants (tools/ab.py) + VALU mix microbench.  usage: tools/gpu_ab.sh lib1 lib2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -x tools/microbench/valu_mix ] && [ -n "$MIX" ]; then timeout -k 5 60 ./tools/microbench/valu_mix > gpurun_out/valu_mix.txt || exit 1; cat gpurun_out/valu_mix.txt; fi
timeout -k 10 400 python tools/ab.py "$@" --rounds 6 --iters 10 > gpurun_out/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab.txt | tail -12; exit $rc

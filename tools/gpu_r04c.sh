#!/bin/bash
# round 4: A/B of the comb-step variants (tools/ab.py, one process, interleaved), the GPU parity suite on the
# in-tree library, the replica flush timeline probe, then the bench line.  Each step under its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python tools/ab.py build/ab/libpbft_base.so@3=20000 build/ab/libpbft_asm.so@3=20000 build/ab/libpbft_asmk.so@3=20000 build/ab/libpbft_asm_min16.so@3=20000 --rounds 6 --iters 10 --sizes 131072,1048576 > gpurun_out/ab_r04c.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab_r04c.txt | tail -10; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_r04c.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04c.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/replica_probe.py 6 > gpurun_out/probe_r04c.json 2> gpurun_out/probe_r04c.err; rc=$?
grep replica-trace gpurun_out/probe_r04c.err | tail -2; cat gpurun_out/probe_r04c.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04c.json 2> gpurun_out/bench_r04c.err; rc=$?
tail -c 300 gpurun_out/bench_r04c.err
exit $rc

#!/bin/bash
# round 4: host-cost microbenchmark (hipMalloc of large buffers, pinned H2D), parity suite, replica timeline
# probe, bench line.  Each step under its own limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 180 ./tools/microbench/alloc_h2d 64 > gpurun_out/alloc_h2d.txt 2>&1; rc=$?
cat gpurun_out/alloc_h2d.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_r04d.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04d.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/replica_probe.py 6 > gpurun_out/probe_r04d.json 2> gpurun_out/probe_r04d.err; rc=$?
grep replica-trace gpurun_out/probe_r04d.err | tail -2; cat gpurun_out/probe_r04d.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04d.json 2> gpurun_out/bench_r04d.err; rc=$?
tail -c 300 gpurun_out/bench_r04d.err
exit $rc

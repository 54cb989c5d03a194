#!/bin/bash
# GPU parity suite, then the replica flush timeline probe, then the bench line (no profiles).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -s --timeout 300 --timeout-method thread > gpurun_out/pt_r04b.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r04b.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/replica_probe.py 6 > gpurun_out/probe_r04b.json 2> gpurun_out/probe_r04b.err; rc=$?
grep replica-trace gpurun_out/probe_r04b.err | tail -3; cat gpurun_out/probe_r04b.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r04b.json 2> gpurun_out/bench_r04b.err; rc=$?
tail -c 300 gpurun_out/bench_r04b.err
exit $rc

#!/bin/bash
# progressive votes submit: its parity tests, then the replica leg of the bench (twice)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_replica.py -x -v -m gpu -s --timeout 200 --timeout-method thread > gpurun_out/prog_pt.log 2>&1; rc=$?
grep -E "replica 2\^20|FAILED|ERROR|passed|failed" gpurun_out/prog_pt.log | tail -12
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --stream-s 2 --latency-iters 50 \
    > gpurun_out/prog_$i.json 2> gpurun_out/prog_$i.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/prog_$i.json').read().strip().splitlines()[-1])
r=d['replica_flush_2^20']; print('run $i value %.1f M/s' % (d['value']/1e6), {k: r[k] for k in r if k not in ('path',)})"
done

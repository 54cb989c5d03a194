#!/bin/bash
# replica host threads A/B: bench side legs with PBFT_REPLICA_THREADS = 8, 16, 8, 16 (one process each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for t in 8 16 8 16; do
  PBFT_REPLICA_THREADS=$t timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --stream-s 2 --latency-iters 50 \
    > gpurun_out/thr_$t.json 2> gpurun_out/thr_$t.err || exit $?
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/thr_$t.json').read().strip().splitlines()[-1])
r={k:v for k,v in d.items() if 'replica' in k}; print('threads $t', json.dumps(r)[:900])"
done

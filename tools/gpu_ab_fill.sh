#!/bin/bash
# replica fill A/B: A = build/ab/libpbft_spin.so (launching thread only waits), B = the in-tree library (it fills
# its share too); bench side legs, A B A B, one process each
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in A B A B; do
  if [ $v = A ]; then export PBFT_VERIFY_LIB=$PWD/build/ab/libpbft_spin.so; else unset PBFT_VERIFY_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --stream-s 2 --latency-iters 50 \
    > gpurun_out/fill_$v.json 2> gpurun_out/fill_$v.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/fill_$v.json').read().strip().splitlines()[-1]); r=d['replica_flush_2^20']
print('$v', round(r['value']/1e6,1), 'M/s', 'ms', round(r['ms_per_round'],3), r['ms_per_round_min_max'], 'submit', round(r['flush_submit_ms'],3), 'apply', round(r['apply_ms'],3))"
done

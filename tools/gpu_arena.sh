#!/bin/bash
# Replica row arena: the replica GPU tests, then the replica leg alone with the arena handed to
# the GPU as it is (PBFT_REPLICA_DIRECT=1, default) and through the staging fill (=0), interleaved, 1 and 2 contexts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_replica.py -x -v --timeout 200 --timeout-method thread > gpurun_out/arena_tests.log 2>&1 || { tail -30 gpurun_out/arena_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/arena_tests.log | tail -3
for rep in 1 2; do
  for d in 1 0; do
    for k in 1 2; do
      PBFT_REPLICA_DIRECT=$d timeout -k 10 240 \
        python -u tools/replica_probe.py 9 $k > gpurun_out/arena_d${d}_k${k}_r${rep}.json 2> gpurun_out/arena_d${d}_k${k}_r${rep}.err || exit 1
      python - gpurun_out/arena_d${d}_k${k}_r${rep}.json $d $k <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"direct={sys.argv[2]} ctx={sys.argv[3]} round {d['ms_per_round']:.3f} push {d['push_many_ms']:.3f} flush {d['flush_ms']:.3f} submit {d['flush_submit_ms']:.3f} apply {d['apply_ms']:.3f} wait {d['gpu_wait_ms']:.3f}", flush=True)
PY
    done
  done
done

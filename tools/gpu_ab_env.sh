#!/bin/bash
# A/B of an environment switch on the replica round: tools/gpu_ab_env.sh VAR "v1 v2" [reps]
# (separate processes, alternating; tools/replica_probe.py 8 each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
VAR=$1; VALS=$2; REPS=${3:-2}
for rep in $(seq 1 $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python -u tools/replica_probe.py 8 > gpurun_out/abenv_$v.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/abenv_$v.json')); print('$VAR=$v', {k: round(d[k],3) for k in ('ms_per_round','push_many_ms','flush_ms','flush_submit_ms','apply_ms')})"
  done
done

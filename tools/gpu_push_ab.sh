#!/bin/bash
# push_many variants alternating round by round in one process (tools/replica_probe.py NAME=v1,v2): software
# prefetch distance, then the arena handed over as it is vs the staging fill.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for spec in ${SPECS:-PBFT_REPLICA_EARLY=1,0}; do
  tag=$(echo $spec | tr '=,' '__')
  timeout -k 10 300 python -u tools/replica_probe.py 24 1 $spec > gpurun_out/pab_$tag.json 2> gpurun_out/pab_$tag.err || exit 1
  python - gpurun_out/pab_$tag.json $spec <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for m, x in d["by_mode"].items():
    print(f"{sys.argv[2].split('=')[0]}={m} round {x['total_ms']:.3f} push {x['push_ms']:.3f} flush {x['flush_ms']:.3f} submit {x['submit_ms']:.3f} apply {x['apply_ms']:.3f}", flush=True)
PY
done

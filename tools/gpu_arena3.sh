#!/bin/bash
# The replica leg alone, the row arena handed over as it is (PBFT_REPLICA_DIRECT=1) and the staging fill (=0)
# alternating round by round in one process (by_mode medians), 1 and 2 contexts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 300 python -u tools/replica_probe.py 24 $k 1,0 > gpurun_out/arena3_k$k.json 2> gpurun_out/arena3_k$k.err || exit 1
  python - gpurun_out/arena3_k$k.json $k <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for m, x in d["by_mode"].items():
    print(f"ctx={sys.argv[2]} direct={m} round {x['total_ms']:.3f} push {x['push_ms']:.3f} flush {x['flush_ms']:.3f} submit {x['submit_ms']:.3f} apply {x['apply_ms']:.3f}", flush=True)
PY
done

#!/bin/bash
# The -m gpu suite, then the replica round over 2 contexts (one GPU here) with the early batch on and off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt_h.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_h.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/replica_probe.py 16 2 PBFT_REPLICA_EARLY=1,0 > gpurun_out/ctx2_ab.json 2> gpurun_out/ctx2_ab.err || exit 1
python - <<'PY'
import json
d = json.loads(open("gpurun_out/ctx2_ab.json").read().strip().splitlines()[-1])
for m, x in d["by_mode"].items():
    print(f"2 contexts early={m} round {x['total_ms']:.3f} push {x['push_ms']:.3f} flush {x['flush_ms']:.3f} submit {x['submit_ms']:.3f} apply {x['apply_ms']:.3f}")
PY

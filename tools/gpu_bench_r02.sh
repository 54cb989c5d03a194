#!/bin/bash
# The default bench line on one GPU (as the driver runs it), timed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json'))
for k in ['value','ms_per_step','p50_ms_4k_round','stream_4k','votes_device_2^20']: print(k, json.dumps(d.get(k))[:400])"

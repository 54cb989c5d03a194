#!/bin/bash
# sequential vs pipelined rounds (bench.py --pipeline), ABAB, each run time-limited
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/pipe.log
for rep in 1 2; do
  for mode in "" "--pipeline"; do
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-extras $mode > gpurun_out/pipe_one.json 2>> gpurun_out/pipe.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/pipe.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/pipe_one.json').read().strip().splitlines()[-1]); print('mode', '$mode' or 'sequential', 'value', round(d['value']/1e6,1), 'ms', round(d['ms_per_step'],4))" | tee -a gpurun_out/pipe.log
  done
done

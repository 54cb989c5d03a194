#!/bin/bash
# Config #5 latency legs under two PBFT_SPIN_WAIT modes (1: spin, yield after 2 ms; 2: never yield; 3: yield every
# 64 polls), alternating processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for m in ${MODES:-1 3}; do
  PBFT_SPIN_WAIT=$m timeout -k 10 200 python -u tools/stream_ab.py 3 > gpurun_out/stream_ab_${m}_$rep.json 2> gpurun_out/stream_ab_${m}_$rep.err || exit 1
  cat gpurun_out/stream_ab_${m}_$rep.json
done; done

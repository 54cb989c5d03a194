#!/bin/bash
# rocprofv3 kernel-trace summary + bench (separate PMC passes are in tools/gpu_pmc.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "rocprof failed"; tail -30 gpurun_out/prof.err; exit 1; }
find gpurun_out/prof -name '*stats*' | head
for f in $(find gpurun_out/prof -name '*kernel_stats.csv'); do cat "$f"; done

#!/bin/bash
# The 131k shard: kernel-timing events on/off A/B, then a rocprofv3 kernel trace of 200 launch pairs and their gaps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/gaps; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/shard_gap_probe.py ab > gpurun_out/gaps/ab.txt 2>&1 || { tail -5 gpurun_out/gaps/ab.txt; exit 1; }
cat gpurun_out/gaps/ab.txt | grep kernel
rm -rf gpurun_out/gaps/trace
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps/trace -o run -- python3 tools/shard_gap_probe.py trace > gpurun_out/gaps/trace.out 2>&1 || { tail -5 gpurun_out/gaps/trace.out; exit 1; }
f=$(find gpurun_out/gaps/trace -name "*kernel_trace.csv" | head -1)
python3 tools/gap_stats.py $f | tee gpurun_out/gaps/gaps.txt
rm -f $(find gpurun_out/gaps/trace -name "*results.db") 2>/dev/null; true

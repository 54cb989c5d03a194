#!/bin/bash
# microbench of the carry ops + kernel trace of the 131k shard (the 8-GPU node's per-GPU launch pair)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
D=gpurun_out/r05d; rm -rf $D; mkdir -p $D
timeout -k 10 120 tools/microbench/valu64 > $D/valu64.txt 2>&1 || { cat $D/valu64.txt; exit 1; }
cat $D/valu64.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --steps 50 --warmup 3 --no-cpu --no-extras --seqs 256 > $D/trace.out 2>&1 || { tail -5 $D/trace.out; exit 1; }
find $D/trace -name "*kernel_stats.csv" -exec cp {} $D/shard_kernel_stats.csv \;
find $D/trace -name "*kernel_trace.csv" -exec cp {} $D/shard_kernel_trace.csv \;
cut -c1-150 $D/shard_kernel_stats.csv | head -6
rm -rf $D/trace

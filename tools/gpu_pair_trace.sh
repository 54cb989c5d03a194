#!/bin/bash
# r04: rocprofv3 kernel trace of the bench headline at --seqs 128 (2^16 signatures, 256 keys) with the pair comb
# (default at this size) and with the single-wave comb (PBFT_COMB_PAIR=0); kernel_stats per mode
set -o pipefail
cd "$GRAFT_REPO_ROOT"; D=gpurun_out/pair_trace; rm -rf $D; mkdir -p $D; export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 3 --no-cpu --no-extras --seqs 128"
for m in 1 0; do
  export PBFT_COMB_PAIR=$m
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/t$m -o run -- $B > $D/t$m.out 2>&1 || exit 1
  find $D/t$m -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats_pair$m.csv \;
  grep -h '"value"' $D/t$m.out | cut -c1-200
done
rm -rf $D/t?

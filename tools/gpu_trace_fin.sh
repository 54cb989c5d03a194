#!/bin/bash
# per-kernel durations (rocprofv3 --kernel-trace --stats) of finish configurations, one config per traced run
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tf; export TMPDIR=/tmp
B=build/ab
i=0
for spec in "$B/libpbft_w2.so" "$B/libpbft_w2.so@2=8,4=6,8=2" "$B/libpbft_w2.so@2=4,4=6,8=2" "$B/libpbft_w2.so@2=16,4=6,8=1"; do
  i=$((i+1))
  PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tf/t$i -o run -- python3 tools/ab.py "$spec" --sizes ${1:-1048576} --rounds 4 > gpurun_out/tf/t$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/tf/t$i.log; exit $rc; }
  echo "== $spec"; grep -E "N=" gpurun_out/tf/t$i.log | sed 's/\[pbft.*//'
  f=$(find gpurun_out/tf/t$i -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | grep -E "comb_kernel|finish" | sed 's/(.*)"/"/'
done
find gpurun_out/tf -name "*.db" -delete; true

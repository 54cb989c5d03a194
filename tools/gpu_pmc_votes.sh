#!/bin/bash
# VALU instructions per signature of the votes-form comb (envelope schedule shared): one --pmc pass over a
# 2^20-signature votes-form round launched by tools/ab.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; D=gpurun_out/pmc_votes; rm -rf $D; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $D/p1 -o run -- python3 tools/ab.py pbft_amd/libpbft_verify.so --votes --sizes 1048576 --rounds 1 --iters 2 > $D/p1.out 2>&1
rc=$?; echo "pmc votes rc=$rc"; tail -2 $D/p1.out
[ $rc -ne 0 ] && exit $rc
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/pmc_votes/p1/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, m in agg.items():
    if "comb_kernel" in k or "finish" in k or "env_sched" in k:
        v = max(m["SQ_INSTS_VALU"]); w = max(m["SQ_WAVES"])
        print(f"{k[:60]:60s} SQ_INSTS_VALU {v:.4g} SQ_WAVES {w:.0f} -> VALU/sig (2^20) {v * 64 / 2**20:.0f}")
PY

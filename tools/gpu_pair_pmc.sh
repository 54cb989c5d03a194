#!/bin/bash
# r04: the 131k shard (bench --seqs 256) with comb_kernel (PBFT_COMB_PAIR=0) and comb_pair_kernel (=1): kernel trace,
# then one PMC pass each of VALU / wave / instruction-cache counters (--pmc only, each pass its own time limit)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; D=gpurun_out/pair_pmc; rm -rf $D; mkdir -p $D; export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras --seqs 256"
for m in 0 1; do
  export PBFT_COMB_PAIR=$m
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/t$m -o run -- $B > $D/t$m.out 2>&1 || exit 1
  find $D/t$m -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats_$m.csv \;
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $D/p$m -o run -- $B > $D/p$m.out 2>&1 || { tail -3 $D/p$m.out; exit 1; }
  find $D/p$m -name "*counter_collection.csv" -exec cp {} $D/pmc_$m.csv \;
  timeout -s KILL 120 rocprofv3 --pmc VALUBusy --output-format csv -d $D/q$m -o run -- $B > $D/q$m.out 2>&1 || { tail -3 $D/q$m.out; exit 1; }
  find $D/q$m -name "*counter_collection.csv" -exec cp {} $D/busy_$m.csv \;
done
rm -rf $D/t? $D/p? $D/q?
python3 - <<'PY'
import csv, collections
D="gpurun_out/pair_pmc"
for m in (0,1):
    for f in (f"{D}/kernel_stats_{m}.csv",):
        for r in csv.DictReader(open(f)):
            print(m, r["Name"][:40], r["Calls"], r["AverageNs"])
    for f in (f"{D}/pmc_{m}.csv", f"{D}/busy_{m}.csv"):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "comb" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(m, {k: round(sum(v) / len(v), 1) for k, v in acc.items()})
PY

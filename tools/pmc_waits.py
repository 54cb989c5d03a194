#!/usr/bin/env python3
"""Wait-state breakdown of comb_kernel / finish_kernel from one rocprofv3 --pmc pass of SQ counters (per size).
SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked: s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stall: dependency / pipe)
+ SQ_ACTIVE_INST_ANY (issuing), all in quad-cycles (MI355X_MICROARCH.md, rocprofv3 PMC slots).
usage: tools/pmc_waits.py counters.csv [...]"""
import collections
import csv
import sys

for path in sys.argv[1:]:
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "")
        k = "comb" if "comb_kernel" in name or "comb_pair" in name else "finish" if "finish_kernel" in name else None
        if k:
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {path}")
    for k, m in vals.items():
        a = {c: sum(v) / len(v) for c, v in m.items()}
        wc = a.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"  {k}: wave-cycles {wc:.3e} (quad-cycles, summed over waves)")
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU"):
            if c in a:
                print(f"    {c:22s} {a[c]:.3e}  {100 * a[c] / wc:5.1f} % of wave-cycles")
        if "SQ_BUSY_CYCLES" in a:
            print(f"    SQ_BUSY_CYCLES         {a['SQ_BUSY_CYCLES']:.3e}")
        if "SQ_INSTS_VALU" in a:
            print(f"    SQ_INSTS_VALU          {a['SQ_INSTS_VALU']:.3e}")

#!/usr/bin/env python3
"""profiles/<run>/derived.json from rocprofv3 --pmc pass CSVs of the verify launch pair (read by bench.py).

usage: python tools/pmc_derive.py PMC_DIR PB PA [n_sigs [KERNEL_STATS_CSV]]   (comb positions of the plans)

With the rocprofv3 --kernel-trace --stats CSV of the same command, each kernel also gets its average duration and
the shader clock it ran at: GRBM_GUI_ACTIVE (GPU-busy cycles of the dispatch) / the average duration.
"""
import collections
import csv
import glob
import json
import os
import sys

d, pb, pa = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
n = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 20
stats = {}
if len(sys.argv) > 5:
    for r in csv.DictReader(open(sys.argv[5])):
        stats[r["Name"]] = float(r["AverageNs"])


def avg_ns(name):
    hits = [v for k, v in stats.items() if name in k and "entry" not in k and "base" not in k]
    return max(hits) if hits else None


def agg(name):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "*.csv")):
        for r in csv.DictReader(open(f)):
            if name in r.get("Kernel_Name", ""):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


out = {"launch": f"comb_kernel<85> PB={pb} PA={pa} + finish_kernel, one {n}-signature launch", "sigs_per_launch": n}
tot = 0.0
for k in ("comb_kernel", "finish_kernel"):
    m = agg(k)
    fb, wbytes = 2 * m["FETCH_SIZE"] * 1024, m["WRITE_SIZE"] * 1024
    out[k] = {"fetch_bytes": fb, "write_bytes": wbytes, "valu_busy_pct": m.get("VALUBusy"),
              "valu_lane_utilisation_pct": m.get("VALUUtilization"),
              "valu_insts_per_lane": m["SQ_INSTS_VALU"] / m["SQ_WAVES"], "waves": m["SQ_WAVES"],
              # wave-instructions x 64 lanes / signatures: the VALU instructions one signature costs
              "valu_insts_per_sig": m["SQ_INSTS_VALU"] * 64 / n}
    ns = avg_ns(k)
    if ns and "GRBM_GUI_ACTIVE" in m:
        out[k]["avg_ns"] = ns
        out[k]["grbm_gui_active"] = m["GRBM_GUI_ACTIVE"]
        # rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back).  The quotient
        # "reads high on dispatches shorter than about 0.3 ms" (same section): the 131k shard's kernels gave 2.46 and
        # 3.20 GHz, above the 2.4-GHz engine clock.  So below 0.3 ms no clock is derived
        # from it; the in-kernel clock (s_memtime / s_memrealtime stamps, PMC_CLOCK_GHZ=<GHz>) is used when given.
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        clk = cyc / ns
        kclk = float(os.environ["PMC_CLOCK_GHZ"]) if os.environ.get("PMC_CLOCK_GHZ") else None
        if ns >= 300_000 and clk <= 2.4:
            out[k]["clock_ghz"] = clk
            out[k]["clock_source"] = "GRBM_GUI_ACTIVE / 8 / avg duration"
        elif kclk:
            out[k]["clock_ghz"] = kclk
            out[k]["clock_source"] = "in-kernel s_memtime / s_memrealtime (PMC_CLOCK_GHZ)"
            out[k]["grbm_clock_ghz_invalid"] = clk
        else:
            out[k]["clock_ghz"] = None
            out[k]["clock_source"] = (f"none: GRBM_GUI_ACTIVE / 8 / avg duration = {clk:.2f} GHz is not valid for a "
                                      f"{ns / 1e3:.0f}-us dispatch (< 300 us, MI355X_MICROARCH.md DVFS give-back)")
        if out[k]["clock_ghz"]:
            c = out[k]["clock_ghz"] * ns  # cycles of the dispatch at that clock
            # VALU wave-instructions per SIMD per cycle (1024 SIMDs) at that clock
            out[k]["valu_issue_per_simd_cycle"] = m["SQ_INSTS_VALU"] / 1024 / c
    tot += fb + wbytes
out["traffic_bytes_per_launch"] = tot
out["valu_insts_per_sig_total"] = sum(out[k]["valu_insts_per_sig"] for k in ("comb_kernel", "finish_kernel"))
out["note"] = ("rocprofv3 --pmc passes (one counter group per run, no tracing) of `python3 bench.py --steps 5 "
               "--warmup 1 --no-cpu --no-extras` (tools/gpu_prof.sh); FETCH_SIZE (KB) doubled per the "
               "gfx950 correction of MI355X_MICROARCH.md's HBM section; WRITE_SIZE taken as is")
json.dump(out, open(os.path.join(d, "derived.json"), "w"), indent=1)
print(json.dumps(out, indent=1))

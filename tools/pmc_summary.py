#!/usr/bin/env python3
"""Derive VALU issue / occupancy / traffic numbers for verify_kernel from rocprofv3 --pmc CSVs.

usage: python tools/pmc_summary.py profiles/r01_pmc [n_sigs_per_dispatch] [kernel_avg_ms]
"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
ms = float(sys.argv[3]) if len(sys.argv) > 3 else None
KERNEL = os.environ.get("KERNEL", "comb_kernel")
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.csv"))):
    for r in csv.DictReader(open(f)):
        if KERNEL in r.get("Kernel_Name", ""):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
out = []
for k in sorted(m):
    out.append(f"{k:28s} {m[k]:.6g} per dispatch")
simds = 1024
if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
    out.append(f"VALU instructions per signature (= per lane) : {m['SQ_INSTS_VALU'] / m['SQ_WAVES']:.0f}")
if "GRBM_GUI_ACTIVE" in m:
    cyc = m["GRBM_GUI_ACTIVE"] / 8  # summed over 8 XCDs
    out.append(f"GPU busy cycles per dispatch (per XCD)        : {cyc:.4g}")
    if ms:
        out.append(f"effective clock                               : {cyc / (ms * 1e-3) / 1e9:.3f} GHz")
    if "SQ_INSTS_VALU" in m:
        ipc = m["SQ_INSTS_VALU"] / (simds * cyc)
        out.append(f"VALU wave-instructions / cycle / SIMD          : {ipc:.3f}  (VOP3 issue limit measured ~0.25)")
if "SQ_THREAD_CYCLES_VALU" in m and "SQ_ACTIVE_INST_VALU" in m:
    out.append(f"VALU lane utilisation (active lanes / 64)      : "
               f"{m['SQ_THREAD_CYCLES_VALU'] / (64 * m['SQ_ACTIVE_INST_VALU']):.3f}")
if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
    out.append(f"wave cycles waiting (s_waitcnt / barrier)       : {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
if "FETCH_SIZE" in m:
    out.append(f"FETCH_SIZE x2 (gfx950 correction) per signature : {2 * m['FETCH_SIZE'] * 1024 / n:.0f} B")
if "WRITE_SIZE" in m:
    out.append(f"WRITE_SIZE per dispatch                         : {m['WRITE_SIZE'] * 1024:.0f} B (bitmap = {n // 8} B)")
if "TCC_HIT_sum" in m:
    out.append(f"L2 hit rate                                     : {m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}")
print("\n".join(out))

#!/usr/bin/env python3
"""Print the GPU timeline (kernels + copies, from rocprofv3 --kernel-trace --memory-copy-trace CSVs) of the last
replica round in a trace: tools/timeline.py DIR [--rounds-back K] [--gap-ms 2]
Rounds are split at idle gaps longer than --gap-ms; times in us from the round's first event."""
import argparse
import csv
import glob
import os


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            short = n.split("(")[0].replace("void ", "")
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K s%s" % r["Stream_Id"], short[:48], ""))
    for f in glob.glob(os.path.join(d, "*memory_copy_trace.csv")):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C s%s" % r["Stream_Id"],
                       r["Direction"].replace("MEMORY_COPY_", ""), r.get("Size", "")))
    ev.sort()
    return ev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--rounds-back", type=int, default=1)
    ap.add_argument("--gap-ms", type=float, default=2.0)
    a = ap.parse_args()
    ev = load(a.dir)
    groups, cur, last_end = [], [], None
    for e in ev:
        if last_end is not None and e[0] - last_end > a.gap_ms * 1e6:
            groups.append(cur)
            cur = []
        cur.append(e)
        last_end = max(last_end or 0, e[1])
    groups.append(cur)
    g = groups[-a.rounds_back]
    t0 = g[0][0]
    busy_k = sum(e[1] - e[0] for e in g if e[2].startswith("K"))
    busy_c = sum(e[1] - e[0] for e in g if e[2].startswith("C"))
    print("# %d events, span %.1f us, kernel time %.1f us, copy time %.1f us" %
          (len(g), (max(e[1] for e in g) - t0) / 1e3, busy_k / 1e3, busy_c / 1e3))
    for s, e, kind, name, size in g:
        print("%9.1f %9.1f %8.1f  %-5s %s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, kind, name, size))


if __name__ == "__main__":
    main()

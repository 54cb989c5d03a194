#!/usr/bin/env python3
"""Gaps between consecutive kernel dispatches in a rocprofv3 kernel_trace.csv: for each kernel name, its mean
duration; for each (previous kernel -> next kernel) pair, the mean idle time between the end of one and the start
of the next.   usage: python tools/gap_stats.py kernel_trace.csv"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    short = lambda name: name.split("(")[0].replace("void ", "")[:60]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = short(r["Kernel_Name"])
        dur[name].append(e - s)
        if prev is not None:
            gap[(prev[0], name)].append(s - prev[1])
        prev = (name, e)
    for k, x in dur.items():
        x = sorted(x)
        print(f"{k:60s} n={len(x):5d} mean {sum(x) / len(x) / 1e3:8.2f} us  median {x[len(x) // 2] / 1e3:8.2f} us")
    for (a, b), x in gap.items():
        x = sorted(x)
        print(f"gap {a[:28]:28s} -> {b[:28]:28s} n={len(x):5d} median {x[len(x) // 2] / 1e3:7.2f} us  "
              f"mean {sum(x) / len(x) / 1e3:7.2f} us")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Symbolize the sampling profiles the ingress driver writes with PBFT_INGRESS_PROFILE=file (tools/ingress/
ingress_driver.cpp, Sampler): per timed loop, the share of samples per function (llvm-symbolizer over the module
offsets).  usage: python tools/ingress_profile.py FILE [--top 25]"""
import argparse
import collections
import subprocess

SYM = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def symbolize(module, offsets):
    if module == "?" or not offsets:
        return {o: "?" for o in offsets}
    inp = "".join("0x%x\n" % o for o in offsets)
    out = subprocess.run([SYM, "--obj=" + module, "--functions=linkage", "--demangle", "--no-inlines"],
                         input=inp, capture_output=True, text=True, timeout=120).stdout
    # output: for every address, "function\nfile:line:col\n\n"
    blocks = [b.split("\n") for b in out.strip("\n").split("\n\n")]
    names = [b[0] if b else "?" for b in blocks]
    return {o: (names[i] if i < len(names) else "?") for i, o in enumerate(offsets)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    sections, cur = [], None
    for line in open(a.file):
        if line.startswith("#"):
            cur = {"title": line[1:].strip(), "rows": []}
            sections.append(cur)
            continue
        c, mod, off = line.split()
        cur["rows"].append((int(c), mod, int(off, 16)))
    for sec in sections:
        by_mod = collections.defaultdict(list)
        for c, mod, off in sec["rows"]:
            by_mod[mod].append(off)
        names = {}
        for mod, offs in by_mod.items():
            for o, n in symbolize(mod, sorted(set(offs))).items():
                names[(mod, o)] = n
        fn = collections.Counter()
        total = 0
        for c, mod, off in sec["rows"]:
            short = mod.rsplit("/", 1)[-1]
            fn[(names.get((mod, off), "?")[:90], short)] += c
            total += c
        print("## " + sec["title"])
        for (name, mod), c in fn.most_common(a.top):
            print("%6.2f %%  %-90s %s" % (100.0 * c / max(1, total), name, mod))
        print()


if __name__ == "__main__":
    main()

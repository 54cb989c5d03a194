"""Per-loop VALU instruction histogram of one kernel in a gfx950 .s file (hipcc -S --cuda-device-only).

usage: python tools/asm_hist.py file.s kernel_substring
Finds the kernel body, every loop (a label targeted by a later branch), and prints the opcode histogram of
the largest loop body (the comb step) plus whole-kernel totals, by class (mad, 64-bit, VOP2/3 32-bit, LDS,
memory, scalar).
"""
import collections
import re
import sys


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:", l) and sub in l.split(":")[0] and not l.startswith("_ZZ"):
            start = i
            break
    if start is None:
        raise SystemExit("kernel not found")
    end = start + 1
    while end < len(lines) and not lines[end].startswith(".Lfunc_end"):
        end += 1
    return lines[start:end]


def ops(body):
    out = []
    for l in body:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        out.append(s.split()[0])
    return out


def klass(op):
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mad_i64_i32"):
        return "mad64"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu/ctl"
    if op.startswith("v_"):
        if "64" in op or op.startswith(("v_addc", "v_subb", "v_lshl_add_u64")):
            return "valu64"
        return "valu32"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, sub)
    labels = {}
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
        if m:
            t = m.group(1) or m.group(2)
            if t in labels:
                loops.append((labels[t], i))
    all_ops = ops(body)
    print(f"kernel: {len(all_ops)} instructions, "
          f"{sum(1 for o in all_ops if o.startswith('v_'))} VALU")
    if loops:
        lo, hi = max(loops, key=lambda x: x[1] - x[0])
        lops = ops(body[lo:hi + 1])
        c = collections.Counter(lops)
        k = collections.Counter(klass(o) for o in lops)
        nv = sum(v for o, v in c.items() if o.startswith("v_"))
        print(f"largest loop: lines {lo}-{hi}: {len(lops)} instructions, {nv} VALU")
        for kk, v in k.most_common():
            print(f"  class {kk:10s} {v}")
        for o, v in c.most_common(60):
            print(f"  {o:28s} {v}")
        nvalu = lambda a, b: sum(1 for o in ops(body[a:b]) if o.startswith("v_"))
        print(f"VALU before the largest loop: {nvalu(0, lo)}, after it: {nvalu(hi + 1, len(body))}")
        print("all loops (start line, end line, VALU in body):")
        for a, b in sorted(set(loops)):
            print(f"  {a:6d} {b:6d} {nvalu(a, b + 1):6d}")


if __name__ == "__main__":
    main()

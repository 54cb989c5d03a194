"""Interval analysis for the radix-2^25.5 field code in pbft_amd/csrc/fe25519.h.

Checks that no 64-bit column accumulator of fe_mul/fe_sq can overflow and that
every u32 limb stays below 2^32, for the exact add/sub/mul sequence used by the
mixed addition (comb step) and doubling.  Run: python tools/limb_bounds.py
"""
import math
E26, E25 = 1 << 26, 1 << 25
CARRIED = [E26 if i % 2 == 0 else E25 for i in range(10)]
CARRIED[1] += 1 << 14; CARRIED[5] += 1 << 14   # carry-chain overshoot allowance
CARRIED[0] = E26
P2 = [0x7FFFFDA] + [0x3FFFFFE if i % 2 else 0x7FFFFFE for i in range(1, 10)]
P4 = [2 * x for x in P2]

def add(a, b): return [x + y for x, y in zip(a, b)]
def sub(a, b, off):
    for x, o in zip(b, off): assert x <= o, "sub underflow"
    return [x + o for x, o in zip(a, off)]
def mulmax(f, g):
    worst, cols = 0, []
    for k in range(10):
        s = 0
        for i in range(10):
            for j in range(10):
                if (i + j) % 10 != k: continue
                c = 2 if (i % 2 and j % 2) else 1
                if i + j >= 10: c *= 19
                s += c * f[i] * g[j]
        worst = max(worst, s)
        cols.append(s)
    for x in f + g: assert x < 2**32
    for i, x in enumerate(g): assert 19 * x < 2**32, "19*g overflows u32"
    for i, x in enumerate(f):
        if i % 2: assert 2 * x < 2**32
    if f is g:  # fe_sq precomputes 38*f_odd and 19*f_even
        for i, x in enumerate(f): assert (38 if i % 2 else 19) * x < 2**32, "fe_sq premult overflow"
    assert worst < 2**64, math.log2(worst)
    chain1(cols)
    return math.log2(worst)


def chain1(cols):
    """fe_reduce_wide with PBFT_REDUCE_1CHAIN (0 -> 1 -> ... -> 9 -> 0 x19 -> 1) on columns <= cols: the
    result must stay within CARRIED (h1 is the only limb above its width) and no step may overflow u64."""
    h = list(cols)
    for i in range(10):
        w = 26 if i % 2 == 0 else 25
        c = h[i] >> w
        h[i] = (1 << w) - 1
        if i < 9:
            h[i + 1] += c
        else:
            h[0] += 19 * c
        assert max(h) < 2**64
    c = h[0] >> 26
    h[0] = (1 << 26) - 1
    h[1] += c
    for x, b in zip(h, CARRIED):
        assert x <= b, "chain1 overshoot"

C = CARRIED
# mixed add (comb step): P3 + halved affine Niels ((y+x)/2, (y-x)/2, dxy) with canonical table limbs
ymx = sub(C, C, P2); ypx = add(C, C)
print("madd a=(Y-X)*ymx   log2 max col:", mulmax(ymx, C))
print("madd b=(Y+X)*ypx   log2 max col:", mulmax(ypx, C))
d = C   # D = Z1: halved table entries (ge25519.h), no doubling of Z1
e = sub(C, C, P2); f = sub(d, C, P2); g = add(d, C); h = add(C, C)
# operand order as coded in ge25519.h: the second operand is the one premultiplied by 19
for neg in (False, True):
    F, G = (g, f) if neg else (f, g)   # negative digit swaps d-c and d+c
    for nm, (x, y) in {"X3=F*E": (F, e), "Y3=G*H": (G, h), "Z3=dmc*dpc": (f, g), "T3=E*H": (e, h)}.items():
        print("madd neg=%d" % neg, nm, " log2 max col:", mulmax(x, y))
# madd v2 (PBFT_MADD_V2, verify_core.h): k' = +-k (2p - k for a negative digit), F = D - c, G = D + c never
# swap; X3 = F*E, T3 = H*E, Y3 = H*G, Z3 = F*G (second operand premultiplied by 19)
for neg in (False, True):
    kk = P2 if neg else C            # 2p - k <= 2p limb-wise (k canonical)
    print("madd v2 neg=%d c=T*k'" % neg, " log2 max col:", mulmax(C, kk))
e = sub(C, C, P2); F = sub(d, C, P2); G = add(d, C); h = add(C, C)
for nm, (x, y) in {"X3=F*E": (F, e), "T3=H*E": (h, e), "Y3=H*G": (h, G), "Z3=F*G": (F, G)}.items():
    print("madd v2", nm, " log2 max col:", mulmax(x, y))
# doubling (dbl-2008-hwcd, a=-1): A=X^2, B=Y^2, C2=2Z^2, H=A+B, E=H-(X+Y)^2, G=A-B, F=C2+G
xy = add(C, C)
print("dbl (X+Y)^2         log2 max col:", mulmax(xy, xy))
print("sq of carried       log2 max col:", mulmax(C, C))
# precomputation-only doubling: E, F, G, H are carried before the products
H = C; E = C; G = C; F = C
for nm, (x, y) in {"X=E*F": (E, F), "Y=G*H": (G, H), "T=E*H": (E, H), "Z=F*G": (F, G)}.items():
    print("dbl", nm, " log2 max col:", mulmax(x, y))
print("all bounds OK")

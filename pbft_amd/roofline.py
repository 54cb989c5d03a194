"""Roofline constants for the verify kernel.

The verify path is bound by integer VALU work, not HBM and not MFMA: per
signature it reads ~161 B (R 32, S 32, key index 2, message 85, table lines
from L2/MALL) but issues ~6e4 32x32->64 multiply-accumulates.

PRODUCTS_PER_VERIFY counts the v_mad_u64_u32 products the implemented
algorithm needs per signature (16-bit comb windows on both scalars, WB = WA = 16;
Montgomery batch inversion over FIN_M = 16 signatures per lane):
  comb       (16 + 16) mixed additions x 7 field muls x 100 products = 22,400
  inversion  (254 squarings x 55 + 11 muls x 100) / 16               =    942
  batch      3 muls per signature (prefix, 1/Z_m, running inverse) +
             2 affine muls (x, y), x 100                              =    500
  Barrett    9x9 + 44 word products (k mod L)                         =    125
                                                               total = 23,967
(SHA-512, carries, additions and selects are additional VALU work, not
counted as products; the VALU-issue view is in profiles/*/summary.txt.)

VALU_MAD_PEAK_PER_S is the measured chip-wide v_mad_u64_u32 issue rate on
MI355X (tools/microbench/valu_rates.hip, profiles/r01_valu_rates.txt).
"""
WB = 16
WA = 16
FIN_M = 16
_P = lambda w: (254 + w - 1) // w  # noqa: E731
COMB_MADDS = _P(WB) + _P(WA)
PRODUCTS_PER_VERIFY = COMB_MADDS * 7 * 100 + (254 * 55 + 11 * 100) // FIN_M + 5 * 100 + (81 + 44)
VALU_MAD_PEAK_PER_S = 30.25e12
VALU_OP_PEAK_PER_S = 37.2e12  # 32-bit VOP3 integer ops (v_add3_u32 / v_alignbit_b32), measured

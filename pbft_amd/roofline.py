"""Roofline constants for the verify kernels.

The verify path is bound by integer VALU work (and, before the line-coalesced
gather, by random 128-B table gathers), not by streaming HBM and not by MFMA:
per signature it reads 161 B of batch input and gathers (PB + PA) table lines
of 128 B, but issues ~2e4 32x32->64 multiply-accumulates.

products_per_verify(PB, PA) counts the v_mad_u64_u32 products the implemented
algorithm needs per signature (comb plans with PB positions for [s]B and PA for
[k](-A), i.e. PB + PA steps; Montgomery batch inversion over FIN_M signatures
per lane):
  comb       (PB + PA - 1) mixed additions x 7 field muls x 100 products
             + 1 mul for the first step, built directly from its table entry
             (10 + 14 positions with the default balanced plans)
  inversion  one divsteps inversion (20 x 90 products) / FIN_M
  batch      3 muls per signature (prefix, 1/Z_m, running inverse) +
             2 affine muls (x, y), x 100
  Barrett    9x9 + 44 word products (k mod L)
(SHA-512, carries, additions and selects are additional VALU work, not counted
as products; the VALU-issue view is in profiles/*/summary*.txt.)

VALU_MAD_PEAK_PER_S is the measured chip-wide v_mad_u64_u32 issue rate on
MI355X at the clock the chip holds under that load (tools/microbench/valu_clock.hip,
profiles/r03/valu_clock.txt: 8 independent chains per lane, 8 waves per SIMD, >= 2 s
of back-to-back launches first; the clock is stamped in-kernel as
d(s_memtime) / d(s_memrealtime) x 100 MHz).  It issues one wave-instruction per
4.53 cycles per SIMD at 2.157 GHz: 1024 SIMDs x 64 lanes / 4.53 x 2.157e9 = 31.2e12.
(r01's 30.25e12 came from the same loop without a clock stamp; its "@2.4GHz"
columns assumed the spec clock.  v_fma_f32 runs 2.29 cycles per wave-instruction
with three distinct source VGPRs -- the guide's 2 -- but 3.79 with src1 == src2,
the form r01 timed: that, not the VALU, was the gap to MI355X_MICROARCH.md's rate.)
"""
import re

FIN_M = 8            # finish signatures per lane at >= 2^19 signatures (pbft_verify.hip PBFT_FIN_FM_BIG)
FIN_TREE_LEVELS = 4  # finish.hip PBFT_FIN_LV: the product tree spans a 16-lane row (r04; 6 = the wave before)
VALU_MAD_PEAK_PER_S = 31.19e12   # measured, profiles/r03/valu_clock.txt
MAD_CYCLES_PER_WAVE_INSTR = 4.53  # per SIMD, at the measured clock
MAD_CLOCK_HZ = 2.157e9            # in-kernel clock during that measurement
SIMDS = 256 * 4


def mad_peak_at(clock_hz: float) -> float:
    """v_mad_u64_u32 products/s the chip can issue at clock_hz (1024 SIMDs x 64 lanes / 4.53 cycles)."""
    return SIMDS * 64 / MAD_CYCLES_PER_WAVE_INSTR * clock_hz


VALU_OP_PEAK_PER_S = 37.2e12  # 32-bit VOP3 integer ops (v_add3_u32 / v_alignbit_b32), measured
ENTRY_BYTES = 128
INPUT_BYTES = 32 + 32 + 2 + 85  # R, S, key index, envelope


# wave-uniform inversion (inv25519.h fe_invert_wave): per batch of 30 divsteps the lane-parallel f, g update (4 x 9
# lane products) and D, E update (4 x 10), ~18 batches, then one field multiply by 2^-30k
INV_PRODUCTS = 18 * (4 * 9 + 4 * 10) + 100


def products_comb(pb: int, pa: int) -> int:
    """comb_kernel alone: (PB + PA - 1) mixed additions x 7 muls + 1 mul (first step) + Barrett k mod L."""
    return ((pb + pa - 1) * 7 + 1) * 100 + (81 + 44)


def products_per_verify(pb: int, pa: int) -> int:
    """comb_kernel + finish_kernel<8, 4, 2>: 3 batch-inversion muls and 2 affine muls per signature, the product
    tree's 2 x FIN_TREE_LEVELS muls per lane over FIN_M signatures, one row-uniform inversion per
    2^FIN_TREE_LEVELS x FIN_M signatures."""
    return (products_comb(pb, pa) + 5 * 100 + 2 * FIN_TREE_LEVELS * 100 // FIN_M
            + INV_PRODUCTS // ((1 << FIN_TREE_LEVELS) * FIN_M))


def gather_bytes_per_verify(pb: int, pa: int) -> int:
    return (pb + pa) * ENTRY_BYTES


def positions_from_build_info(info: str):
    """(PB, widest PA) from pbft_build_info(), e.g. 'pbft_verify gfx950 PB=10 PA=13|14|16|32 ...'."""
    m = re.search(r"PB=(\d+) PA=(\d+)", info)
    if not m:
        raise ValueError(f"unexpected build info: {info!r}")
    return int(m.group(1)), int(m.group(2))


# defaults of the shipped build (base point 10 positions, keys 13 for n = 256 on a 288-GB MI355X)
PB = 10
PA = 13
PRODUCTS_PER_VERIFY = products_per_verify(PB, PA)

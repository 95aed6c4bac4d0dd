"""Algorithmic work of the sieve, for roofline accounting.

marks(range) = sum over odd primes p <= sqrt(max value) of the number of odd
multiples of p in [max(p^2, lo), hi]; an LDS-resident sieve pays one 4-byte
LDS read + one 4-byte write per mark (8 B/mark), and writes
the mask (nbits/8 bytes) to HBM once.
"""
from __future__ import annotations

import math

import numpy as np

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md): 256 CUs at 2.4 GHz,
# LDS 128 B/clk/CU for 4-byte-per-lane access (ds_read_b32 row of the LDS
# table; "~75 TB/s for ds_read_b32" aggregate), HBM3E 8 TB/s spec.
NUM_CUS = 256
CLOCK_HZ = 2.4e9
LDS_PEAK_GBS = NUM_CUS * 128 * CLOCK_HZ / 1e9      # 78,643 GB/s (SURVEY 8(d)'s figure)
HBM_PEAK_GBS = 8000.0
BYTES_PER_MARK = 8
# An executed mark is one lane of a ds_or_b32 (4 B read-modify-write). Its
# peak is the LDS store path: ds_write_b32 moves 64 B/clk/CU (4 cycles per
# wave-instruction, MI355X_MICROARCH.md section LDS), 39,322 GB/s chip-wide.
LDS_OR_BYTES_PER_MARK = 4
LDS_OR_PEAK_GBS = NUM_CUS * 64 * CLOCK_HZ / 1e9    # 39,322 GB/s
# The measured conflict-free ds_or_b32 rate: 2.6 CU-cycles per wave-instruction
# (profiles/r02/lds_conflict_microbench.txt), i.e. 256 B / 2.6 clk / CU,
# 60,494 GB/s chip-wide -- the peak the mark instruction itself reaches.
DS_OR_CYCLES_PER_WAVE_INSTR = 2.6
LDS_DS_OR_PEAK_GBS = NUM_CUS * 256 / DS_OR_CYCLES_PER_WAVE_INSTR * CLOCK_HZ / 1e9
# VALU ceiling: a wave64 VALU instruction issues over 2 cycles on each of the
# 4 SIMD-32 of a CU (MI355X_MICROARCH.md "Wave scheduling"): 2.0 per CU-cycle.
VALU_PEAK_PER_CU_CYCLE = 2.0


def odd_primes_upto(x: int) -> np.ndarray:
    if x < 3:
        return np.zeros(0, dtype=np.int64)
    s = np.ones(x // 2 + 1, dtype=bool)  # s[i] <-> 2i+1
    s[0] = False
    for i in range(1, (math.isqrt(x) - 1) // 2 + 1):
        if s[i]:
            p = 2 * i + 1
            s[p * p // 2::p] = False
    return (2 * np.flatnonzero(s) + 1).astype(np.int64)


def marks_for_range(g_start: int, nbits: int) -> int:
    """Odd multiples >= p^2 of every odd prime p <= sqrt(vmax) that fall in
    the odd-index range [g_start, g_start+nbits) (values 3+2g)."""
    if nbits <= 0:
        return 0
    va = 3 + 2 * g_start
    vb = 3 + 2 * (g_start + nbits - 1)
    ps = odd_primes_upto(math.isqrt(vb))
    if ps.size == 0:
        return 0
    lo = np.maximum(ps * ps, va)
    m0 = (lo + ps - 1) // ps
    m0 += (m0 % 2 == 0)
    m1 = vb // ps
    m1 -= (m1 % 2 == 0)
    cnt = np.where(m1 >= m0, (m1 - m0) // 2 + 1, 0)
    return int(cnt.sum())


R30 = (1, 7, 11, 13, 17, 19, 23, 29)
WHEEL_OUT_BITS = 15 * 2**17  # odd candidates per wheel-kernel segment (csrc/dse_internal.h kWheelOutBits)
WHEEL_PATTERN_MAX = 79  # the wheel kernel's init lays down the patterns of 7..79 (no LDS marks; csrc kQMax)
WHEEL_PATTERN_GROUPS = 9  # in 9 groups of 1-3 primes (csrc kNG)


def _coprime30_upto(x: np.ndarray) -> np.ndarray:
    """#{1 <= m <= x : gcd(m, 30) = 1} (x >= 0)."""
    q, r = np.divmod(x, 30)
    return 8 * q + np.searchsorted(np.array(R30), r, side="right")


def wheel_marks_for_range(g_start: int, nbits: int) -> int:
    """LDS marks the mod-30 wheel kernel issues for the odd-index range:
    multiples p*m >= p^2 with gcd(m, 30) = 1 of every prime 79 < p <= sqrt(vmax)
    (multiples of 3 and 5 are not stored, primes 7..79 are init patterns)."""
    if nbits <= 0:
        return 0
    va = 3 + 2 * g_start
    vb = 3 + 2 * (g_start + nbits - 1)
    ps = odd_primes_upto(math.isqrt(vb))
    ps = ps[ps > WHEEL_PATTERN_MAX]
    if ps.size == 0:
        return 0
    lo = np.maximum(ps * ps, va)
    m0 = (lo + ps - 1) // ps
    m1 = vb // ps
    cnt = np.where(m1 >= m0, _coprime30_upto(m1) - _coprime30_upto(m0 - 1), 0)
    return int(cnt.sum())


BUCKET_LO = 2**19  # ranges with bucketed primes bucket every prime above this (csrc kBucketLoLog)


def bucket_entries_for_range(g_start: int, nbits: int, lo_p: int = BUCKET_LO) -> int:
    """Bucket entries the bucketed pass writes (and the wheel kernel reads
    back) for the odd-index range: one per multiple p*m in the range with
    gcd(m, 30) = 1 and p*m >= p^2 of every prime lo_p < p <= sqrt(vmax)
    (csrc/dse_wheel.hip bucket_fill_stage_kernel; the range must reach past
    2^20, or the wheel kernel takes all its primes itself). Needs the primes up
    to sqrt(vmax): ~0.5 GB and ~10 s of numpy for the 1e18 window
    (tools/window_entries.py keeps that one as WINDOW_BUCKET_ENTRIES)."""
    if nbits <= 0:
        return 0
    va = 3 + 2 * g_start
    vb = 3 + 2 * (g_start + nbits - 1)
    ps = odd_primes_upto(math.isqrt(vb))
    ps = ps[ps > lo_p]
    if ps.size == 0:
        return 0
    lo = np.maximum(ps * ps, va)
    m0 = (lo + ps - 1) // ps
    m1 = vb // ps
    cnt = np.where(m1 >= m0, _coprime30_upto(m1) - _coprime30_upto(m0 - 1), 0)
    return int(cnt.sum())


# bucket_entries_for_range of bench.py --window's range (odd values 1e18 + 1 ..
# 1e18 + 1e10 - 1; tools/window_entries.py): 8 B each is written and read back
WINDOW_BUCKET_ENTRIES = 1_208_549_165
BUCKET_ENTRY_BYTES = 4


def roofline(g_start: int, nbits: int, seconds: float, launches: int = 1) -> dict:
    """t_roof = max(8*marks/BW_LDS, (nbits/8)/BW_HBM), marks =
    the algorithmic odd-only count. The wheel kernel issues fewer LDS marks
    (wheel_marks): frac_executed prices those instead."""
    marks = marks_for_range(g_start, nbits)
    wmarks = wheel_marks_for_range(g_start, nbits)
    lds_bytes = BYTES_PER_MARK * marks
    hbm_bytes = (nbits + 7) // 8
    t = seconds / launches
    t_lds = lds_bytes / (LDS_PEAK_GBS * 1e9)
    t_hbm = hbm_bytes / (HBM_PEAK_GBS * 1e9)
    return {
        "marks": marks,
        "lds_bytes": lds_bytes,
        "hbm_bytes": hbm_bytes,
        "t_roof_s": max(t_lds, t_hbm),
        "bound": "lds" if t_lds >= t_hbm else "hbm",
        "lds_achieved_gbs": lds_bytes / t / 1e9,
        "hbm_achieved_gbs": hbm_bytes / t / 1e9,
        "frac": max(t_lds, t_hbm) / t,
        "wheel_marks": wmarks,
        "frac_executed": max(BYTES_PER_MARK * wmarks / (LDS_PEAK_GBS * 1e9), t_hbm) / t,
    }

"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper around oracle/liboracle.so.

CPU restatement of /root/reference/src/mail_sieve_e/sieve.clj (see
dse_oracle.c for the line-by-line citations). Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product path
(libdse.so and the mail_sieve_e package) never does.

Parity status: unpinned by the reference itself (it ships no fixtures and
cannot run in this image); pinned by published pi(10^k), sympy sweeps and the
SURVEY.md section 4 known-answer table (tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i64, i32, u64 = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64
        p64, pu64 = ctypes.POINTER(i64), ctypes.POINTER(u64)
        L.ref_spread_work.argtypes = [i64, i32, p64, p64]
        L.ref_sieve.argtypes = [i64, i32, pu64, pu64, p64, pu64]
        L.ref_sieve_flags.argtypes = [i64, i32, ctypes.c_void_p, pu64]
        L.ref_finish.argtypes = [ctypes.c_char_p, i32, i64, i32, pu64]
        L.fast_sieve_range.argtypes = [u64, u64, pu64, pu64]
        L.ref_sieve_threaded.argtypes = [i64, i32, pu64, pu64, p64, pu64]
        L.fast_count_window.argtypes = [u64, u64, pu64]
        for f in (L.ref_spread_work, L.ref_sieve, L.ref_sieve_flags, L.ref_finish, L.fast_sieve_range,
                  L.ref_sieve_threaded, L.fast_count_window):
            f.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(arr, ctype):
    return arr.ctypes.data_as(ctypes.POINTER(ctype)) if arr is not None else None


def spread_work(n: int, P: int):
    """sieve.clj:15-34 -> (cs, [(lo, hi), ...]) in exact integers."""
    lo_hi = np.zeros(2 * P, dtype=np.int64)
    cs = ctypes.c_int64()
    rc = lib().ref_spread_work(n, P, _p(lo_hi, ctypes.c_int64), ctypes.byref(cs))
    if rc:
        raise ValueError(f"ref_spread_work rc={rc}")
    return cs.value, [(int(lo_hi[2 * k]), int(lo_hi[2 * k + 1])) for k in range(P)]


def words_for(cs: int) -> int:
    return (cs + 63) // 64


def sieve(n: int, P: int):
    """Faithful restatement of the whole lead/follower run.

    Returns (cs, masks[P, words] uint64, counts[P] uint64, n_prime_messages).
    """
    cs, _ = spread_work(n, P)
    if cs < 1:
        raise ValueError("empty chunk")
    w = words_for(cs)
    masks = np.zeros((P, w), dtype=np.uint64)
    counts = np.zeros(P, dtype=np.uint64)
    csv = ctypes.c_int64()
    msgs = ctypes.c_uint64()
    rc = lib().ref_sieve(n, P, _p(masks, ctypes.c_uint64), _p(counts, ctypes.c_uint64),
                         ctypes.byref(csv), ctypes.byref(msgs))
    if rc:
        raise RuntimeError(f"ref_sieve rc={rc}")
    return cs, masks, counts, msgs.value


def sieve_threaded(n: int, P: int, want_masks: bool = True):
    """The lead/follower run as P machine threads + machine 1's relay thread,
    exchanging [mi ps p] messages through in-process queues (the reference's
    run on one host). Same results as sieve().

    Returns (cs, masks[P, words] or None, counts[P], n_prime_messages)."""
    cs, _ = spread_work(n, P)
    if cs < 1:
        raise ValueError("empty chunk")
    masks = np.zeros((P, words_for(cs)), dtype=np.uint64) if want_masks else None
    counts = np.zeros(P, dtype=np.uint64)
    csv, msgs = ctypes.c_int64(), ctypes.c_uint64()
    rc = lib().ref_sieve_threaded(n, P, _p(masks, ctypes.c_uint64), _p(counts, ctypes.c_uint64),
                                  ctypes.byref(csv), ctypes.byref(msgs))
    if rc:
        raise RuntimeError(f"ref_sieve_threaded rc={rc}")
    return cs, masks, counts, msgs.value


def count_window(lo: int, hi: int) -> int:
    """Independent OpenMP count of the primes among the odd values in [lo, hi]."""
    cnt = ctypes.c_uint64()
    rc = lib().fast_count_window(lo, hi, ctypes.byref(cnt))
    if rc:
        raise RuntimeError(f"fast_count_window rc={rc}")
    return cnt.value


def pi_ref(counts) -> int:
    """1 (the injected 2, sieve.clj:88-96) + odd primes inside the chunks."""
    return 1 + int(np.sum(np.asarray(counts, dtype=np.uint64)))


def finish(path: str, my_num: int, n: int, P: int, mask) -> None:
    """sieve.clj:82-108: write primes{my_num}.txt byte-exactly."""
    mask = np.ascontiguousarray(mask, dtype=np.uint64)
    rc = lib().ref_finish(path.encode(), my_num, n, P, _p(mask, ctypes.c_uint64))
    if rc:
        raise RuntimeError(f"ref_finish rc={rc}")


def fast_sieve_range(g0: int, nbits: int, want_mask: bool = True):
    """Independent OpenMP segmented sieve of odd indices [g0, g0+nbits)."""
    mask = np.zeros(words_for(nbits), dtype=np.uint64) if want_mask else None
    cnt = ctypes.c_uint64()
    rc = lib().fast_sieve_range(g0, nbits, _p(mask, ctypes.c_uint64), ctypes.byref(cnt))
    if rc:
        raise RuntimeError(f"fast_sieve_range rc={rc}")
    return mask, cnt.value


def tail_range(n: int, P: int):
    """Odd indices [P*cs, nums) that spread-work drops (sieve.clj:21-34)."""
    nums = (n - 1) // 2 if n >= 1 else 0
    cs = nums // P
    return P * cs, nums - P * cs

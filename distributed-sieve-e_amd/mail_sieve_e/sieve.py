"""Mirror of mail-sieve-e.sieve (/root/reference/src/mail_sieve_e/sieve.clj).

Same names and argument meaning as the reference's public functions; the
chunk vector with zeroed composites becomes a bit-packed odd-only mask
produced by libdse.so's gfx950 kernels:

  gen-table    (sieve.clj:9-13)   -> gen_table: a Chunk descriptor [lower, upper)
  spread-work  (sieve.clj:15-34)  -> spread_work: exact integer bounds
  sieve-e      (sieve.clj:118-172)-> sieve_e: segmented sieve of the chunk on a GPU
  finish       (sieve.clj:82-108) -> finish: byte-exact ~/primes{k}.txt

indices / mark-composites / find-next-non-zero / find-first-prime
(sieve.clj:36-80,110-116) are the reference's inner loop; they have no
counterpart here because the kernel replaces them (DESIGN.md "Path").
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _dse
from ._dse import check, lib, u64p


class Context:
    """A libdse context: one process driving ``num_gpus`` devices, or one
    device (``device=``) for one-process-per-GPU ranks. ``logical=k`` (tests
    only, include/dse.h dse_debug_init_logical): k logical devices on device 0,
    the multi-device code path with the collectives replaced by copies."""

    def __init__(self, num_gpus: int = 1, device: Optional[int] = None, logical: Optional[int] = None):
        L = lib()
        if logical is not None:
            self._ptr = L.dse_debug_init_logical(logical)
        else:
            self._ptr = L.dse_init_device(device) if device is not None else L.dse_init(num_gpus)
        if not self._ptr:
            raise _dse.DseError(L.dse_last_status(), "dse_init", L.dse_last_error().decode(errors="replace"))

    @property
    def ptr(self):
        if not self._ptr:
            raise RuntimeError("context closed")
        return self._ptr

    @property
    def num_devices(self) -> int:
        return lib().dse_ctx_num_devices(self.ptr)

    def close(self) -> None:
        if self._ptr:
            lib().dse_destroy(self._ptr)
            self._ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host-buffer entry points ------------------------------------------
    def sieve_odd_range(self, g_start: int, nbits: int, want_mask: bool = True):
        mask = np.zeros((nbits + 63) // 64, dtype=np.uint64) if want_mask else None
        cnt = ctypes.c_uint64()
        check(lib().dse_sieve_odd_range(self.ptr, g_start, nbits, u64p(mask), ctypes.byref(cnt)),
              "dse_sieve_odd_range")
        return mask, cnt.value

    def sieve_chunk(self, n: int, P: int, my_num: int, want_mask: bool = True):
        cs, _ = _spread(n, P)
        mask = np.zeros((cs + 63) // 64, dtype=np.uint64) if want_mask else None
        cnt = ctypes.c_uint64()
        check(lib().dse_sieve_chunk(self.ptr, n, P, my_num, u64p(mask), ctypes.byref(cnt)),
              "dse_sieve_chunk")
        return mask, cnt.value

    def sieve_all(self, n: int, P: int):
        """-> (per-chunk counts, pi_ref, pi_full); masks stay on the devices."""
        counts = np.zeros(P, dtype=np.uint64)
        pr, pf = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().dse_sieve_all(self.ptr, n, P, u64p(counts), ctypes.byref(pr), ctypes.byref(pf)),
              "dse_sieve_all")
        return counts, pr.value, pf.value

    def copy_chunk_mask(self, n: int, P: int, my_num: int) -> np.ndarray:
        cs, _ = _spread(n, P)
        mask = np.zeros((cs + 63) // 64, dtype=np.uint64)
        check(lib().dse_copy_chunk_mask(self.ptr, my_num, u64p(mask)), "dse_copy_chunk_mask")
        return mask

    def sieve_window(self, lo: int, hi: int) -> int:
        cnt = ctypes.c_uint64()
        check(lib().dse_sieve_window(self.ptr, lo, hi, ctypes.byref(cnt)), "dse_sieve_window")
        return cnt.value

    def device_status(self) -> None:
        """Raise DseError (DSE_EINTERNAL) if a device pass of this context broke
        an invariant since the last check (the *_dev_async calls report here)."""
        check(lib().dse_device_status(self.ptr), "dse_device_status")

    def debug_set_option(self, name: str, value: int) -> None:
        """Test-only knob of this context (include/dse.h dse_debug_set_option)."""
        check(lib().dse_debug_set_option(self.ptr, name.encode(), int(value)), "dse_debug_set_option")

    def debug_get_stat(self, name: str) -> int:
        """Test-only statistic of this context (include/dse.h dse_debug_get_stat)."""
        v = ctypes.c_int64(0)
        check(lib().dse_debug_get_stat(self.ptr, name.encode(), ctypes.byref(v)), "dse_debug_get_stat")
        return v.value

    # -- device-buffer entry points (torch tensors' data_ptr()) --------------
    def base_primes_dev_async(self, limit: int, table_ptr: int, table_bytes: int, stream_ptr: int = 0):
        check(lib().dse_base_primes_dev_async(self.ptr, limit, table_ptr, table_bytes, stream_ptr or None),
              "dse_base_primes_dev_async")

    def base_table_finish_dev_async(self, limit: int, table_ptr: int, table_bytes: int, stream_ptr: int = 0):
        """Barrett factors + wheel offsets for a table whose primes arrived by broadcast."""
        check(lib().dse_base_table_finish_dev_async(self.ptr, limit, table_ptr, table_bytes, stream_ptr or None),
              "dse_base_table_finish_dev_async")

    def sieve_range_dev_async(self, table_ptr: int, g_start: int, nbits: int, mask_ptr: int,
                              count_ptr: int, stream_ptr: int = 0):
        check(lib().dse_sieve_range_dev_async(self.ptr, table_ptr, g_start, nbits, mask_ptr or None,
                                              count_ptr, stream_ptr or None),
              "dse_sieve_range_dev_async")


def base_table_bytes(limit: int) -> int:
    return int(lib().dse_base_table_bytes(limit))


def base_table_prime_bytes(limit: int) -> int:
    """Leading bytes of a base table that hold the primes: what ranks broadcast."""
    return int(lib().dse_base_table_prime_bytes(limit))


def base_table_broadcast_bytes(limit: int) -> int:
    """Bytes rank 0 broadcasts for a table of odd primes <= limit, or 0 when
    every rank builds its own table (include/dse.h dse_base_table_broadcast_bytes:
    the primes move while they fit in 8 MiB; the 1e18 window's 203 MB are
    rebuilt on every device, which is faster than moving them)."""
    return int(lib().dse_base_table_broadcast_bytes(limit))


def base_limit_for_range(g_start: int, nbits: int) -> int:
    return int(lib().dse_base_limit_for_range(g_start, nbits))


_default_ctx: Optional[Context] = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(num_gpus=1)
    return _default_ctx


def _spread(n: int, P: int):
    lo_hi = np.zeros(2 * P, dtype=np.int64)
    cs = ctypes.c_int64()
    check(lib().dse_spread_work(n, P, lo_hi.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                ctypes.byref(cs)), "dse_spread_work")
    return cs.value, [[int(lo_hi[2 * k]), int(lo_hi[2 * k + 1])] for k in range(P)]


def spread_work(n: int, num_comps: int) -> List[List[int]]:
    """sieve.clj:15-34: P equal chunks [lo, hi) of the odd numbers from 3,
    cs = floor(floor((n-1)/2)/P); the remainder is dropped. Exact integers
    (the reference computes Doubles, identical below 2^53)."""
    return _spread(n, num_comps)[1]


def tail_range(n: int, P: int):
    """Odd indices [g, g+len) that spread-work drops (len <= P-1)."""
    g, nb = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().dse_tail_range(n, P, ctypes.byref(g), ctypes.byref(nb)), "dse_tail_range")
    return g.value, nb.value


@dataclass
class Chunk:
    """gen-table's result (sieve.clj:9-13): the odd numbers in [lower, upper).

    ``mask`` (after sieve_e) holds bit j = 1 iff element j (value lower+2j)
    is still non-zero, i.e. prime."""

    lower: int
    upper: int
    mask: Optional[np.ndarray] = None
    n_primes: Optional[int] = None

    @property
    def cs(self) -> int:  # (count chunk), sieve.clj:128
        return len(range(self.lower, self.upper, 2))

    @property
    def g_start(self) -> int:
        return (self.lower - 3) // 2

    def primes(self) -> np.ndarray:
        """Non-zero elements of the chunk in order (before finish's hack)."""
        if self.mask is None:
            raise ValueError("chunk not sieved")
        bits = np.unpackbits(self.mask.view(np.uint8), bitorder="little")[: self.cs]
        return (self.lower + 2 * np.flatnonzero(bits)).astype(np.int64)


def gen_table(bounds: Sequence[int]) -> Chunk:
    """sieve.clj:9-13: [lower upper] -> the chunk of odd values in [lower, upper)."""
    lower, upper = int(bounds[0]), int(bounds[1])
    if lower < 3 or lower % 2 == 0:
        raise ValueError("chunks start at an odd number >= 3 (spread-work bounds)")
    return Chunk(lower, upper)


def finish(raw_chunk: Chunk, my_num: int, *, path: Optional[str] = None) -> str:
    """sieve.clj:82-108: write the chunk's primes to user.home/primes{my_num}.txt
    (chunk 1 as Doubles with the 2/3/5/7 hack), 10 per line, ", "-joined."""
    if raw_chunk.mask is None:
        raise ValueError("chunk not sieved")
    if path is None:
        path = os.path.join(os.path.expanduser("~"), f"primes{my_num}.txt")
    mask = np.ascontiguousarray(raw_chunk.mask, dtype=np.uint64)
    check(lib().dse_write_range_file(path.encode(), my_num, raw_chunk.g_start, raw_chunk.cs, u64p(mask)),
          "dse_write_range_file")
    return path


def sieve_e(my_num: int, lead: bool, in_channel, chunk: Chunk, out_channel, *,
            ctx: Optional[Context] = None, write_file: bool = True, path: Optional[str] = None) -> Chunk:
    """sieve.clj:118-172: sieve this machine's chunk, then finish it.

    The reference marks the chunk prime by prime, receiving earlier chunks'
    primes on ``in_channel`` and reporting its own on ``out_channel``. Here the
    chunk is sieved in one pass on a GPU with the base primes <= sqrt(upper)
    computed on the device, so the channels carry nothing; they are accepted
    for call compatibility. ``lead`` likewise no longer orders the work."""
    del lead, in_channel, out_channel
    ctx = ctx or default_context()
    if chunk.cs < 1:
        raise ValueError("empty chunk (find-first-prime would throw)")
    chunk.mask, chunk.n_primes = ctx.sieve_odd_range(chunk.g_start, chunk.cs, want_mask=True)
    if write_file:
        finish(chunk, my_num, path=path)
    return chunk

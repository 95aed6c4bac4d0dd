"""ctypes binding of libdse.so (include/dse.h).

The shared library sits next to this file (built in-tree by
``make -C distributed-sieve-e_amd/csrc``). Loading fails loudly when it is
missing: there is no CPU fallback in the product path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdse.so")
CSRC = os.path.normpath(os.path.join(_HERE, "..", "csrc"))

DSE_OK = 0
ERRORS = {
    -1: "DSE_EINVAL",
    -2: "DSE_EHIP",
    -3: "DSE_ENCCL",
    -4: "DSE_ENOMEM",
    -5: "DSE_EIO",
    -6: "DSE_ERANGE",
    -7: "DSE_EINTERNAL",
}

# name -> (restype, argtypes); every symbol include/dse.h declares.
_i32, _i64, _u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
_vp, _cp = ctypes.c_void_p, ctypes.c_char_p
_pi64, _pu64 = ctypes.POINTER(_i64), ctypes.POINTER(_u64)
SIGNATURES = {
    "dse_version": (_cp, []),
    "dse_last_error": (_cp, []),
    "dse_last_status": (_i32, []),
    "dse_device_count": (_i32, []),
    "dse_init": (_vp, [_i32]),
    "dse_init_device": (_vp, [_i32]),
    "dse_destroy": (None, [_vp]),
    "dse_ctx_num_devices": (_i32, [_vp]),
    "dse_spread_work": (_i32, [_i64, _i32, _pi64, _pi64]),
    "dse_tail_range": (_i32, [_i64, _i32, _pu64, _pu64]),
    "dse_sieve_chunk": (_i32, [_vp, _i64, _i32, _i32, _pu64, _pu64]),
    "dse_sieve_odd_range": (_i32, [_vp, _u64, _u64, _pu64, _pu64]),
    "dse_sieve_all": (_i32, [_vp, _i64, _i32, _pu64, _pu64, _pu64]),
    "dse_copy_chunk_mask": (_i32, [_vp, _i32, _pu64]),
    "dse_sieve_window": (_i32, [_vp, _u64, _u64, _pu64]),
    "dse_write_primes_file": (_i32, [_cp, _i32, _i64, _i32, _pu64]),
    "dse_write_range_file": (_i32, [_cp, _i32, _u64, _u64, _pu64]),
    "dse_base_table_bytes": (_u64, [_u64]),
    "dse_base_limit_max": (_u64, []),
    "dse_base_limit_for_range": (_u64, [_u64, _u64]),
    "dse_base_primes_dev_async": (_i32, [_vp, _u64, _vp, _u64, _vp]),
    "dse_base_table_prime_bytes": (_u64, [_u64]),
    "dse_base_table_broadcast_bytes": (_u64, [_u64]),
    "dse_base_table_finish_dev_async": (_i32, [_vp, _u64, _vp, _u64, _vp]),
    "dse_sieve_range_dev_async": (_i32, [_vp, _vp, _u64, _u64, _vp, _vp, _vp]),
    "dse_device_status": (_i32, [_vp]),
    "dse_debug_set_option": (_i32, [_vp, _cp, _i64]),
    "dse_debug_init_logical": (_vp, [_i32]),
    "dse_debug_get_stat": (_i32, [_vp, _cp, _pi64]),
}

_lib = None


class DseError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Load libdse.so; raise if it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libdse.so not built at {LIB_PATH}; run `make -C {CSRC}` "
                "(the HIP extension is required, there is no CPU fallback)")
        # torch (the device-memory/stream plumbing) ships its own copy of
        # libamdhip64.so.7; load it first so libdse binds to that same HIP
        # runtime instead of /opt/rocm's (two runtimes in one process cannot
        # both open the GPU, and torch's stream handles must be understood).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if name.startswith("dse_debug_") and not hasattr(L, name):
                continue  # test-only entry point absent from an older A/B build (tools/ab_libs.py)
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int, where: str) -> None:
    if rc != DSE_OK:
        raise DseError(rc, where, lib().dse_last_error().decode(errors="replace"))


def u64p(arr):
    """numpy uint64 array -> POINTER(c_uint64) (None passes through)."""
    if arr is None:
        return None
    return arr.ctypes.data_as(_pu64)

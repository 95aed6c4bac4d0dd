"""The multi-device code path of dse_sieve_all / dse_sieve_window on one GPU.

dse_debug_init_logical(k) (include/dse.h) builds a context of k logical
devices that all run on device 0, each with its own stream, table, counts,
resident masks and scratch; only the two RCCL collectives are
replaced (the prime broadcast by device-to-device copies of device 0's table,
the count all-reduce by a gather + sum on device 0 and a copy back, each
ordered with events where the RCCL calls sit). So the chunk map of
sieve.clj:24-34 over devices (chunk k on device (k-1) mod k_dev), the table
completion on the non-root devices (dse_base_table_finish: Barrett factors and
wheel offsets derived locally), the tail on the last device, several chunks
of a device pooled into one persistent launch, window slices and the
per-device flag checks all
run here against the golden fixtures -- what dse_init(8) runs on an 8-GPU
node, collectives aside.
"""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def sha(a):
    return hashlib.sha256(memoryview(np.ascontiguousarray(a)).cast("B")).hexdigest()


@pytest.fixture(scope="module")
def S():
    from mail_sieve_e import sieve
    return sieve


@pytest.mark.parametrize("P,ndev", [(2, 2), (4, 4), (8, 8), (8, 3), (4, 8)])
def test_1e10_golden_on_logical_devices(S, P, ndev):
    """BASELINE config 3 (N=1e10 over 2/4/8 GPUs): one chunk per device as on
    a P-GPU node, and the uneven maps (8 chunks on 3 devices: several chunks
    pooled into one persistent launch per device; 4 chunks on 8 devices: idle
    devices)."""
    g = GOLDEN["big"][f"1e10_P{P}"]
    with S.Context(logical=ndev) as c:
        assert c.num_devices == ndev
        counts, pi_ref, pi_full = c.sieve_all(10**10, P)
        assert [int(x) for x in counts] == g["counts"]
        assert pi_ref == pi_full == 455_052_511
        for k in range(P):
            assert sha(c.copy_chunk_mask(10**10, P, k + 1)) == g["mask_sha256"][k], (P, ndev, k + 1)
        # a second call reuses the resident masks and tables (and the counts are re-zeroed)
        counts2, pi_ref2, _ = c.sieve_all(10**10, P)
        assert pi_ref2 == pi_ref and [int(x) for x in counts2] == g["counts"]


def test_1e11_p8_golden_on_8_logical_devices(S):
    """The headline N=1e11 as the 8-GPU run maps it: chunk k on device k-1."""
    g = GOLDEN["big"]["1e11_P8"]
    with S.Context(logical=8) as c:
        counts, pi_ref, pi_full = c.sieve_all(10**11, 8)
        assert pi_ref == pi_full == 4_118_054_813
        assert [int(x) for x in counts] == g["counts"]
        for k in range(1, 9):
            assert sha(c.copy_chunk_mask(10**11, 8, k)) == g["mask_sha256"][k - 1], k


def test_1e12_p8_on_8_logical_devices(S):
    """north_star's pi(1e12) = 37607912018 on 8 devices (BASELINE config 4):
    the reference's chunks give 37607912017, the tail (on the last device)
    adds 999999999989."""
    g = GOLDEN["big"].get("1e12_P8")
    with S.Context(logical=8) as c:
        counts, pi_ref, pi_full = c.sieve_all(10**12, 8)
        assert pi_ref == 37_607_912_017
        assert pi_full == 37_607_912_018
        assert g is not None
        assert [int(x) for x in counts] == g["counts"]
        # chunk 8 (values 8.75e11 .. 1e12, on the last device) is the 8-GPU
        # critical path: every large prime live in every segment
        assert sha(c.copy_chunk_mask(10**12, 8, 8)) == g["mask_sha256"][7]


def test_window_on_logical_devices(S, oracle):
    """BASELINE config 5's code path: table built once (two-level) on device
    0, copied to the others, one contiguous slice per device, each with its
    own bucketed passes and scratch, counts summed."""
    lo, hi = 10**18, 10**18 + 10**7
    c1 = oracle.count_window(lo, hi)
    for nd in (2, 5, 8):
        with S.Context(logical=nd) as c:
            assert c.sieve_window(lo, hi) == c1, nd


@pytest.mark.parametrize("share", ["local", "broadcast"])
def test_window_full_on_8_logical_devices(S, share):
    """[1e18, 1e18+1e10] over 8 devices: 241,272,176 (oracle fast_count_window).
    The table's 50.8 M primes (203 MB) exceed the broadcast cap, so by default
    every device builds its own table (table_local_builds); with the cap
    raised the primes take the broadcast path (copies from device 0 here)."""
    with S.Context(logical=8) as c:
        if share == "broadcast":
            c.debug_set_option("table_broadcast_max_bytes", 1 << 40)
        assert c.sieve_window(10**18, 10**18 + 10**10) == GOLDEN["big"]["window_1e18"]["count"] == 241_272_176
        assert c.debug_get_stat("table_local_builds") == (8 if share == "local" else 0)
        # chunk configs keep the broadcast (the reference's prime broadcast)
        assert c.sieve_all(10**10, 8)[2] == 455_052_511
        assert c.debug_get_stat("table_local_builds") == (8 if share == "local" else 0)


def test_logical_rejects_bad_count(S):
    from mail_sieve_e import _dse
    for k in (0, -1, 65):
        with pytest.raises(_dse.DseError) as e:
            S.Context(logical=k)
        assert e.value.code == -1

"""The RCCL branch of dse_sieve_all / dse_sieve_window executed on one GPU.

dse_debug_set_option(ctx, "rccl_single", 1) gives a one-device context a
1-rank communicator from ncclCommInitAll, the call dse_init(8) makes for 8
GPUs; share_table and allreduce_counts then issue the grouped ncclBroadcast of
the base primes (device 0's table as send and receive buffer, the reference's
prime broadcast, sieve.clj:139, core.clj:94-95,126) and the grouped
ncclAllReduce of the counts on the device's stream, instead of returning early
for one device. Results are checked against the golden fixtures, and the
context's statistics show that RCCL accepted every collective.
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


def test_sieve_all_1e10_p2_through_rccl(S):
    g = GOLDEN["big"]["1e10_P2"]
    with S.Context() as c:
        assert c.debug_get_stat("rccl_comms") == 0 and c.debug_get_stat("rccl_ranks") == 0
        c.debug_set_option("rccl_single", 1)
        assert c.debug_get_stat("rccl_comms") == 1 and c.debug_get_stat("rccl_ranks") == 1
        counts, pi_ref, pi_full = c.sieve_all(10**10, 2)
        # one ncclBroadcast + one ncclAllReduce, both accepted by RCCL
        assert c.debug_get_stat("rccl_calls") == 2
        assert [int(x) for x in counts] == g["counts"]
        assert pi_ref == pi_full == 455_052_511
        for k in range(2):
            assert sha(c.copy_chunk_mask(10**10, 2, k + 1)) == g["mask_sha256"][k], k + 1
        # a second call through the same communicator
        counts2, _, _ = c.sieve_all(10**10, 2)
        assert [int(x) for x in counts2] == g["counts"] and c.debug_get_stat("rccl_calls") == 4


def test_sieve_all_1e12_p8_through_rccl(S):
    """north_star's pi(1e12) with the broadcast and all-reduce through RCCL."""
    g = GOLDEN["big"].get("1e12_P8")
    with S.Context() as c:
        c.debug_set_option("rccl_single", 1)
        counts, pi_ref, pi_full = c.sieve_all(10**12, 8)
        assert (pi_ref, pi_full) == (37_607_912_017, 37_607_912_018)
        if g is not None:
            assert [int(x) for x in counts] == g["counts"]
        assert c.debug_get_stat("rccl_calls") == 2


@pytest.mark.parametrize("share", ["local", "broadcast"])
def test_window_full_through_rccl(S, share):
    """[1e18, 1e18+1e10], the count by ncclAllReduce: 241,272,176 (oracle
    fast_count_window). The 50.8 M base primes (203 MB) are past the
    broadcast cap, so by default every device builds its own table and the
    only collective is the all-reduce; with the cap raised they go through
    ncclBroadcast as well."""
    with S.Context() as c:
        c.debug_set_option("rccl_single", 1)
        if share == "broadcast":
            c.debug_set_option("table_broadcast_max_bytes", 1 << 40)
        assert c.sieve_window(10**18, 10**18 + 10**10) == GOLDEN["big"]["window_1e18"]["count"] == 241_272_176
        assert c.debug_get_stat("rccl_calls") == (1 if share == "local" else 2)
        assert c.debug_get_stat("table_local_builds") == (1 if share == "local" else 0)


def test_rccl_single_off_again_and_rejections(S):
    from mail_sieve_e import _dse
    with S.Context() as c:
        c.debug_set_option("rccl_single", 1)
        c.debug_set_option("rccl_single", 0)
        assert c.debug_get_stat("rccl_comms") == 0
        assert c.sieve_all(10**9, 1)[2] == 50_847_534
        assert c.debug_get_stat("rccl_calls") == 0  # one device, no communicator: no collective
        for bad in (-1, 2):
            with pytest.raises(_dse.DseError) as e:
                c.debug_set_option("rccl_single", bad)
            assert e.value.code == -1
        with pytest.raises(_dse.DseError):
            c.debug_get_stat("no_such_stat")
    with S.Context(logical=2) as c:  # logical devices replace the collectives by copies
        with pytest.raises(_dse.DseError) as e:
            c.debug_set_option("rccl_single", 1)
        assert e.value.code == -1

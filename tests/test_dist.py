"""Multi-process lead/follower orchestration (mail_sieve_e.core) on CPU with
gloo: rendezvous on host:port, machine numbers in arrival order, base-table
broadcast, count all-reduce, per-machine finish files, final barrier.

The per-chunk sieve is injected: these CPU tests use an oracle-backed engine
(tests only); the product engine is the HIP one (GpuEngine), covered by the
-m gpu tests.
"""
import hashlib
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleEngine:
    """Test double of core.GpuEngine on CPU tensors (gloo)."""

    backend = "gloo"

    def __init__(self, my_num):
        import torch
        self.torch = torch

    def _primes(self, limit):
        from mail_sieve_e.work import odd_primes_upto
        return odd_primes_upto(limit).astype(np.int32)

    def new_table(self, limit):
        self.limit = limit
        return self.torch.zeros(len(self._primes(limit)), dtype=self.torch.int32)

    def build_table(self, limit, table):
        table.copy_(self.torch.from_numpy(self._primes(limit)))

    def table_primes(self, limit, table):
        return table

    def finish_table(self, limit, table):
        pass

    def new_counts(self):
        return self.torch.zeros(2, dtype=self.torch.int64)

    def sieve(self, table, g_start, nbits, counts, slot, want_mask):
        from oracle import oracle as o
        # the broadcast must have delivered exactly the lead's base primes
        assert np.array_equal(table.numpy(), self._primes(self.limit)), "bad table"
        mask, c = o.fast_sieve_range(g_start, nbits, want_mask=want_mask)
        counts[slot] += c
        return mask

    def to_host_mask(self, mask):
        return mask

    def close(self):
        pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _machine(role, args, out_dir, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd"), os.path.join(ROOT, "tests")]
    from mail_sieve_e import core
    from test_dist import OracleEngine
    try:
        if role == "lead":
            r = core.lead_start(*args, out_dir=out_dir, engine_factory=OracleEngine, timeout_s=120)
        else:
            r = core.client_start(*args, out_dir=out_dir, engine_factory=OracleEngine, timeout_s=120)
        q.put(("ok", r.my_num, r.count, r.pi_ref, r.pi_full, r.bounds))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("err", repr(e)))


def _run(P, N, tmp_path):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_machine, args=("lead", (P, N, port), str(tmp_path), q))]
    procs += [ctx.Process(target=_machine, args=("follower", ("127.0.0.1", port), str(tmp_path), q))
              for _ in range(P - 1)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    errs = [r for r in res if r[0] != "ok"]
    assert not errs, errs
    return sorted(res, key=lambda r: r[1])


def test_readme_example_two_machines(tmp_path, oracle):
    # README.txt:16: N=10000 over 2 machines
    res = _run(2, 10_000, tmp_path)
    assert [r[1] for r in res] == [1, 2]
    assert [r[2] for r in res] == [668, 560]
    assert all(r[3] == 1229 and r[4] == 1229 for r in res)
    assert [list(r[5]) for r in res] == [[3, 5001], [5001, 9999]]
    sha = [hashlib.sha256((tmp_path / f"primes{k}.txt").read_bytes()).hexdigest()[:16] for k in (1, 2)]
    assert sha == ["7532ee1dc544aa7b", "7814a4d36a00515f"]


def test_run_lead_bat_three_machines(tmp_path):
    # Run Lead.bat:1: 3 machines, N=1,000,000
    res = _run(3, 1_000_000, tmp_path)
    assert [r[2] for r in res] == [28664, 25404, 24429]
    assert all(r[3] == 78498 for r in res)
    sha = [hashlib.sha256((tmp_path / f"primes{k}.txt").read_bytes()).hexdigest()[:16] for k in (1, 2, 3)]
    assert sha == ["893331a3af40a499", "7f807e9baa0ff67e", "15254ce843ba8339"]


def test_dropped_tail_is_reported(tmp_path):
    # N=100003, P=2: nums=50001, cs=25000, the tail holds 100003 (prime)
    res = _run(2, 100_003, tmp_path)
    assert res[0][3] + 1 == res[0][4]
    import sympy
    assert res[0][4] == sympy.primepi(100_003)


def test_main_usage():
    sys.path[:0] = [os.path.join(ROOT, "distributed-sieve-e_amd")]
    from mail_sieve_e import core
    assert core.main(["only-one-arg"]) == 2

"""Reference wire protocol (core.clj:13-212): mail_sieve_e.wire's lead and
follower against Python restatements of the reference machines
(oracle/ref_wire.py), checked chunk by chunk against the C oracle.

CPU tests drive the protocol with the oracle's sieve injected as the engine
(the protocol logic is what they test); the gpu tests run the product engine.
"""
import socket
import threading
import time

import numpy as np
import pytest

from mail_sieve_e import wire
from oracle import ref_wire


def _flags_to_mask(flags: bytes, cs: int) -> np.ndarray:
    bits = np.frombuffer(flags, dtype=np.uint8)
    packed = np.packbits(bits, bitorder="little")
    out = np.zeros(((cs + 63) // 64) * 8, dtype=np.uint8)
    out[: packed.size] = packed
    return out.view(np.uint64)


def _oracle_fn(oracle):
    def fn(g0, nb):
        m, c = oracle.fast_sieve_range(g0, nb)
        return m, c
    return fn


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(threads, timeout=120):
    errs = []

    def wrap(fn):
        def go():
            try:
                fn()
            except BaseException as e:  # noqa: BLE001
                errs.append(e)
        return go
    ts = [threading.Thread(target=wrap(f), daemon=True) for f in threads]
    return ts, errs


# ---------------------------------------------------------------- formatting

def test_parse_line():
    assert wire.parse_line("2") == 2
    assert wire.parse_line("[5001.0 9999.0]") == [5001.0, 9999.0]
    assert wire.parse_line("[1 0 3.0]") == [1, 0, 3.0]
    assert wire.parse_line("[2 -1 0]") == [2, -1, 0]
    assert wire.parse_line("[1 7 1.0000019E7]") == [1, 7, 10000019.0]
    assert wire.parse_line("") is None and wire.parse_line("nil") is None
    assert wire.parse_line("true") is True
    with pytest.raises(ValueError):
        wire.parse_line("[1 2")


def test_java_double_str():
    # Double.toString switches to E-notation at 1e7 (SURVEY.md Gotcha 2)
    cases = {3: "3.0", 5001: "5001.0", 9_999_991: "9999991.0", 10_000_000: "1.0E7",
             10_000_019: "1.0000019E7", 120_000_007: "1.20000007E8", 999_999_937: "9.99999937E8",
             2 * 10**9 + 1: "2.000000001E9", 10**16: "1.0E16"}
    for v, s in cases.items():
        assert wire.java_double_str(v) == s
        assert ref_wire._double(v) == s
    rng = np.random.default_rng(3)
    for v in rng.integers(3, 2**40, 2000).tolist():
        assert wire.java_double_str(v) == ref_wire._double(v)


def test_bounds_lines_match_reference_spread_work(oracle):
    for n, P in ((10_000, 2), (10**6, 3), (10**8, 7), (2 * 10**9, 16)):
        _, exact = oracle.spread_work(n, P)
        ref = ref_wire.spread_work(n, P)
        for (lo, hi), (rlo, rhi) in zip(exact, ref):
            assert wire.format_bounds((lo, hi)) == f"[{ref_wire._double(rlo)} {ref_wire._double(rhi)}]"
    assert wire.format_bounds(oracle.spread_work(10_000, 2)[1][1]) == "[5001.0 9999.0]"


def test_prime_lines(oracle):
    from mail_sieve_e.sieve import Chunk
    cs, masks, _, _ = oracle.sieve(10_000, 2)
    c1 = Chunk(3, 5001, masks[0])
    lines = wire.prime_lines(1, c1).decode().splitlines()
    assert lines[:3] == ["[1 0 3.0]", "[1 1 5.0]", "[1 2 7.0]"] and lines[-1] == "[1 -1 0]"
    c2 = Chunk(5001, 9999, masks[1])
    lines2 = wire.prime_lines(2, c2).decode().splitlines()
    assert lines2[0] == "[2 1 5003]" and lines2[-1] == "[2 -1 0]"
    assert len(lines) + len(lines2) - 2 == 1228    # prime messages of the reference run


# ------------------------------------------------------- all-reference pin

def test_reference_machines_match_oracle(oracle):
    """Pins ref_wire's restated machines to the C oracle: one reference lead
    and two reference followers over real sockets."""
    n, P = 30_000, 3
    cs, masks, _, _ = oracle.sieve(n, P)
    srv = socket.create_server(("127.0.0.1", 0))
    port = srv.getsockname()[1]
    res = [dict() for _ in range(P)]
    ts, errs = _run([lambda: ref_wire.ref_lead(P, n, srv, res[0])] +
                    [lambda r=r: ref_wire.ref_client("127.0.0.1", port, r) for r in res[1:]])
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    srv.close()
    assert not errs, errs
    for r in res:
        assert r["cs"] == cs
        np.testing.assert_array_equal(_flags_to_mask(r["flags"], cs), masks[r["my_num"] - 1])


# ------------------------------------------------------------ mixed rings

def _mixed_wire_lead(oracle, tmp_path, sieve_fn, n=40_000, P=4):
    """wire lead (machine 1) + reference, wire, reference followers (2, 3, 4)."""
    cs, masks, _, _ = oracle.sieve(n, P)
    port = _free_port()
    ready = threading.Event()
    out = {}
    refs = [dict(), dict()]

    def lead():
        out["lead"] = wire.lead_start(P, n, port, host="127.0.0.1", out_dir=str(tmp_path), sieve_fn=sieve_fn,
                                      timeout_s=120, ready=ready)

    def follower():
        out["f"] = wire.client_start("127.0.0.1", port, out_dir=str(tmp_path), sieve_fn=sieve_fn, timeout_s=120)

    ts, errs = _run([lead])
    ts[0].start()
    assert ready.wait(30)
    order = [lambda: ref_wire.ref_client("127.0.0.1", port, refs[0]), follower,
             lambda: ref_wire.ref_client("127.0.0.1", port, refs[1])]
    fts, ferrs = _run(order)
    for t in fts:                        # arrival order = machine numbers 2, 3, 4
        t.start()
        time.sleep(0.3)
    for t in fts + ts:
        t.join(120)
    assert not errs and not ferrs, errs + ferrs
    assert [r["my_num"] for r in refs] == [2, 4]
    for r in refs:
        np.testing.assert_array_equal(_flags_to_mask(r["flags"], cs), masks[r["my_num"] - 1])
    np.testing.assert_array_equal(out["lead"].mask, masks[0])
    np.testing.assert_array_equal(out["f"].mask, masks[2])
    for k in (1, 3):
        exp = tmp_path / f"exp{k}.txt"
        oracle.finish(str(exp), k, n, P, masks[k - 1])
        assert (tmp_path / f"primes{k}.txt").read_bytes() == exp.read_bytes()


def _mixed_ref_lead(oracle, tmp_path, sieve_fn, n=40_000, P=3):
    """reference lead (machine 1) + wire follower (2) + reference follower (3)."""
    cs, masks, _, _ = oracle.sieve(n, P)
    srv = socket.create_server(("127.0.0.1", 0))
    port = srv.getsockname()[1]
    acc = threading.Semaphore(0)
    lead_res, ref_res, out = dict(), dict(), {}

    def follower():
        out["f"] = wire.client_start("127.0.0.1", port, out_dir=str(tmp_path), sieve_fn=sieve_fn, timeout_s=120)

    ts, errs = _run([lambda: ref_wire.ref_lead(P, n, srv, lead_res, acc), follower,
                     lambda: ref_wire.ref_client("127.0.0.1", port, ref_res)])
    ts[0].start()
    ts[1].start()
    assert acc.acquire(timeout=60)       # the wire follower is machine 2
    ts[2].start()
    for t in ts:
        t.join(120)
    srv.close()
    assert not errs, errs
    assert ref_res["my_num"] == 3
    np.testing.assert_array_equal(_flags_to_mask(lead_res["flags"], cs), masks[0])
    np.testing.assert_array_equal(out["f"].mask, masks[1])
    np.testing.assert_array_equal(_flags_to_mask(ref_res["flags"], cs), masks[2])
    exp = tmp_path / "exp2.txt"
    oracle.finish(str(exp), 2, n, P, masks[1])
    assert (tmp_path / "primes2.txt").read_bytes() == exp.read_bytes()


def test_wire_lead_protocol_cpu(oracle, tmp_path):
    _mixed_wire_lead(oracle, tmp_path, _oracle_fn(oracle))


def test_wire_follower_protocol_cpu(oracle, tmp_path):
    _mixed_ref_lead(oracle, tmp_path, _oracle_fn(oracle))


def test_wire_single_machine_ends(oracle, tmp_path):
    # P = 1: the reference lead waits forever for an appoint; this one returns
    c = wire.lead_start(1, 10_000, _free_port(), host="127.0.0.1", out_dir=str(tmp_path),
                        sieve_fn=_oracle_fn(oracle), timeout_s=30)
    assert c.n_primes == 1228


@pytest.mark.gpu
def test_wire_lead_gpu(oracle, tmp_path):
    _mixed_wire_lead(oracle, tmp_path, None, n=400_000, P=4)


@pytest.mark.gpu
def test_wire_follower_gpu(oracle, tmp_path):
    _mixed_ref_lead(oracle, tmp_path, None, n=400_000, P=3)


def _silent_lead(behaviour):
    """A lead that accepts one follower and then `behaviour(conn)`; listens on
    a port of its own choosing (bound here, so no other test can take it
    between a free-port probe and the bind) and returns (thread, port)."""
    srv = socket.create_server(("127.0.0.1", 0))
    port = srv.getsockname()[1]
    def go():
        c, _ = srv.accept()
        try:
            behaviour(c)
        finally:
            c.close()
            srv.close()
    t = threading.Thread(target=go, daemon=True)
    t.start()
    return t, port


def test_wire_follower_finite_timeout_is_a_protocol_error(oracle):
    """A finite timeout (tests only; the default waits forever like the
    reference) ends in a RuntimeError naming the wait, not queue.Empty."""
    done = threading.Event()  # the lead stays silent until the client has given up (a fixed sleep
    t, port = _silent_lead(lambda c: done.wait(60))  # raced the 0.5 s wait on a loaded host)
    try:
        with pytest.raises(RuntimeError, match="within"):
            wire.client_start("127.0.0.1", port, sieve_fn=_oracle_fn(oracle), timeout_s=0.5, write_file=False)
    finally:
        done.set()
    t.join(5)


def test_wire_follower_eof_before_number(oracle):
    t, port = _silent_lead(lambda c: None)  # closes at once
    with pytest.raises(RuntimeError, match="machine number"):
        wire.client_start("127.0.0.1", port, sieve_fn=_oracle_fn(oracle), write_file=False)
    t.join(5)


def test_wire_default_waits_are_unbounded():
    import inspect
    assert inspect.signature(wire.client_start).parameters["timeout_s"].default is None
    assert inspect.signature(wire.lead_start).parameters["timeout_s"].default is None


def test_main_rejects_bad_timeout(capsys):
    """-main's optional --timeout: missing or non-positive values print the
    usage line and return 2 instead of raising."""
    from mail_sieve_e import wire
    for argv in (["localhost", "1", "--timeout"], ["localhost", "1", "--timeout", "abc"],
                 ["--timeout", "-3", "localhost", "1"], ["just-one-arg"]):
        assert wire.main(argv) == 2, argv
        assert "usage:" in capsys.readouterr().err

"""The oracle (oracle/dse_oracle.c) pinned before it is trusted.

The reference ships no fixtures and cannot run here (Clojure/JVM absent), so
the faithful restatement is pinned by: the README's chunk size
(README.txt:16), the SURVEY.md section 4 known-answer table, published
pi(10^k), sympy.isprime sweeps, and the committed golden fixtures.
"""
import hashlib
import json
import os

import numpy as np
import pytest

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def test_spread_work_readme_example(oracle):
    # README.txt:16 - N=10000 over two machines: "~2500" per chunk; exact cs=2499
    cs, bounds = oracle.spread_work(10_000, 2)
    assert cs == 2499
    assert bounds == [(3, 5001), (5001, 9999)]


@pytest.mark.parametrize("N,P,cs,dropped", [
    (10**4, 2, 2499, 1), (10**9, 1, 499_999_999, 0),
    (10**10, 2, 2_499_999_999, 1), (10**10, 4, 1_249_999_999, 3), (10**10, 8, 624_999_999, 7),
    (10**11, 1, 49_999_999_999, 0), (10**11, 2, 24_999_999_999, 1), (10**11, 4, 12_499_999_999, 3),
    (10**11, 8, 6_249_999_999, 7), (10**12, 8, 62_499_999_999, 7)])
def test_spread_work_survey_table(oracle, N, P, cs, dropped):
    # SURVEY.md section 8 table, Appendix A.1
    got, bounds = oracle.spread_work(N, P)
    assert got == cs
    assert (N - 1) // 2 - P * cs == dropped
    assert bounds[0][0] == 3 and all(bounds[k][1] == bounds[k + 1][0] for k in range(P - 1))


def test_tail_holds_largest_prime_below_1e12(oracle):
    # SURVEY.md Gotcha 1: the dropped tail at N=1e12, P=8 contains 999999999989
    g, nb = oracle.tail_range(10**12, 8)
    vals = [3 + 2 * (g + i) for i in range(nb)]
    assert 999_999_999_989 in vals
    _, c = oracle.fast_sieve_range(g, nb)
    assert c == 1


def test_survey_known_answer_files(oracle, tmp_path):
    # bytes, lines, sha256[:16] of primes{k}.txt
    want = {(10_000, 1): (5088, 67, "7532ee1dc544aa7b", 669), (10_000, 2): (3304, 56, "7814a4d36a00515f", 560),
            (10**6, 1): (272765, 2867, "893331a3af40a499", 28665), (10**6, 2): (200691, 2541, "7f807e9baa0ff67e", 25404),
            (10**6, 3): (192989, 2443, "15254ce843ba8339", 24429)}
    for (N, P) in [(10_000, 2), (10**6, 3)]:
        cs, masks, counts, msgs = oracle.sieve(N, P)
        for k in range(P):
            p = str(tmp_path / f"primes{k + 1}.txt")
            oracle.finish(p, k + 1, N, P, masks[k])
            b = open(p, "rb").read()
            nbytes, lines, sha16, nonzero = want[(N, k + 1)]
            assert (len(b), b.count(b"\n"), hashlib.sha256(b).hexdigest()[:16]) == (nbytes, lines, sha16)
            assert int(counts[k]) + (1 if k == 0 else 0) == nonzero
    assert oracle.sieve(10_000, 2)[3] == 1228      # prime messages
    assert oracle.sieve(10**6, 3)[3] == 78497


def test_first_file_format(oracle, tmp_path):
    # sieve.clj:93-105: 2.0 3.0 5.0 7.0 hack, Doubles in chunk 1, 10 per line
    cs, masks, _, _ = oracle.sieve(10_000, 2)
    p = tmp_path / "p1.txt"
    oracle.finish(str(p), 1, 10_000, 2, masks[0])
    lines = p.read_bytes().split(b"\n")
    assert lines[0] == b"2.0, 3.0, 5.0, 7.0, 11.0, 13.0, 17.0, 19.0, 23.0, 29.0"
    assert lines[-1] == b""
    p2 = tmp_path / "p2.txt"
    oracle.finish(str(p2), 2, 10_000, 2, masks[1])
    assert p2.read_bytes().startswith(b"5003, 5009, 5011")


def test_java_double_formatting(oracle, tmp_path):
    # Double.toString switches to E-notation at 1e7 (SURVEY.md Gotcha 2)
    N = 2 * 10**9
    cs, _ = oracle.spread_work(N, 1)
    mask = np.zeros((cs + 63) // 64, dtype=np.uint64)
    for v in (9_999_991, 10_000_019, 120_000_007, 999_999_937):
        j = (v - 3) // 2
        mask[j // 64] |= np.uint64(1) << np.uint64(j % 64)
    p = tmp_path / "p.txt"
    oracle.finish(str(p), 1, N, 1, mask)
    assert p.read_bytes() == b"2.0, 3.0, 5.0, 7.0, 9999991.0, 1.0000019E7, 1.20000007E8, 9.99999937E8\n"


def _sympy():
    return pytest.importorskip("sympy")


def test_oracle_vs_sympy_sweep(oracle):
    sympy = _sympy()
    rng = np.random.default_rng(0x5EED)
    iso = np.zeros(60_001, dtype=bool)
    for p in sympy.primerange(3, 60_001):
        iso[p] = True
    n_cases = 0
    while n_cases < 150:
        N = int(rng.integers(20, 60_001))
        P = int(rng.integers(1, 9))
        cs, bounds = oracle.spread_work(N, P)
        if cs < 4:
            continue
        _, masks, counts, _ = oracle.sieve(N, P)
        for k in range(P):
            bits = np.unpackbits(masks[k].view(np.uint8), bitorder="little")[:cs].astype(bool)
            vals = np.arange(bounds[k][0], bounds[k][1], 2)
            assert np.array_equal(bits, iso[vals]), (N, P, k)
        assert oracle.pi_ref(counts) == sympy.primepi(1 + 2 * P * cs)
        g, nb = oracle.tail_range(N, P)
        _, ct = oracle.fast_sieve_range(g, nb, want_mask=False)
        assert oracle.pi_ref(counts) + ct == sympy.primepi(N)
        n_cases += 1


def test_oracle_pi_1e8(oracle):
    _, _, counts, _ = oracle.sieve(10**8, 1)
    assert oracle.pi_ref(counts) == 5_761_455


def test_fast_sieve_matches_ref(oracle):
    rng = np.random.default_rng(7)
    for _ in range(10):
        N = int(rng.integers(10**5, 3 * 10**6))
        P = int(rng.integers(1, 9))
        cs, masks, counts, _ = oracle.sieve(N, P)
        for k in range(P):
            m, c = oracle.fast_sieve_range(k * cs, cs)
            assert np.array_equal(m, masks[k]) and c == int(counts[k])


def test_golden_sweep_reproduces(oracle):
    # fixtures in tests/golden/golden.json are what the oracle computes
    for case in GOLDEN["sweep"][:40]:
        cs, masks, counts, msgs = oracle.sieve(case["N"], case["P"])
        assert cs == case["cs"]
        assert [int(c) for c in counts] == case["counts"]
        assert [hashlib.sha256(m.view(np.uint8).tobytes()).hexdigest() for m in masks] == case["mask_sha256"]
        assert msgs == case["prime_messages"]


def test_golden_big_constants():
    big = GOLDEN["big"]
    assert big["1e9_P1"]["pi_ref"] == 50_847_534
    for P in (2, 4, 8):
        assert big[f"1e10_P{P}"]["pi_ref"] == 455_052_511 == big[f"1e10_P{P}"]["pi_full"]


@pytest.mark.parametrize("N,P", [(10_000, 2), (1_000_000, 3), (54_321, 7), (2_000_003, 8), (777, 1)])
def test_threaded_run_equals_faithful(oracle, N, P):
    """ref_sieve_threaded (P machine threads + the relay thread, in-process
    queues; bench.py's cpu_baseline) reproduces ref_sieve bit for bit,
    including the number of prime messages (1,228 / 78,497)."""
    a = oracle.sieve(N, P)
    b = oracle.sieve_threaded(N, P)
    assert a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and a[3] == b[3]


@pytest.mark.parametrize("lo,hi", [(3, 10**6), (2, 2), (10**9, 10**9 + 10**6), (10**12 + 7, 10**12 + 3 * 10**6),
                                   (10**15, 10**15 + 2 * 10**6), (999_999_999_989, 10**12)])
def test_count_window_vs_fast_sieve(oracle, lo, hi):
    """fast_count_window (the independent window counter behind the golden
    [1e18, 1e18+1e10] count) agrees with the segmented fast sieve."""
    a = max(lo, 3) | 1
    b = hi if hi % 2 else hi - 1
    want = 0 if b < a else oracle.fast_sieve_range((a - 3) // 2, (b - a) // 2 + 1, want_mask=False)[1]
    assert oracle.count_window(lo, hi) == want


def test_golden_streamed_headline_entries():
    """1e11 P=1/2/4/8 (and, when generated, 1e12 P=8) golden chunk hashes:
    counts add up to the published pi, chunk sizes follow spread-work."""
    for P in (1, 2, 4, 8):
        g = GOLDEN["big"][f"1e11_P{P}"]
        assert g["cs"] == (10**11 - 1) // 2 // P and len(g["mask_sha256"]) == P
        assert 1 + sum(g["counts"]) == g["pi_ref"] == g["pi_full"] == 4_118_054_813
    g = GOLDEN["big"].get("1e12_P8")
    if g is not None:
        assert g["pi_ref"] == 37_607_912_017 and g["pi_full"] == 37_607_912_018
    assert GOLDEN["big"]["window_1e18"]["count"] == 241_272_176

"""The analytic work counts behind bench.py's rooflines (mail_sieve_e/work.py),
checked against direct enumeration on small ranges (CPU only)."""
import math

import numpy as np

from mail_sieve_e import work


def _brute_wheel_marks(va, vb, pmin, pmax):
    ps = [int(p) for p in work.odd_primes_upto(pmax) if p > pmin]
    n = 0
    for p in ps:
        m = max(p, -(-va // p))
        while p * m <= vb:
            n += math.gcd(m, 30) == 1
            m += 1
    return n


def test_wheel_marks_small_ranges():
    rng = np.random.default_rng(5)
    for _ in range(6):
        g0 = int(rng.integers(0, 10**7))
        nb = int(rng.integers(1, 2 * 10**5))
        va, vb = 3 + 2 * g0, 3 + 2 * (g0 + nb - 1)
        want = _brute_wheel_marks(va, vb, work.WHEEL_PATTERN_MAX, math.isqrt(vb))
        assert work.wheel_marks_for_range(g0, nb) == want, (g0, nb)


def test_bucket_entries_small_window():
    """Bucketed primes 2^19 < p <= sqrt(vmax) of a high window: one entry per
    multiple p*m with gcd(m, 30) = 1 (every such multiple is >= p^2 here)."""
    lo = 10**13 + 12345
    g0, nb = (lo - 3) // 2, 150_000
    va, vb = 3 + 2 * g0, 3 + 2 * (g0 + nb - 1)
    want = _brute_wheel_marks(va, vb, work.BUCKET_LO, math.isqrt(vb))
    assert want > 0
    assert work.bucket_entries_for_range(g0, nb) == want


def test_window_bucket_entries_constant():
    """WINDOW_BUCKET_ENTRIES against the Mertens estimate 1e10 * 8/30 *
    (ln ln 1e9 - ln ln 2^19) (within 2%); tools/window_entries.py recomputes it
    exactly (15 s, 1 GB)."""
    est = 1e10 * 8 / 30 * (math.log(math.log(1e9)) - math.log(math.log(2**19)))
    assert abs(work.WINDOW_BUCKET_ENTRIES / est - 1) < 0.02

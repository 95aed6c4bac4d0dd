"""Long randomized parity sweep (beyond the unit tests): random odd-index
ranges at magnitudes 1e3..1e17, lengths 1..3e7, GPU (C ABI) against the
oracle's independent segmented sieve, bit for bit. Stops after a time budget.

  python tools/parity_sweep.py [seconds] [seed]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
import numpy as np  # noqa: E402
from mail_sieve_e.sieve import Context  # noqa: E402
from oracle import oracle as o  # noqa: E402  (the checker)


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0x5EED
    rng = np.random.default_rng(seed)
    ctx = Context(1)
    t0 = time.time()
    n = bad = 0
    bits_checked = 0
    while time.time() - t0 < budget:
        mag = rng.uniform(3, 17)
        g0 = int(10 ** mag) // 2 + int(rng.integers(0, 1 << 20))
        nb = int(10 ** rng.uniform(0, 7.5))
        if mag > 15:
            nb = min(nb, 2_000_000)   # keep the oracle's base sieve and segment work bounded
        m, c = ctx.sieve_odd_range(g0, nb)
        m_ref, c_ref = o.fast_sieve_range(g0, nb)
        ok = c == c_ref and np.array_equal(m, m_ref)
        n += 1
        bits_checked += nb
        if not ok:
            bad += 1
            diff = np.flatnonzero(m != m_ref)
            print(f"MISMATCH g0={g0} nb={nb} count {c} vs {c_ref} first words {diff[:4]}", flush=True)
        if n % 50 == 0:
            print(f"{n} ranges, {bits_checked:.3e} odd candidates, {bad} mismatches, {time.time() - t0:.0f} s",
                  flush=True)
    print(f"done: {n} ranges, {bits_checked:.3e} odd candidates checked bit for bit, {bad} mismatches", flush=True)
    ctx.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

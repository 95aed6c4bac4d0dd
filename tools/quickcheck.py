"""Ad-hoc GPU check used during development: parity on small ranges + timing."""
import os, sys, time, hashlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
import numpy as np
from oracle import oracle as o
from mail_sieve_e.sieve import Context

ctx = Context(1)
rng = np.random.default_rng(0x5EED)
bad = 0
for t in range(200):
    N = int(rng.integers(20, 2_000_000)); P = int(rng.integers(1, 9))
    cs, _ = o.spread_work(N, P)
    if cs < 4: continue
    _, m_ref, c_ref, _ = o.sieve(N, P)
    for k in range(P):
        m, c = ctx.sieve_chunk(N, P, k + 1)
        if c != int(c_ref[k]) or not np.array_equal(m, m_ref[k]):
            bad += 1
            diff = np.flatnonzero(m != m_ref[k])
            print("MISMATCH", N, P, k + 1, c, int(c_ref[k]), diff[:5], flush=True)
print("sweep mismatches:", bad, flush=True)
for g0, nb in [(0, 1), (0, 5), (1, 63), (123457, 999), (10**9 + 7, 3 * 2**20 + 13), (5 * 10**10, 2**21 + 777)]:
    m_ref, c_ref = o.fast_sieve_range(g0, nb)
    m, c = ctx.sieve_odd_range(g0, nb)
    print("range", g0, nb, c, c_ref, np.array_equal(m, m_ref), flush=True)
for N, P in [(10**9, 1), (10**10, 2), (10**11, 1)]:
    ctx.sieve_all(N, P)
    t = time.time(); counts, pr, pf = ctx.sieve_all(N, P); dt = time.time() - t
    print(f"N={N:.0e} P={P} pi_ref={pr} pi_full={pf} t={dt*1e3:.2f} ms  {N/dt:.3e} int/s", flush=True)

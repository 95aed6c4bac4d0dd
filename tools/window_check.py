"""Dev check: high-offset windows vs the oracle, MR spot checks, timing."""
import os, sys, time, random
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
import numpy as np
from oracle import oracle as o
from mail_sieve_e.sieve import Context

def is_prime(n):
    if n < 2: return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0: return n == p
    d, s = n - 1, 0
    while d % 2 == 0: d //= 2; s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1): continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1: break
        else: return False
    return True

c = Context(1)
for lo, w in [(4 * 10**12, 10**8), (10**15, 10**7), (10**18, 2 * 10**6)]:
    a = lo | 1; g0 = (a - 3) // 2; nb = w // 2
    t = time.time(); m, cnt = c.sieve_odd_range(g0, nb); tg = time.time() - t
    t = time.time(); mr, cr = o.fast_sieve_range(g0, nb); tc = time.time() - t
    print(f"lo={lo:.0e} w={w:.0e} gpu={cnt} oracle={cr} equal={np.array_equal(m, mr)} t_gpu={tg:.3f}s t_cpu={tc:.1f}s", flush=True)
rng = random.Random(5)
g0 = (10**18 + 1 - 3) // 2; nb = 5 * 10**7
m, cnt = c.sieve_odd_range(g0, nb)
bits = np.unpackbits(m.view(np.uint8), bitorder="little")
bad = 0
idx = [rng.randrange(nb) for _ in range(3000)] + list(np.flatnonzero(bits[:nb])[:3000])
for j in idx:
    v = 3 + 2 * (g0 + int(j))
    if bool(bits[j]) != is_prime(v): bad += 1
print("MR spot checks:", len(idx), "mismatches:", bad, flush=True)
c.sieve_window(10**18, 10**18 + 10**9)
t = time.time(); cw = c.sieve_window(10**18, 10**18 + 10**10); dt = time.time() - t
print(f"window [1e18, 1e18+1e10]: count={cw} t={dt:.3f}s {1e10/dt:.3e} int/s", flush=True)
parts = sum(c.sieve_window(10**18 + k * 10**9 + (1 if k else 0), 10**18 + (k + 1) * 10**9) for k in range(10))
print("sum of 10 sub-windows:", parts, "equal:", parts == cw, flush=True)

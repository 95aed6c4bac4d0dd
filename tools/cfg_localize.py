"""Profiling aid: find where DSE_CFG=1 diverges from the oracle (sqrt thresholds)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
import numpy as np
from oracle import oracle as o
from mail_sieve_e.sieve import Context
c = Context(1)
for sq in [3000, 5000, 8000, 8500, 12000, 16000, 17000, 30000, 33000, 40000]:
    vmax = sq * sq
    nb = 2**19 * 3 + 11
    g0 = (vmax - 3) // 2 - nb
    m, cnt = c.sieve_odd_range(g0, nb)
    mr, cr = o.fast_sieve_range(g0, nb)
    bad = np.flatnonzero(m != mr)
    extra = ""
    if bad.size:
        w = bad[0]; x = int(m[w]) ^ int(mr[w]); b = w * 64 + (x & -x).bit_length() - 1
        v = 3 + 2 * (g0 + b)
        fs = [p for p in range(3, 50000, 2) if v % p == 0][:3]
        extra = f" first bad bit {b} (seg {b >> 19}, in-seg {b & (2**19-1)}, col {(b & (2**19-1)) >> 13}) value {v} gpu={int(m[w])>>((x&-x).bit_length()-1)&1} factors {fs}"
    print(sq, cnt, cr, "OK" if cnt == cr and not bad.size else "BAD" + extra, flush=True)

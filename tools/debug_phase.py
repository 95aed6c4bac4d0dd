"""Debug aid: compare one kernel phase (DSE_PHASES) with a numpy sieve restricted
to that phase's primes on one range. Usage: DSE_PHASES=.. debug_phase.py lo hi"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
import numpy as np
from mail_sieve_e import _dse
if os.environ.get("DSE_LIB"): _dse.LIB_PATH = os.environ["DSE_LIB"]
from mail_sieve_e.sieve import Context
from mail_sieve_e.work import odd_primes_upto
plo, phi = int(sys.argv[1]), int(sys.argv[2])
g0, nb = 10**7 + 12345, 3 * 2**20 + 77
c = Context(1)
m, cnt = c.sieve_odd_range(g0, nb)
bits = np.unpackbits(m.view(np.uint8), bitorder="little")[:nb].astype(bool)
vals = 3 + 2 * (g0 + np.arange(nb, dtype=np.int64))
comp = np.zeros(nb, dtype=bool)
for p in odd_primes_upto(int(vals[-1] ** 0.5) + 1):
    if p <= 61 or plo < p <= phi:
        start = max(p * p, ((vals[0] + p - 1) // p) * p)
        if start % 2 == 0: start += p
        comp[(start - vals[0]) // 2::p] = True
ref = ~comp
bad = np.flatnonzero(bits != ref)
print(os.environ.get("DSE_PHASES"), plo, phi, "bad", bad.size, "extra marks", int((ref[bad]).sum()),
      "missing marks", int((~ref[bad]).sum()), "first", bad[:5], flush=True)
for b in bad[:6]:
    v = int(vals[b]); fs = [int(p) for p in odd_primes_upto(5000) if v % p == 0][:3]
    print("  bit", b, "seg", b >> 20, "col", (b & (2**20 - 1)) >> 14, "off", b & 16383, "v", v, "factors", fs, "gpu", bits[b])

"""Exact bucket-entry count of the 1e18 window (BASELINE config 5) for
work.WINDOW_BUCKET_ENTRIES: every multiple p*m of the primes 2^19 < p <= 1e9 + 4
with gcd(m, 30) = 1 among the window's odd values [1e18 + 1, 1e18 + 1e10 - 1]
(bench.py --window's range). One-off, ~10 s and ~1 GB of numpy."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-sieve-e_amd"))
from mail_sieve_e import work  # noqa: E402

lo, hi = 10**18, 10**18 + 10**10
g = (lo + 1 - 3) // 2
nb = (hi - 1 - (lo + 1)) // 2 + 1
t = time.time()
print(work.bucket_entries_for_range(g, nb), f"({time.time() - t:.1f} s)")

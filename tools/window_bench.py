"""Window [1e18, 1e18+1e10] on one GPU: base table (odd primes <= 1e9+4) +
bucketed sieve, timed end to end (profiling aid; config 4 of BASELINE.json)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
from mail_sieve_e import _dse
if os.environ.get("DSE_LIB"): _dse.LIB_PATH = os.environ["DSE_LIB"]
from mail_sieve_e.sieve import Context
lo, hi = 10**18, 10**18 + 10**10
c = Context(1)
c.sieve_window(lo, hi)
ts = []
for _ in range(3):
    t = time.perf_counter(); n = c.sieve_window(lo, hi); ts.append(time.perf_counter() - t)
assert n == 241272176 or os.environ.get('DSE_NOCHECK'), n
print(f"window [1e18, 1e18+1e10]: {n} primes, best {min(ts)*1e3:.2f} ms, {(hi-lo)/min(ts):.3e} integers/s", flush=True)

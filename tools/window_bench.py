"""Window [1e18, 1e18+1e10] on one GPU: base table (odd primes <= 1e9+4) +
bucketed sieve, timed end to end (profiling aid; config 4 of BASELINE.json).
Test-only context options: `python tools/window_bench.py name=value ...`
(dse_debug_set_option, e.g. bucket_overlap=0 bucket_pass_segments=768)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
from mail_sieve_e import _dse
if os.environ.get("DSE_LIB"): _dse.LIB_PATH = os.environ["DSE_LIB"]
from mail_sieve_e.sieve import Context
lo, hi = 10**18, 10**18 + 10**10
c = Context(1)
for kv in sys.argv[1:]:
    k, v = kv.split("=")
    c.debug_set_option(k, int(v))
c.sieve_window(lo, hi)
ts = []
for _ in range(5):
    t = time.perf_counter(); n = c.sieve_window(lo, hi); ts.append(time.perf_counter() - t)
assert n == 241272176 or os.environ.get('DSE_NOCHECK'), n
ts.sort()
print(f"window [1e18, 1e18+1e10] {' '.join(sys.argv[1:])}: {n} primes, best {ts[0]*1e3:.2f} ms, median {ts[2]*1e3:.2f} ms, "
      f"{(hi-lo)/ts[0]:.3e} integers/s", flush=True)

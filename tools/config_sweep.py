"""Every BASELINE.json config on ONE MI355X through the C ABI (dse_sieve_all /
dse_sieve_window), timed as SURVEY.md 8(d) scopes it: from the call to the
count on the host, median of 5 after one warm call. Chunks of a P-chunk config
run back to back on the one device (the driver's multi-GPU runs are bench.py's).

  python tools/config_sweep.py [out.json]
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
from mail_sieve_e import _dse  # noqa: E402
if os.environ.get("DSE_LIB"):  # A/B another build of the library
    _dse.LIB_PATH = os.environ["DSE_LIB"]
from mail_sieve_e import work  # noqa: E402
from mail_sieve_e.sieve import Context  # noqa: E402

KNOWN = {10**9: 50_847_534, 10**10: 455_052_511, 10**11: 4_118_054_813, 10**12: 37_607_912_018}
CONFIGS = [(10**9, 1), (10**10, 2), (10**10, 4), (10**10, 8), (10**11, 1), (10**11, 8), (10**12, 8)]
WINDOW = (10**18, 10**18 + 10**10, 241_272_176)


def timed(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t)
    return r, statistics.median(ts), min(ts)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    ctx = Context(1)
    rows = []
    for N, P in CONFIGS:
        (counts, pi_ref, pi_full), med, best = timed(lambda: ctx.sieve_all(N, P))
        marks = work.marks_for_range(0, (N - 1) // 2)
        row = {"config": f"N={N:.0e} P={P}", "N": N, "P": P, "pi_ref": pi_ref, "pi_full": pi_full,
               "verified": pi_full == KNOWN[N], "ms_median": med * 1e3, "ms_best": best * 1e3,
               "integers_per_s": N / med, "lds_roof_frac": 8 * marks / (work.LDS_PEAK_GBS * 1e9) / med}
        rows.append(row)
        print(json.dumps(row), flush=True)
    lo, hi, exp = WINDOW
    n, med, best = timed(lambda: ctx.sieve_window(lo, hi))
    row = {"config": "window [1e18, 1e18+1e10]", "count": n, "verified": n == exp, "ms_median": med * 1e3,
           "ms_best": best * 1e3, "integers_per_s": (hi - lo) / med}
    rows.append(row)
    print(json.dumps(row), flush=True)
    ctx.close()
    if out:
        with open(out, "w") as f:
            json.dump({"gpus": 1, "timing": "call to count on host, median of 5 after one warm call",
                       "rows": rows}, f, indent=1)
    if not all(r["verified"] for r in rows):
        sys.exit(1)


if __name__ == "__main__":
    main()

"""Per-wave phase and unit-class cycles of the wheel kernel from a timing build
(tools/instrument_timing.py -> variants/libdse_timing.so): for each config,
one warm call, then the s_memtime sums of one call, divided by the waves of
the launch(es), at 2.4 GHz. Profiling aid.

  python tools/wave_timing.py [1e11] [1e12] [window]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
from mail_sieve_e import _dse  # noqa: E402
_dse.LIB_PATH = os.path.join(ROOT, "variants", os.environ.get("DSE_TIMING_LIB", "libdse_timing.so"))
from mail_sieve_e.sieve import Context  # noqa: E402

NAMES = ["mark", "mark barrier wait", "expand", "init", "segment barrier wait",
         "  A units", "  B1 units", "  B2 units", "  L units", "  bucket units"]
CLK = 2.4e9


def take():
    buf = (ctypes.c_ulonglong * 96)()
    assert _dse.lib().dse_debug_timing(buf) == 0
    return list(buf)


def report(label, fn, waves):
    fn()
    take()
    fn()
    t = take()
    total = sum(t[:5])
    print(f"== {label}")
    for i, n in enumerate(NAMES):
        ms = t[i] / waves / CLK * 1e3
        share = f"({100 * t[i] / total:5.1f}%)" if i < 5 else f"({100 * t[i] / max(t[0], 1):5.1f}% of mark)"
        print(f"{n:24s} {ms:8.3f} ms per wave  {share}")
    rest = t[0] - sum(t[5:10])
    print(f"{'  unit loop rest':24s} {rest / waves / CLK * 1e3:8.3f} ms per wave")
    print(f"{'sum':24s} {total / waves / CLK * 1e3:8.3f} ms per wave", flush=True)
    # per wave id (256 waves each): mark, mark barrier, expand, init, segment barrier
    print("wave id   mark  mark-wait  expand   init  seg-wait  (ms per wave)")
    for w in range(16):
        r = [t[16 + 5 * w + i] / (waves // 16) / CLK * 1e3 for i in range(5)]
        print(f"{w:7d} " + " ".join(f"{x:7.3f}" for x in r), flush=True)


def main():
    which = sys.argv[1:] or ["1e11", "1e12", "window"]
    c = Context(1)
    waves = 256 * 16
    for w in which:
        if w == "window":
            report("window [1e18, 1e18+1e10]", lambda: c.sieve_window(10**18, 10**18 + 10**10), waves)
        else:
            n = int(float(w))
            mask = n <= 10**11  # the bench's mask write at 1e11; count only at 1e12 (62.5 GB)
            report(f"N={w}, P=1{'' if mask else ' (count only)'}",
                   lambda: c.sieve_odd_range(0, (n - 1) // 2, want_mask=mask), waves)
    c.close()


if __name__ == "__main__":
    main()

"""Profiling aid: where a wave's time goes in the wheel kernel, from the
s_memtime stamps of a -DDSE_TIMING build (variants/libdse_timing.so:
bash tools/build_variant.sh timing -DDSE_TIMING). Prints the per-wave cycles of
each phase summed over a launch at N (default 1e11) or the window, as ms of kernel time."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
from mail_sieve_e import _dse
_dse.LIB_PATH = os.path.join(ROOT, "variants", os.environ.get("DSE_TIMING_LIB", "libdse_timing.so"))
from mail_sieve_e.sieve import Context
arg = sys.argv[1] if len(sys.argv) > 1 else "1e11"
c = Context(1)
buf = (ctypes.c_ulonglong * 8)()
# "window": [1e18, 1e18+1e10] (its base-table build runs the wheel kernel too: both are summed)
run = (lambda: c.sieve_window(10**18, 10**18 + 10**10)) if arg == "window" else (lambda: c.sieve_all(int(float(arg)), 1))
run()                                  # warm up
assert _dse.lib().dse_debug_timing(buf) == 0
run()
assert _dse.lib().dse_debug_timing(buf) == 0
waves = 256 * 16
clk = 2.4e9 / 1e3                      # s_memtime ticks per ms at the 2.4 GHz shader clock (approximate)
names = ["mark", "mark barrier wait", "expand", "init", "segment barrier wait"]
tot = sum(buf[:5])
for n, v in zip(names, buf[:5]):
    print(f"{n:22s} {v / waves / clk:7.3f} ms per wave  ({100 * v / tot:5.1f}%)")
print(f"{'sum':22s} {tot / waves / clk:7.3f} ms per wave")
for n, v in zip(["  A units", "  B units", "  L units"], buf[5:]):
    print(f"{n:22s} {v / waves / clk:7.3f} ms per wave  ({100 * v / buf[0]:5.1f}% of mark)")
print(f"{'  unit loop rest':22s} {(buf[0] - sum(buf[5:])) / waves / clk:7.3f} ms per wave")

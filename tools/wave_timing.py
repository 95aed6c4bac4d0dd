"""Debug aid: per-wave phase cycle counts of the wheel kernel (DSE_TIMING build,
variants/libdse_timing.so), segment 5 of each workgroup, N=1e11."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
import numpy as np
from mail_sieve_e import _dse
_dse.LIB_PATH = os.path.join(ROOT, "variants", os.environ.get("DSE_TIMING_LIB", "libdse_timing.so"))
from mail_sieve_e.sieve import Context
c = Context(1)
c.sieve_all(10**11, 1)
buf = (ctypes.c_ulonglong * (256 * 16 * 5))()
assert _dse.lib().dse_debug_timing(buf) == 0
t = np.frombuffer(buf, dtype=np.uint64).reshape(256, 16, 5).astype(np.int64)
t -= t[:, :, :1].min(axis=1, keepdims=True)
init_end = t[:, :, 1]
mark_busy = t[:, :, 2] - t[:, :, 1]
mark_wall = t[:, :, 3].max(axis=1) - t[:, :, 1].min(axis=1)
exp = t[:, :, 4] - t[:, :, 3]
seg = t[:, :, 4].max(axis=1)
# stamps: 0 = 1 = mark start (the segment's init ran at the end of the previous
# iteration), 2 = mark done, 3 = after the barrier, 4 = expand + next init done
print("cycles per segment (median over WGs): total %d  init %d  mark wall %d  expand+next init %d" % (
    np.median(seg), np.median(init_end.max(axis=1)), np.median(mark_wall), np.median(exp.max(axis=1))))
print("mark busy per wave: min %d median %d max %d (median over WGs); imbalance max/mean = %.3f" % (
    np.median(mark_busy.min(axis=1)), np.median(np.median(mark_busy, axis=1)), np.median(mark_busy.max(axis=1)),
    np.median(mark_busy.max(axis=1) / mark_busy.mean(axis=1))))
print("per-wave mark busy, WG 0:", mark_busy[0].tolist())

"""Full vs half-size segment geometry (test option wheel_geometry: 0 auto,
1 full only, 2 half only) on the chunks of the multi-chunk configs, one GPU:
kernel ms from HIP events on the launch stream (median of 5), counts checked
equal across geometries. Measures DSE_HALF_SEG_COST and the tail split.

  python tools/geometry_ab.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
import torch  # noqa: E402
from mail_sieve_e import _dse  # noqa: E402
if os.environ.get("DSE_LIB"):
    _dse.LIB_PATH = os.environ["DSE_LIB"]
from mail_sieve_e import sieve as S  # noqa: E402

SEG = 1966080  # odd candidates per full segment


def main():
    dev = torch.device("cuda", 0)
    ctx = S.Context(device=0)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    cases = [("1 segment", 2 * SEG * 256 - 1, 256, 0), ("256 segments", 2 * SEG * 256 + 1, 1, 0), ("1e9 P=1", 10**9, 1, 0), ("1e10 P=8 chunk 8", 10**10, 8, 7), ("1e10 P=4 chunk 4", 10**10, 4, 3),
             ("1e10 P=2 chunk 2", 10**10, 2, 1), ("1e11 P=8 chunk 8", 10**11, 8, 7), ("1e11 P=1", 10**11, 1, 0)]
    for name, N, P, k in cases:
        cs = (N - 1) // 2 // P
        limit = S.base_limit_for_range(0, (N - 1) // 2)
        table = torch.empty(S.base_table_bytes(limit), dtype=torch.uint8, device=dev)
        ctx.base_primes_dev_async(limit, table.data_ptr(), table.numel(), sp)
        mask = torch.empty((cs + 63) // 64, dtype=torch.int64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        res = {}
        for geo in (1, 2, 0):
            ctx.debug_set_option("wheel_geometry", geo)
            ts, c = [], None
            for r in range(6):
                cnt.zero_()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                ctx.sieve_range_dev_async(table.data_ptr(), k * cs, cs, mask.data_ptr(), cnt.data_ptr(), sp)
                b.record(stream)
                b.synchronize()
                if r:
                    ts.append(a.elapsed_time(b))
                c = int(cnt.item())
            res[geo] = (statistics.median(ts), c)
        assert res[0][1] == res[1][1] == res[2][1], (name, res)
        nseg = -(-cs // SEG)
        print(f"{name:20s} segments={nseg:6d} ({nseg / 256:6.2f} rounds)  full {res[1][0]:8.3f} ms  "
              f"half {res[2][0]:8.3f} ms (x{res[2][0] / res[1][0]:.3f})  auto {res[0][0]:8.3f} ms  count {res[0][1]}",
              flush=True)
    ctx.debug_set_option("wheel_geometry", 0)


if __name__ == "__main__":
    main()

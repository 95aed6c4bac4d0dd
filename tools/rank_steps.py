"""What each rank of an N-GPU bench step would cost, measured on one GPU:
the base table build plus the sieve of every spread-work chunk k of P, each
timed with HIP events on the launch stream (median of 5). The max over chunks
is the multi-GPU critical path without the collectives.

  python tools/rank_steps.py [N] [P]     (DSE_OPTS=name=value,... sets test-only options)
  python tools/rank_steps.py window [P]  the [1e18, 1e18+1e10] window as bench.py --window
                                         splits it: each rank builds its own table (the
                                         203 MB of primes are not broadcast) and sieves a slice
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
import torch  # noqa: E402
from mail_sieve_e import _dse, sieve as S  # noqa: E402

if os.environ.get("DSE_LIB"):  # A/B another build of the library
    _dse.LIB_PATH = os.environ["DSE_LIB"]


def window(P):
    dev = torch.device("cuda", 0)
    ctx = S.Context(device=0)
    lo, hi = 10**18, 10**18 + 10**10
    g_all, nb_all = (lo + 1 - 3) // 2, (hi - 1 - (lo + 1)) // 2 + 1
    part = (nb_all + P - 1) // P
    limit = S.base_limit_for_range(g_all, nb_all)
    tbytes = S.base_table_bytes(limit)
    table = torch.empty(tbytes, dtype=torch.uint8, device=dev)
    counts = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def timed(fn, reps=5):
        fn()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn()
            b.record(stream)
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return statistics.median(ts)

    t_base = timed(lambda: ctx.base_primes_dev_async(limit, table.data_ptr(), tbytes, sp))
    pb = S.base_table_prime_bytes(limit)
    print(f"window P={P} slice={part} odd values; local base table (limit {limit}, {pb / 1e6:.0f} MB of primes, "
          f"not broadcast: {S.base_table_broadcast_bytes(limit)} B): {t_base * 1e3:.1f} us", flush=True)
    worst, total = 0.0, 0
    for r in range(P):
        g0 = g_all + min(nb_all, part * r)
        n = min(nb_all, part * (r + 1)) - min(nb_all, part * r)
        counts.zero_()
        t = timed(lambda: ctx.sieve_range_dev_async(table.data_ptr(), g0, n, 0, counts.data_ptr(), sp))
        worst = max(worst, t)
        counts.zero_()
        ctx.sieve_range_dev_async(table.data_ptr(), g0, n, 0, counts.data_ptr(), sp)
        total += int(counts.item())
        print(f"slice {r + 1}: {t:.3f} ms", flush=True)
    print(f"window critical path (local table + worst slice): {t_base + worst:.3f} ms -> "
          f"{(hi - lo) / (t_base + worst) / 1e-3:.3e} integers/s over {P} GPUs, all-reduce excluded; "
          f"primes {total} ({'ok' if total == 241272176 else 'WRONG'})", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "window":
        return window(int(sys.argv[2]) if len(sys.argv) > 2 else 8)
    N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**11
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda", 0)
    ctx = S.Context(device=0)
    for kv in filter(None, os.environ.get("DSE_OPTS", "").split(",")):  # test-only options, name=value
        k, v = kv.split("=")
        ctx.debug_set_option(k, int(v))
    cs = (N - 1) // 2 // P
    tail_n = (N - 1) // 2 - P * cs
    limit = S.base_limit_for_range(0, P * cs + tail_n)
    tbytes = S.base_table_bytes(limit)
    table = torch.empty(tbytes, dtype=torch.uint8, device=dev)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    mask = torch.empty((cs + 63) // 64, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def timed(fn, reps=5):
        fn()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn()
            b.record(stream)
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return statistics.median(ts)

    t_base = timed(lambda: ctx.base_primes_dev_async(limit, table.data_ptr(), tbytes, sp))
    print(f"N={N:.0e} P={P} cs={cs} base table: {t_base * 1e3:.1f} us", flush=True)
    worst = 0.0
    for k in range(P):
        t = timed(lambda: ctx.sieve_range_dev_async(table.data_ptr(), k * cs, cs, mask.data_ptr(), counts.data_ptr(), sp))
        worst = max(worst, t)
        print(f"chunk {k + 1}: {t:.3f} ms", flush=True)
    print(f"critical path (base + worst chunk): {t_base + worst:.3f} ms -> {N / (t_base + worst) / 1e-3:.3e} integers/s "
          f"over {P} GPUs, collectives excluded", flush=True)


if __name__ == "__main__":
    main()

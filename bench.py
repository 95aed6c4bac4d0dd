#!/usr/bin/env python3
"""bench.py -- sieved integers/s at N=1e11 on 1/2/4/8 MI355X (BASELINE.json metric).

One step = the whole hot path for N over P = n_gpus chunks (spread-work,
sieve.clj:15-34), with every rank's inputs already on its GPU:
  rank 0 builds the base primes <= sqrt(N) on its GPU -> RCCL broadcast of the
  primes to the other ranks (mirrors the reference's prime broadcast,
  sieve.clj:139), which derive Barrett factors and wheel offsets -> each
  rank sieves its chunk into an odd-only bitmask in HBM + count -> the last rank
  also sieves the dropped tail -> RCCL all-reduce of the counts -> the counts
  on the host.
Timing: every step runs from the call to the counts on the
host; the headline is the median over the K timed steps of the per-step
maximum over ranks. The K steps are also bracketed by barrier + synchronize
(ms_per_step_bracketed), and K launches are timed back to back without host
round trips (ms_per_step_pipelined).
--window: the high-offset window [1e18, 1e18+1e10] split over the ranks
(BASELINE config 5): rank 0 builds the base primes <= 1e9 + 4, RCCL
broadcast, every rank sieves one contiguous slice, RCCL all-reduce.
Single GPU: `python bench.py`; N GPUs: torch.distributed.run --nproc-per-node N.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import datetime
import faulthandler
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mail_sieve_e import _dse  # noqa: E402
if os.environ.get("DSE_LIB"):  # profiling only: A/B another build of the library
    _dse.LIB_PATH = os.environ["DSE_LIB"]
from mail_sieve_e import sieve as S  # noqa: E402
from mail_sieve_e import work  # noqa: E402

METRIC = "sieved integers/sec at N=1e11, 1/2/4/8 MI355X; % of LDS/HBM roofline"
WINDOW_METRIC = "sieved integers/sec, window [1e18, 1e18+1e10] (BASELINE config 5), 1/8 MI355X"
KNOWN_PI = {10**9: 50847534, 10**10: 455052511, 10**11: 4118054813, 10**12: 37607912018}
WINDOW = (10**18, 10**18 + 10**10)
WINDOW_COUNT = 241272176  # oracle fast_count_window, tests/golden/golden.json


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", "--N", dest="n", type=float, default=1e11,
                    help="sieve limit N (default 1e11, the headline); spell it --N under torch.distributed.run")
    ap.add_argument("--window", action="store_true", help="the [1e18, 1e18+1e10] window instead of [3, N]")
    ap.add_argument("--no-mask", action="store_true", help="count only (not the product path; diagnostics)")
    ap.add_argument("--cpu-baseline", choices=["on", "off"], default="on")
    ap.add_argument("--cpu-max-n", type=float, default=1e8, help="largest N of the CPU baseline runs")
    ap.add_argument("--rccl-single", action="store_true",
                    help="one GPU only: form a 1-rank nccl (RCCL) process group and run the step's broadcast and "
                         "all-reduce through it, as every rank of an N-GPU run does (exercises the RCCL path)")
    return ap.parse_args()


def cpu_baseline(max_n: int, reps: int = 3) -> dict:
    """The reference's lead + followers on this host's cores (SURVEY.md 8(d)
    fallback: no JVM in the image): oracle/dse_oracle.c ref_sieve_threaded,
    P machine threads + machine 1's relay thread exchanging [mi ps p]
    messages through in-process queues (core.clj:118-134, sieve.clj:131-172),
    at P = 2 and 3 on the README (1e4) and Run Lead.bat (1e6) workloads and up
    to max_n. Each (N, P) runs `reps` times and reports the median; the
    calling thread is pinned to P + 1 cores of its allowed set for the run
    (os.sched_setaffinity, inherited by the machine threads; restored after),
    so the threads do not migrate across the box's cores. Test infrastructure:
    reported only, never the measured path."""
    from oracle import oracle as o
    o.lib()
    allowed = sorted(os.sched_getaffinity(0))
    runs = []
    ns = [n for n in (10**4, 10**6, 10**7, 10**8, 10**9) if n <= max_n]
    try:
        for n in ns:
            for P in (2, 3):
                cores = allowed[:P + 1]
                os.sched_setaffinity(0, cores)
                ts = []
                for _ in range(reps):
                    t = time.perf_counter()
                    _, _, counts, msgs = o.sieve_threaded(n, P, want_masks=False)
                    ts.append(time.perf_counter() - t)
                    if n in KNOWN_PI:
                        tail_g, tail_n = o.tail_range(n, P)
                        _, ct = o.fast_sieve_range(tail_g, tail_n, want_mask=False) if tail_n else (None, 0)
                        assert o.pi_ref(counts) + ct == KNOWN_PI[n], (n, P)
                dt = statistics.median(ts)
                runs.append({"N": n, "P": P, "threads": P + 1, "cores": cores, "seconds": dt,
                             "seconds_all": ts, "integers_per_s": n / dt, "prime_messages": int(msgs)})
    finally:
        os.sched_setaffinity(0, allowed)
    top = max(r["N"] for r in runs)
    h2 = next(r for r in runs if r["N"] == top and r["P"] == 2)
    h3 = next(r for r in runs if r["N"] == top and r["P"] == 3)
    return {"value": h3["integers_per_s"], "unit": "integers/s", "cores": h3["threads"], "kind": "port",
            "nproc": os.cpu_count(), "allowed_cores": len(allowed), "pinned_cores": h3["cores"],
            "value_P2": h2["integers_per_s"], "value_P3": h3["integers_per_s"],
            "sample": f"N={top:.0e}, P=3 (P=2 beside it as value_P2): oracle/dse_oracle.c ref_sieve_threaded, the "
                      f"reference's lead + 2 followers as 3 machine threads + the relay thread pinned to cores "
                      f"{h3['cores']} of {len(allowed)} allowed ({os.cpu_count()} on the host), per-prime [mi ps p] "
                      f"messages through in-process queues ({h3['prime_messages']} messages), median of {reps} runs "
                      f"{h3['seconds']:.2f} s; the Clojure reference cannot run (no JVM in the image)",
            "runs": runs}


def lib_build():
    """The library this run loaded: its path and the first 16 hex digits of its
    SHA-256, the id that profiles/<round>/pmc_build.json records for the build
    its traces and counters were taken from (so a line, e.g. the one printed
    under a rocprofv3 trace, names its own build)."""
    import hashlib
    from mail_sieve_e import _dse
    path = _dse.LIB_PATH
    with open(path, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    return {"libdse": os.path.relpath(path, ROOT), "libdse_sha256_16": sha}


def pmc_summary(N: int, P: int, window: bool):
    """Per-launch figures of the sieve kernel from the committed rocprofv3 PMC
    passes for this config (profiles/<round>/pmc_*_sieve_kernel.csv, N=1e11,
    P=1): HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB counters; MI355X_MICROARCH.md:
    gfx950 FETCH_SIZE counts half of a wide coalesced read, WRITE_SIZE is exact);
    VALU issue against the 2.0 wave-instructions per CU-cycle ceiling, LDS busy
    (SQ_LDS_IDX_ACTIVE per CU-cycle) and the bank-conflict share of it
    (GRBM_GUI_ACTIVE is summed over the 8 XCDs). Figures are per step: a
    step's range may run as a main launch plus a half-geometry tail launch
    (DESIGN.md section 4.1.2), so each counter is summed over every row of
    the kernel and divided by the number of main (largest-grid) dispatches."""
    import collections
    import csv
    import glob
    if window or (N, P) != (10**11, 1):
        return None
    for d in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")), reverse=True):
        try:
            tot = collections.defaultdict(float)
            steps = {}
            for f in ("pmc_fetch_sieve_kernel.csv", "pmc_write_sieve_kernel.csv", "pmc_sq_sieve_kernel.csv",
                      "pmc_wait_sieve_kernel.csv"):
                rows = [r for r in csv.DictReader(open(os.path.join(d, f)))
                        if "wheel_segments_kernel" in r["Kernel_Name"]]
                grid = max(int(r["Grid_Size"]) for r in rows)
                for r in rows:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"])
                    if int(r["Grid_Size"]) == grid:
                        steps.setdefault(r["Counter_Name"], set()).add(r["Dispatch_Id"])
            v = {k: x / len(steps[k]) for k, x in tot.items()}
            cyc = v["GRBM_GUI_ACTIVE"] / 8
            try:
                build = json.load(open(os.path.join(d, "pmc_build.json")))
            except OSError:
                build = None
            return {"traffic": (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024, "source": os.path.relpath(d, ROOT),
                    "build": build, "cycles": cyc, "sq_insts_valu": v["SQ_INSTS_VALU"],
                    "valu_issue_per_cu_cycle": v["SQ_INSTS_VALU"] / work.NUM_CUS / cyc,
                    "valu_frac": v["SQ_INSTS_VALU"] / work.NUM_CUS / cyc / work.VALU_PEAK_PER_CU_CYCLE,
                    "lds_busy": v["SQ_LDS_IDX_ACTIVE"] / work.NUM_CUS / cyc,
                    "lds_conflict_share": v["SQ_LDS_BANK_CONFLICT"] / v["SQ_LDS_IDX_ACTIVE"],
                    "sq_insts_lds": v["SQ_INSTS_LDS"]}
        except (OSError, KeyError, ZeroDivisionError):
            continue
    return None


def pmc_window_traffic():
    """HBM bytes of one --window sieve call from the newest committed PMC passes
    (profiles/<round>/pmc_window_{fetch,write}.csv: rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE of `bench.py --window`): 2*FETCH_SIZE + WRITE_SIZE (KiB counters,
    MI355X_MICROARCH.md gfx950 correction) summed over every kernel, divided by
    the wheel-kernel dispatches (one per call)."""
    import csv
    import glob
    for d in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")), reverse=True):
        try:
            tot = {}
            for c, f in (("FETCH_SIZE", "pmc_window_fetch.csv"), ("WRITE_SIZE", "pmc_window_write.csv")):
                rows = list(csv.DictReader(open(os.path.join(d, f))))
                calls = {r["Dispatch_Id"] for r in rows if "wheel_segments_kernel" in r["Kernel_Name"]}
                tot[c] = sum(float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == c) / len(calls)
            try:
                build = json.load(open(os.path.join(d, "pmc_build.json")))
            except OSError:
                build = None
            return {"traffic": (2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024, "source": os.path.relpath(d, ROOT),
                    "build": build}
        except (OSError, KeyError, ZeroDivisionError):
            continue
    return None


def lds_instr_check(wm: int, cs: int, pmc):
    """The analytic executed-mark count against the PMC's LDS wave-instructions
    per launch: SQ_INSTS_LDS = the marks (wm / 64 full-wave ds_or_b32) + the
    expansion and init instructions, which the kernel's structure fixes per
    segment (expand: 2 ds_read_b128 + 32 LUT ds_read_b32 per lane-block, 4,096
    blocks; init: 9 x (5 + 5 + 1) ds_read_b128 table reads + 33 ds_write_b32
    per lane, 1,024 lanes; csrc/dse_wheel.hip expand_segment / init_segment) +
    a rest: unit claims, the mid-prime residue reads and writes, and the ds_or
    of predicated marks issued with part of the wave (A-class and B tails, L
    planes with <= 2 hits), which the analytic count of hits cannot see. A
    negative rest, or one far above ~10%, would mean the analytic count is
    off. (A half-geometry tail segment has half the blocks and fewer init
    instructions per lane: counted here as full segments, < 0.1% at N=1e11.)"""
    if not pmc:
        return None
    nseg = -(-cs // work.WHEEL_OUT_BITS)
    mark_i = wm / 64
    expand_i = nseg * (4096 // 64) * 34
    init_i = nseg * (1024 // 64) * (work.WHEEL_PATTERN_GROUPS * 11 + 33)
    rest = pmc["sq_insts_lds"] - mark_i - expand_i - init_i
    return {"sq_insts_lds": pmc["sq_insts_lds"], "marks_analytic": mark_i, "expand": expand_i, "init": init_i,
            "rest": rest, "rest_share": rest / pmc["sq_insts_lds"],
            "unit": "LDS wave-instructions per launch"}


class Watchdog:
    """A stuck rank must end the run with a diagnosable non-zero exit, not run
    into the driver's time limit: every phase (rendezvous, warmup, timed steps,
    gather of the per-rank figures ...) has a deadline; past it the rank
    prints its rank, world size and phase and every thread's stack to stderr
    and exits with status 3. Collectives also carry the process group's
    timeout (init_process_group(timeout=...)). DSE_BENCH_PHASE_TIMEOUT_S
    (default 300) sets both."""

    def __init__(self, rank: int, world: int, limit_s: float):
        self.rank, self.world, self.limit = rank, world, limit_s
        self.name, self.t0 = "start", time.monotonic()
        self.lock = threading.Lock()
        threading.Thread(target=self._run, daemon=True).start()

    def phase(self, name: str) -> None:
        with self.lock:
            self.name, self.t0 = name, time.monotonic()

    def where(self) -> str:
        return f"bench.py rank {self.rank}/{self.world} in phase '{self.name}'"

    def _run(self):
        while True:
            time.sleep(1.0)
            with self.lock:
                late = time.monotonic() - self.t0 > self.limit
                msg = f"{self.where()}: no progress for {self.limit:.0f} s, exiting"
            if late:
                print(msg, file=sys.stderr, flush=True)
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                os._exit(3)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    wd = Watchdog(rank, world, float(os.environ.get("DSE_BENCH_PHASE_TIMEOUT_S", "300")))
    try:
        run(a, world, rank, wd)
    except BaseException as e:  # noqa: BLE001 -- name the rank and phase, then re-raise
        print(f"{wd.where()}: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        raise


def run(a, world: int, rank: int, wd: Watchdog):
    local = int(os.environ.get("LOCAL_RANK", "0"))
    timeout = datetime.timedelta(seconds=wd.limit)
    # DSE_BENCH_REHEARSE=1: rehearsal of the N-rank code path on a 1-GPU box
    # (gloo, every rank on cuda:0); its timings mean nothing.
    rehearse = os.environ.get("DSE_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if a.rccl_single and world != 1:
        sys.exit("--rccl-single is for a one-process run")
    pg = world > 1 or a.rccl_single  # the step's collectives run through a process group
    wd.phase("init_process_group")
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo", timeout=timeout)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
    elif a.rccl_single:
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                                device_id=torch.device("cuda", local), timeout=timeout)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    P = world  # one spread-work chunk (or window slice) per GPU
    if a.window:
        lo, hi = WINDOW
        N = hi - lo                                  # integers covered
        g_all, nb_all = (lo + 1 - 3) // 2, (hi - 1 - (lo + 1)) // 2 + 1  # odd values lo+1 .. hi-1
        part = (nb_all + P - 1) // P
        g0, cs = g_all + min(nb_all, part * rank), min(nb_all, part * (rank + 1)) - min(nb_all, part * rank)
        tail_g = tail_n = 0
        limit = S.base_limit_for_range(g_all, nb_all)
        with_mask = False
    else:
        N = int(a.n)
        cs = (N - 1) // 2 // P
        g0 = rank * cs
        tail_g, tail_n = P * cs, (N - 1) // 2 - P * cs
        limit = S.base_limit_for_range(0, P * cs + tail_n)
        with_mask = not a.no_mask
    words = (cs + 63) // 64

    # the world this run formed (a SCALE line shows its N ranks and their devices)
    me = {"rank": rank, "local_rank": local, "device": torch.cuda.current_device(),
          "pci_bus_id": getattr(torch.cuda.get_device_properties(dev), "pci_bus_id", None)}
    wd.phase("gather rank info")
    ranks = [me]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
    ctx = S.Context(device=local)
    tbytes = S.base_table_bytes(limit)
    # the primes are all a broadcast needs to carry (109 KB at N=1e11); a table
    # past the broadcast cap (the window's 203 MB) is built on every rank
    # instead (include/dse.h dse_base_table_broadcast_bytes)
    pbytes = S.base_table_broadcast_bytes(limit)
    share = "broadcast" if pbytes else "local"
    world_info = {"backend": dist.get_backend() if pg else None, "size": world, "ranks": ranks,
                  "rehearsal": rehearse, "rccl_single": a.rccl_single,
                  "base_table": {"limit": limit, "path": share,
                                 "bytes": pbytes if pbytes else S.base_table_prime_bytes(limit),
                                 "rule": "rank 0 builds and broadcasts the primes while they fit in 8 MiB; "
                                         "above that every rank builds its own table"}}
    table = torch.empty(tbytes, dtype=torch.uint8, device=dev)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    mask = torch.empty(words, dtype=torch.int64, device=dev) if with_mask else None
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    kev = []  # (start, end) HIP events around each sieve launch, on the stream it runs on

    def launch(timed=False):
        counts.zero_()
        if rank == 0 or not pbytes:
            ctx.base_primes_dev_async(limit, table.data_ptr(), tbytes, sp)
        if pg and pbytes:
            dist.broadcast(table[:pbytes], src=0)
            if rank != 0:
                ctx.base_table_finish_dev_async(limit, table.data_ptr(), tbytes, sp)
        if timed:
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            e[0].record(stream)
        ctx.sieve_range_dev_async(table.data_ptr(), g0, cs, mask.data_ptr() if mask is not None else 0,
                                  counts.data_ptr(), sp)
        if timed:
            e[1].record(stream)
            kev.append(e)
        if rank == world - 1 and tail_n:
            ctx.sieve_range_dev_async(table.data_ptr(), tail_g, tail_n, 0, counts.data_ptr() + 8, sp)
        if pg:
            dist.all_reduce(counts)

    def step(timed=False):
        """call -> counts on the host"""
        t = time.perf_counter()
        launch(timed)
        c = counts.cpu().tolist()
        return time.perf_counter() - t, c

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier(device_ids=None if rehearse else [local])

    wd.phase("warmup")
    for _ in range(a.warmup):
        step()
    barrier()
    wd.phase("timed steps")
    t0 = time.perf_counter()
    step_s = []
    for _ in range(a.steps):
        dt, c = step(timed=True)
        step_s.append(dt)
    barrier()
    t1 = time.perf_counter()
    # back-to-back launches without host round trips (the r01 headline method)
    wd.phase("pipelined steps")
    barrier()
    tp0 = time.perf_counter()
    for _ in range(a.steps):
        launch()
    barrier()
    tp1 = time.perf_counter()

    wd.phase("reduce timings")
    step_t = torch.tensor(step_s + [t1 - t0, tp1 - tp0], dtype=torch.float64, device=dev)
    kern = sum(e0.elapsed_time(e1) for e0, e1 in kev) / len(kev) / 1e3  # s per sieve launch
    kern_t = torch.tensor([kern], dtype=torch.float64, device=dev)
    # this rank's own figures, next to its device in world.ranks (a SCALE line
    # can then be checked rank by rank against profiles/*/rank_steps.txt)
    mine = {"step_ms": statistics.median(step_s) * 1e3, "kernel_ms": kern * 1e3,
            "bracketed_ms": (t1 - t0) / a.steps * 1e3, "pipelined_ms": (tp1 - tp0) / a.steps * 1e3,
            "g_start": g0, "nbits": cs, "tail_nbits": tail_n if rank == world - 1 else 0}
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        dist.all_reduce(step_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(kern_t, op=dist.ReduceOp.MAX)
    for r, x in zip(ranks, per_rank):
        r.update(x)
    wd.phase("report")
    st = step_t.cpu().tolist()
    med = statistics.median(st[:a.steps])
    bracketed, pipelined = st[a.steps] / a.steps, st[a.steps + 1] / a.steps
    if a.window:
        pi_ref = pi_full = c[0]
        verified = c[0] == WINDOW_COUNT
    else:
        pi_ref, pi_full = 1 + c[0], 1 + c[0] + c[1]
        verified = KNOWN_PI.get(N) == pi_full if N in KNOWN_PI else None
    if rank == 0:
        ks = kern_t.item()
        if a.window:
            workload = f"window [1e18, 1e18+1e10] split into {P} slice(s), one per GPU (count only, segment-only)"
            rf = None
            # the bucketed pass is the window's dominant cost (bucket fill/stage
            # ~57% of a call): HBM-bound on its entries, 4 B written by the fill
            # and read back by the wheel kernel per hit of a prime > 2^19
            entries = work.WINDOW_BUCKET_ENTRIES * cs / nb_all  # this rank's share (exact at one rank)
            alg = 2 * work.BUCKET_ENTRY_BYTES * entries
            wp = pmc_window_traffic()
            achieved = alg / ks / 1e9
            window_roofline = {
                "bound": "hbm", "achieved": achieved, "peak": work.HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / work.HBM_PEAK_GBS,
                "traffic": wp["traffic"] * cs / nb_all if wp else None,
                "traffic_source": f"committed PMC passes {wp['source']} (not this run; scaled to this rank's share)"
                                  if wp else None,
                "kernel": "the window's bucketed sieve call: every kernel of one sieve_range call (bucket range, "
                          "count, column/start scans, fill + stage, sort, wheel kernel), HIP events on its stream",
                "kernel_ms": ks * 1e3,
                "bucket_entries_per_launch": entries,
                "basis": "8 B per bucket entry (4 B written by bucket_fill_stage_kernel / the band-1 sort, 4 B read "
                         "back by the wheel kernel) of every hit p*m, gcd(m, 30) = 1, of the primes 2^19 < p <= 1e9+4 "
                         "in the window (mail_sieve_e/work.py WINDOW_BUCKET_ENTRIES, tools/window_entries.py) against "
                         "8 TB/s HBM",
            }
        else:
            workload = (f"N={N:.0e} odd-only chunked sieve, P={P} spread-work chunks (one per GPU), mask resident "
                        "in HBM" + (" [count-only diagnostic]" if a.no_mask else ""))
            rf = work.roofline(g0, cs, ks)
        pmc = pmc_summary(N, P, a.window) if with_mask else None
        out = {
            "metric": WINDOW_METRIC if a.window else METRIC,
            "value": N / med,
            "unit": "integers/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": med * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "deterministic (sieve of [3, N]; no input data)" if not a.window else
                    "deterministic (the window's odd values; no input data)",
            "config": {"workload": workload, "N": N, "P": P, "cs": cs,
                       "mask_bytes_per_gpu": words * 8 if with_mask else 0,
                       "parallelism": f"range-partition x{P} (RCCL broadcast + all-reduce)"},
            "timing": "median over steps of the per-step max over ranks, call -> counts on the host",
            "ms_per_step_bracketed": bracketed * 1e3,
            "ms_per_step_pipelined": pipelined * 1e3,
            "pi_ref": pi_ref,
            "pi_full": pi_full,
            "verified": verified,
            "roofline": None,
            "cpu_baseline": None,
            "world": world_info,
            "build": lib_build(),
        }
        if a.window:
            out["roofline"] = window_roofline
        if rf is not None:
            wm = rf["wheel_marks"]
            achieved = work.LDS_OR_BYTES_PER_MARK * wm / ks / 1e9
            mark_instr_per_cu = wm / 64 / work.NUM_CUS  # full-wave ds_or_b32 per CU
            out["roofline"] = {
                "bound": "lds",
                "achieved": achieved,
                "peak": work.LDS_OR_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / work.LDS_OR_PEAK_GBS,
                "traffic": pmc["traffic"] if pmc else None,
                "traffic_source": f"committed PMC pass {pmc['source']} (not this run)" if pmc else None,
                "basis": "executed ds_or_b32 marks (mod-30 wheel, primes > 79) x 4 B per kernel second against "
                         "the LDS store path (64 B/clk/CU); kernel time from HIP events on the launch stream",
                "peak_ds_or": work.LDS_DS_OR_PEAK_GBS,
                "frac_ds_or": achieved / work.LDS_DS_OR_PEAK_GBS,
                "ds_or_basis": f"the measured conflict-free ds_or_b32 rate, {work.DS_OR_CYCLES_PER_WAVE_INSTR} "
                               "CU-cycles per wave-instruction (profiles/r02/lds_conflict_microbench.txt)",
                "cycles_per_mark_instr": ks * work.CLOCK_HZ / mark_instr_per_cu,
                "cycles_per_mark_instr_basis": "live: kernel seconds x 2.4 GHz / (executed marks / 64 / 256 CUs); "
                                               f"floor {work.DS_OR_CYCLES_PER_WAVE_INSTR}",
                "kernel": "wheel_segments_kernel", "kernel_ms": ks * 1e3,
                "executed_marks_per_launch": wm,
                "frac_algorithmic": rf["frac"],
                "algorithmic_marks_per_launch": rf["marks"],
                "algorithmic_basis": "SURVEY 8(d): 8 B x odd-only marks from p^2 / 78.6 TB/s; the wheel executes "
                                     f"{wm / rf['marks']:.3f} of them, so this exceeds 1",
                "hbm_bytes_per_launch": rf["hbm_bytes"],
                "hbm_frac_algorithmic": rf["hbm_bytes"] / ks / 1e9 / work.HBM_PEAK_GBS,
                "executed_marks_source": "analytic (mail_sieve_e/work.py wheel_marks_for_range: multiples p*m >= p^2 "
                                         "with gcd(m, 30) = 1 of the primes 79 < p <= sqrt(N)), cross-checked "
                                         "against SQ_INSTS_LDS in pmc_committed.lds_instr_check",
                # Read from the newest committed rocprofv3 PMC passes of this config
                # (profiles/<round>/pmc_*_sieve_kernel.csv), NOT measured in this run;
                # `build` names the library those passes profiled.
                "pmc_committed": None if not pmc else {
                    "source": pmc["source"],
                    "build": pmc["build"],
                    "same_build": bool(pmc["build"]) and pmc["build"].get("libdse_sha256_16") == out["build"]["libdse_sha256_16"],
                    "traffic": pmc["traffic"],
                    "hbm_frac": pmc["traffic"] / ks / 1e9 / work.HBM_PEAK_GBS,
                    "cycles_per_cu": pmc["cycles"],
                    "cycles_per_mark_instr": pmc["cycles"] / mark_instr_per_cu,
                    "valu_per_mark_instr": pmc["sq_insts_valu"] / (wm / 64),
                    "valu_frac": pmc["valu_frac"],
                    "valu_issue_per_cu_cycle": pmc["valu_issue_per_cu_cycle"],
                    "lds_busy": pmc["lds_busy"],
                    "lds_conflict_share": pmc["lds_conflict_share"],
                    "lds_instr_check": lds_instr_check(wm, cs, pmc),
                },
            }
        if world == 1 and a.cpu_baseline == "on" and not a.window:
            wd.phase("cpu baseline")
            out["cpu_baseline"] = cpu_baseline(int(a.cpu_max_n))
        print(json.dumps(out), flush=True)
    wd.phase("shutdown")
    ctx.close()
    if pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

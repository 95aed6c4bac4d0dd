#!/usr/bin/env python3
"""bench.py -- sieved integers/s at N=1e11 on 1/2/4/8 MI355X (BASELINE.json metric).

One step = the whole hot path for N over P = n_gpus chunks (spread-work,
sieve.clj:15-34), with every rank's inputs already on its GPU:
  rank 0 builds the base primes <= sqrt(N) on its GPU -> RCCL broadcast of the
  primes to the other ranks (mirrors the reference's prime broadcast,
  sieve.clj:139), which derive Barrett factors and wheel offsets -> each
  rank sieves its chunk into an odd-only bitmask in HBM + count -> the last rank
  also sieves the dropped tail -> RCCL all-reduce of the counts.
Single GPU: `python bench.py`; N GPUs: torch.distributed.run --nproc-per-node N.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
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
KNOWN_PI = {10**9: 50847534, 3 * 10**9: 144449537, 10**10: 455052511, 10**11: 4118054813, 10**12: 37607912018}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", "--N", dest="n", type=float, default=1e11,
                    help="sieve limit N (default 1e11, the headline); spell it --N under torch.distributed.run")
    ap.add_argument("--no-mask", action="store_true", help="count only (not the product path; diagnostics)")
    ap.add_argument("--cpu-baseline", choices=["on", "off"], default="on")
    ap.add_argument("--cpu-sample-n", type=float, default=3e9)
    return ap.parse_args()


def cpu_baseline(sample_n: int) -> dict:
    """Time the oracle's faithful single-thread restatement of sieve.clj on a
    bounded sample (rank 0, N=1 only). Test infrastructure: reported only."""
    from oracle import oracle as o
    o.lib()
    t = time.perf_counter()
    _, _, counts, msgs = o.sieve(sample_n, 1)
    dt = time.perf_counter() - t
    assert o.pi_ref(counts) == KNOWN_PI.get(sample_n, o.pi_ref(counts))
    return {"value": sample_n / dt, "unit": "integers/s", "cores": 1, "kind": "port",
            "sample": f"N={sample_n:.0e}, P=1 chunk: oracle/dse_oracle.c ref_sieve (faithful C restatement of "
                      f"sieve.clj's per-prime lead loop, {msgs} prime messages), {dt:.2f} s on 1 host core; "
                      "the Clojure reference cannot run (no JVM in the image)"}


def pmc_summary(N: int, P: int):
    """Per-launch figures of the sieve kernel from the committed rocprofv3 PMC
    passes for this config (profiles/<round>/pmc_*_sieve_kernel.csv, N=1e11,
    P=1): HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB counters; MI355X_MICROARCH.md:
    gfx950 FETCH_SIZE counts half of a wide coalesced read, WRITE_SIZE is exact),
    and the VALU / LDS wave-instruction issue rates per CU per cycle
    (GRBM_GUI_ACTIVE is summed over the 8 XCDs)."""
    import collections
    import csv
    import glob
    if (N, P) != (10**11, 1):
        return None
    for d in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")), reverse=True):
        try:
            vals = collections.defaultdict(list)
            for f in ("pmc_fetch_sieve_kernel.csv", "pmc_write_sieve_kernel.csv", "pmc_sq_sieve_kernel.csv",
                      "pmc_wait_sieve_kernel.csv"):
                for r in csv.DictReader(open(os.path.join(d, f))):
                    if "wheel_segments_kernel" in r["Kernel_Name"]:
                        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            v = {k: sum(x) / len(x) for k, x in vals.items()}
            cyc = v["GRBM_GUI_ACTIVE"] / 8
            return {"traffic": (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024, "source": os.path.relpath(d, ROOT),
                    "valu_issue_per_cu_cycle": v["SQ_INSTS_VALU"] / 256 / cyc,
                    "lds_issue_per_cu_cycle": v["SQ_INSTS_LDS"] / 256 / cyc,
                    "lds_conflict_cycle_share": v["SQ_LDS_BANK_CONFLICT"] / v["SQ_LDS_IDX_ACTIVE"]}
        except (OSError, KeyError, ZeroDivisionError):
            continue
    return None


def main():
    a = parse()
    N = int(a.n)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DSE_BENCH_REHEARSE=1: rehearsal of the N-rank code path on a 1-GPU box
    # (gloo, every rank on cuda:0); its timings mean nothing.
    rehearse = os.environ.get("DSE_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    P = world  # one spread-work chunk per GPU
    cs = (N - 1) // 2 // P
    g0 = rank * cs
    tail_g, tail_n = P * cs, (N - 1) // 2 - P * cs
    words = (cs + 63) // 64

    ctx = S.Context(device=local)
    limit = S.base_limit_for_range(0, P * cs + tail_n)
    tbytes = S.base_table_bytes(limit)
    pbytes = S.base_table_prime_bytes(limit)  # the primes: all a broadcast needs to carry
    table = torch.empty(tbytes, dtype=torch.uint8, device=dev)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    mask = None if a.no_mask else torch.empty(words, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]

    def step(i=None):
        counts.zero_()
        if rank == 0:
            ctx.base_primes_dev_async(limit, table.data_ptr(), tbytes, sp)
        if world > 1:
            dist.broadcast(table[:pbytes], src=0)
            if rank != 0:
                ctx.base_table_finish_dev_async(limit, table.data_ptr(), tbytes, sp)
        if i is not None:
            ev[i][0].record(stream)
        ctx.sieve_range_dev_async(table.data_ptr(), g0, cs, mask.data_ptr() if mask is not None else 0,
                                  counts.data_ptr(), sp)
        if i is not None:
            ev[i][1].record(stream)
        if rank == world - 1 and tail_n:
            ctx.sieve_range_dev_async(table.data_ptr(), tail_g, tail_n, 0, counts.data_ptr() + 8, sp)
        if world > 1:
            dist.all_reduce(counts)

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    g0_ev, g1_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    g0_ev.record(stream)
    for i in range(a.steps):
        step(i)
    g1_ev.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    kern = sum(e0.elapsed_time(e1) for e0, e1 in ev) / a.steps / 1e3  # s per sieve launch
    kern_t = torch.tensor([kern], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(kern_t, op=dist.ReduceOp.MAX)
    c = counts.cpu().tolist()
    pi_ref, pi_full = 1 + c[0], 1 + c[0] + c[1]
    T = elapsed.item()
    if rank == 0:
        rf = work.roofline(g0, cs, kern_t.item())
        pmc = pmc_summary(N, P) if not a.no_mask else None
        out = {
            "metric": METRIC,
            "value": N * a.steps / T,
            "unit": "integers/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": T / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "deterministic (sieve of [3, N]; no input data)",
            "config": {"workload": f"N={N:.0e} odd-only chunked sieve, P={P} spread-work chunks (one per GPU), "
                                   "mask resident in HBM" + (" [count-only diagnostic]" if a.no_mask else ""),
                       "N": N, "P": P, "cs": cs, "mask_bytes_per_gpu": 0 if a.no_mask else words * 8,
                       "parallelism": f"range-partition x{P} (RCCL broadcast + all-reduce)"},
            "ms_per_step_gpu": g0_ev.elapsed_time(g1_ev) / a.steps,
            "pi_ref": pi_ref,
            "pi_full": pi_full,
            "verified": KNOWN_PI.get(N) == pi_full if N in KNOWN_PI else None,
            "roofline": {"bound": rf["bound"],
                         "achieved": rf["lds_achieved_gbs"] if rf["bound"] == "lds" else rf["hbm_achieved_gbs"],
                         "peak": work.LDS_PEAK_GBS if rf["bound"] == "lds" else work.HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": rf["frac"], "traffic": pmc["traffic"] if pmc else None,
                         "pmc_source": pmc["source"] if pmc else None,
                         "wheel_marks_per_launch": rf["wheel_marks"], "frac_executed": rf["frac_executed"],
                         "valu_issue_per_cu_cycle": pmc["valu_issue_per_cu_cycle"] if pmc else None,
                         "lds_issue_per_cu_cycle": pmc["lds_issue_per_cu_cycle"] if pmc else None,
                         "lds_conflict_cycle_share": pmc["lds_conflict_cycle_share"] if pmc else None,
                         "kernel": "wheel_segments_kernel", "kernel_ms": kern_t.item() * 1e3,
                         "marks_per_launch": rf["marks"], "bytes_per_mark": work.BYTES_PER_MARK,
                         "hbm_bytes_per_launch": rf["hbm_bytes"], "hbm_achieved": rf["hbm_achieved_gbs"],
                         "hbm_peak": work.HBM_PEAK_GBS},
            "cpu_baseline": None,
        }
        if world == 1 and a.cpu_baseline == "on":
            out["cpu_baseline"] = cpu_baseline(int(a.cpu_sample_n))
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

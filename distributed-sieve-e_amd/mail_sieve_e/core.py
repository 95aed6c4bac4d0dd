"""Mirror of mail-sieve-e.core (/root/reference/src/mail_sieve_e/core.clj).

The reference's roles stay the drop-in surface:
  lead-start  [num-expected num-primes port]  (core.clj:136-179) -> lead_start
  client-start [host port]                    (core.clj:181-205) -> client_start
  -main, arity 3 = lead, arity 2 = follower    (core.clj:207-212) -> main

What changes underneath:
  - the TCP star + EDN lines (core.clj:13-104) become a torch.distributed
    TCPStore rendezvous on the same host:port plus one process group
    (RCCL over xGMI on GPUs);
  - machine numbers are still handed out in arrival order, lead = 1,
    followers 2..P (core.clj:155-159);
  - the lead still computes the spread-work bounds; every machine reads its
    own (core.clj:151,160);
  - the per-prime [mi ps p] relay and the appoint hand-off (sieve.clj:139,148;
    core.clj:118-134) become ONE broadcast of the base-prime table from the
    lead, after which every machine sieves its chunk concurrently;
  - the counts are all-reduced (the reference never computes pi);
  - each machine writes its own primes{k}.txt via finish (sieve.clj:97-105);
  - the kill signal (core.clj:171, 199-200) is a final barrier.
"""
from __future__ import annotations

import datetime
import os
import sys
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import sieve as S

KEY_N, KEY_P, KEY_JOINED = "dse/num-primes", "dse/num-comps", "dse/joined"


class GpuEngine:
    """The product engine: libdse.so on this machine's GPU, tensors on device."""

    backend = "nccl"

    def __init__(self, my_num: int):
        import torch
        ndev = torch.cuda.device_count()
        if ndev < 1:
            raise RuntimeError("no GPU visible: the HIP engine is required (no CPU fallback)")
        self.torch = torch
        # one process per GPU: the node-local index comes from DSE_DEVICE or
        # LOCAL_RANK when a launcher sets them (needed when machines of several
        # nodes join in arbitrary order), else from the machine number
        local = os.environ.get("DSE_DEVICE", os.environ.get("LOCAL_RANK"))
        self.device = torch.device("cuda", int(local) % ndev if local is not None else (my_num - 1) % ndev)
        torch.cuda.set_device(self.device)
        self.ctx = S.Context(device=self.device.index)

    def new_table(self, limit: int):
        return self.torch.empty(S.base_table_bytes(limit), dtype=self.torch.uint8, device=self.device)

    def build_table(self, limit: int, table) -> None:
        sp = self.torch.cuda.current_stream(self.device).cuda_stream
        self.ctx.base_primes_dev_async(limit, table.data_ptr(), table.numel(), sp)

    def table_primes(self, limit: int, table):
        """The part of the table a broadcast carries: header + primes."""
        return table[: S.base_table_prime_bytes(limit)]

    def finish_table(self, limit: int, table) -> None:
        sp = self.torch.cuda.current_stream(self.device).cuda_stream
        self.ctx.base_table_finish_dev_async(limit, table.data_ptr(), table.numel(), sp)

    def new_counts(self):
        return self.torch.zeros(2, dtype=self.torch.int64, device=self.device)

    def sieve(self, table, g_start: int, nbits: int, counts, slot: int, want_mask: bool):
        t = self.torch
        sp = t.cuda.current_stream(self.device).cuda_stream
        mask = t.empty((nbits + 63) // 64, dtype=t.int64, device=self.device) if want_mask else None
        self.ctx.sieve_range_dev_async(table.data_ptr(), g_start, nbits,
                                       mask.data_ptr() if mask is not None else 0,
                                       counts.data_ptr() + 8 * slot, sp)
        return mask

    def to_host_mask(self, mask) -> np.ndarray:
        return mask.cpu().numpy().view(np.uint64)

    def close(self):
        self.ctx.close()


@dataclass
class MachineResult:
    my_num: int
    num_comps: int
    bounds: tuple
    count: int
    pi_ref: int
    pi_full: int
    path: Optional[str]


def _run_machine(store, my_num: int, num_comps: int, num_primes: int, engine, out_dir: Optional[str],
                 write_file: bool = True) -> MachineResult:
    import torch.distributed as dist
    P, n = num_comps, num_primes
    rank = my_num - 1
    dist.init_process_group(engine.backend, store=dist.PrefixStore("dse-pg", store), rank=rank, world_size=P,
                            timeout=datetime.timedelta(seconds=600))
    try:
        bounds = S.spread_work(n, P)[rank]                  # core.clj:151,157,160
        chunk = S.gen_table(bounds)                          # core.clj:152,192
        if chunk.cs < 4:
            raise ValueError("chunks of < 4 candidates break finish's 2/3/5/7 hack (sieve.clj:93-96)")
        tail_g, tail_n = S.tail_range(n, P)
        limit = S.base_limit_for_range(0, P * chunk.cs + tail_n)
        table = engine.new_table(limit)
        if rank == 0:
            engine.build_table(limit, table)                 # replaces per-prime sends (sieve.clj:139)
        if P > 1:
            dist.broadcast(engine.table_primes(limit, table), src=0)  # replaces the lead's relay (core.clj:118-134)
            if rank != 0:
                engine.finish_table(limit, table)
        counts = engine.new_counts()
        mask = engine.sieve(table, chunk.g_start, chunk.cs, counts, 0, want_mask=True)
        if rank == P - 1 and tail_n:
            engine.sieve(table, tail_g, tail_n, counts, 1, want_mask=False)
        own = int(counts[0].item())
        if P > 1:
            dist.all_reduce(counts)
        total, tail = (int(x) for x in counts.cpu().tolist())
        chunk.mask, chunk.n_primes = engine.to_host_mask(mask), own
        path = None
        if write_file:
            path = os.path.join(out_dir or os.path.expanduser("~"), f"primes{my_num}.txt")
            S.finish(chunk, my_num, path=path)              # sieve.clj:150
        if P > 1:
            dist.barrier()                                   # kill signal (core.clj:171, 199-200)
        return MachineResult(my_num, P, tuple(bounds), own, 1 + total, 1 + total + tail, path)
    finally:
        dist.destroy_process_group()


def lead_start(num_expected: int, num_primes: int, port: int, *, host: str = "127.0.0.1",
               out_dir: Optional[str] = None, engine_factory=GpuEngine, write_file: bool = True,
               timeout_s: float = 600.0) -> MachineResult:
    """core.clj:136-179: serve on port, wait for num_expected-1 followers,
    hand out machine numbers and bounds, run machine 1, wait, shut down."""
    from torch.distributed import TCPStore
    store = TCPStore(host, port, world_size=None, is_master=True, wait_for_workers=False,
                     timeout=datetime.timedelta(seconds=timeout_s))
    store.set(KEY_N, str(num_primes))
    store.set(KEY_P, str(num_expected))
    print("Waiting for computers to join...", flush=True)   # core.clj:112
    engine = engine_factory(1)
    try:
        return _run_machine(store, 1, num_expected, num_primes, engine, out_dir, write_file)
    finally:
        engine.close()
        print("Sieve completed!", flush=True)               # core.clj:179


def client_start(host: str, port: int, *, out_dir: Optional[str] = None, engine_factory=GpuEngine,
                 write_file: bool = True, timeout_s: float = 600.0) -> MachineResult:
    """core.clj:181-205: connect, receive machine number and bounds, sieve,
    finish, wait for the kill signal."""
    from torch.distributed import TCPStore
    print("connecting to host...", flush=True)              # core.clj:184
    store = TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=timeout_s))
    my_num = int(store.add(KEY_JOINED, 1)) + 1              # (+ mi 2), arrival order
    num_primes, num_comps = int(store.get(KEY_N)), int(store.get(KEY_P))
    if my_num > num_comps:
        raise RuntimeError(f"machine {my_num} joined but the lead expects {num_comps}")
    engine = engine_factory(my_num)
    try:
        return _run_machine(store, my_num, num_comps, num_primes, engine, out_dir, write_file)
    finally:
        engine.close()
        print("Done!", flush=True)                          # core.clj:205


def main(argv=None) -> int:
    """core.clj:207-212 -main: 3 args = lead (num-comps num-primes port),
    2 args = follower (host port)."""
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) == 3:
        r = lead_start(int(argv[0]), int(argv[1]), int(argv[2]))
    elif len(argv) == 2:
        r = client_start(argv[0], int(argv[1]))
    else:
        print("usage: lead: <num-comps> <num-primes> <port> | follower: <host> <port>", file=sys.stderr)
        return 2
    print(f"machine {r.my_num}: {r.count} odd primes in {list(r.bounds)}; pi_ref={r.pi_ref} pi_full={r.pi_full}",
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""TEST INFRASTRUCTURE ONLY -- the reference's machines on the wire, in Python.

A CPU restatement of the reference lead and follower as they behave on the
socket (/root/reference/src/mail_sieve_e/core.clj:13-212 and
sieve.clj:36-172): they mark their chunks from the [mi ps p] lines they
receive, exactly as the reference does (early-indices skip included), so
tests can mix them with mail_sieve_e.wire's GPU machines and check that each
side's lines let the other sieve correctly. Pure-Python loops: small n only.
Only tests/ import this module.
"""
from __future__ import annotations

import math
import queue
import socket
import threading
from typing import List, Optional


def spread_work(n: int, P: int):
    """sieve.clj:15-34 in Doubles, as the reference computes it."""
    nums = math.floor((n - 1) / 2)
    cs = math.floor(nums / P)
    return [[3.0 if k == 0 else float(3 + 2 * k * cs), float(3 + 2 * (k + 1) * cs)] for k in range(P)]


def mark_composites(mi: int, cs: int, ps: int, p: int, my_num: int, coll: bytearray) -> None:
    """sieve.clj:47-71 (see oracle/dse_oracle.c ref_mark_composites)."""
    early = (my_num - 1) * math.floor((cs - ps) / p)           # :56, a Double there
    ndrop = early - 1
    first_i = 1 + (math.ceil(ndrop) if ndrop > 0 else 0)       # :57 (drop (dec early) ...)
    k = ps + cs * (mi - 1)                                     # :43 indices
    lower, upper = (my_num - 1) * cs, my_num * cs - 1          # :58-59
    head = k + first_i * p
    if head < lower:                                           # skip to the chunk (same marks)
        head += ((lower - head + p - 1) // p) * p
    for h in range(head, upper + 1, p):                        # :60-67
        coll[h % cs] = 0


def find_next_non_zero(coll, start: int, cs: int) -> Optional[int]:
    """sieve.clj:73-80: returns cs at the chunk's end, None only when start >= cs."""
    for stop in range(start + 1, cs + 1):
        if stop == cs or coll[stop] != 0:
            return stop
    return None


def _double(v: float) -> str:
    """Double.toString of an integer-valued Double (as dse_oracle.c java_double_str)."""
    d = str(int(v))
    if int(v) < 10**7:
        return d + ".0"
    m = d.rstrip("0")
    return f"{m[0]}.{m[1:] or '0'}E{len(d) - 1}"


class _Lines:
    """read-handler (core.clj:46-58): a thread drains the socket into a
    channel, skipping empty lines; write (core.clj:40-44) under a lock."""

    def __init__(self, sock):
        self.sock, self.lock, self.q = sock, threading.Lock(), queue.Queue()
        threading.Thread(target=self._drain, daemon=True).start()

    def _drain(self):
        try:
            for raw in self.sock.makefile("rb"):
                s = raw.decode().strip()
                if s:
                    self.q.put(s)
        except OSError:
            pass
        self.q.put(None)

    def line(self, timeout: Optional[float] = 120):
        return self.q.get(timeout=timeout)

    def read(self):
        """read-string of the next line; "EOF" when the socket closed."""
        s = self.line()
        if s is None:
            return "EOF"
        if s.startswith("["):
            return [float(t) if ("." in t or "E" in t) else int(t) for t in s[1:-1].split()]
        return None if s == "nil" else (float(s) if "." in s else int(s))

    def write(self, msg: str) -> None:                          # core.clj:40-44
        with self.lock:
            self.sock.sendall((msg + "\n").encode())


def lead_body(my_num: int, chunk: List, coll: bytearray, cs: int, out) -> None:
    """sieve.clj:131-150 (lead branch): for every survivor, send [my-num start
    prime] and mark; then appoint [my-num -1 0]. chunk holds the values
    (Doubles for machine 1), coll the zeroed flags."""
    start = 0 if coll[0] else find_next_non_zero(coll, -1, cs)
    while True:
        n_start = find_next_non_zero(coll, start, cs)
        if n_start is None:
            break
        prime = chunk[start]
        out(f"[{my_num} {start} {_double(prime) if my_num == 1 else int(prime)}]")
        mark_composites(my_num, cs, start, int(prime), my_num, coll)
        start = n_start
    out(f"[{my_num} -1 0]")


def ref_client(host: str, port: int, result: dict) -> None:
    """core.clj:181-205 client-start + the follower branch of sieve-e
    (sieve.clj:152-172). result gets my_num, lower, cs and the flags."""
    sock = socket.create_connection((host, port), timeout=60)
    ln = _Lines(sock)
    my_num = int(ln.read())
    lo, hi = (int(x) for x in ln.read())                       # (mapv int bounds)
    ln.read()                                                  # start signal
    chunk = list(range(lo, hi, 2))
    cs = len(chunk)
    coll = bytearray(b"\x01") * cs
    while True:
        msg = ln.read()
        if msg == "EOF":
            raise RuntimeError("lead closed")
        mi, ps, p = (int(x) for x in msg)                      # (mapv int ...)
        if ps != -1:
            mark_composites(mi, cs, ps, p, my_num, coll)
        elif mi == my_num - 1:
            lead_body(my_num, chunk, coll, cs, ln.write)
            break
    while ln.read() not in (0, "EOF"):                         # kill signal
        pass
    sock.close()
    result.update(my_num=my_num, lower=lo, cs=cs, flags=bytes(coll))


def ref_lead(num_expected: int, n: int, srv: socket.socket, result: dict,
             accepted: Optional[threading.Semaphore] = None) -> None:
    """core.clj:136-179 lead-start on an already-listening socket: hand out
    numbers and bounds, lead with chunk 1, relay [mi ps p] to connections
    (drop (dec mi)) and answer each with the handler's nil (an empty line),
    stop at the appoint from machine P, send 0."""
    P = num_expected
    conns = []
    while len(conns) < P - 1:
        s, _ = srv.accept()
        conns.append(_Lines(s))
        if accepted is not None:
            accepted.release()
    chunks = spread_work(n, P)
    for mi, c in enumerate(conns):
        c.write(str(mi + 2))
        c.write(f"[{_double(chunks[mi + 1][0])} {_double(chunks[mi + 1][1])}]")
        c.write("1")
    done = threading.Event()

    def relay(src: _Lines):
        while True:
            s = src.line(None)
            if s is None:
                return
            mi, ps, _ = (int(float(t)) for t in s[1:-1].split())
            for dst in conns[mi - 1:]:
                dst.write(s)
            src.write("")                                      # (write sock nil)
            if ps == -1 and mi == P:
                done.set()

    for c in conns:
        threading.Thread(target=relay, args=(c,), daemon=True).start()
    lo, hi = chunks[0]
    chunk = [lo + 2.0 * j for j in range(len(range(int(lo), int(hi), 2)))]
    cs = len(chunk)
    coll = bytearray(b"\x01") * cs

    def bcast(msg):
        for c in conns:
            c.write(msg)
    lead_body(1, chunk, coll, cs, bcast)
    if P > 1:
        done.wait(120)
    for c in conns:
        c.write("0")
        c.sock.close()
    result.update(my_num=1, lower=3, cs=cs, flags=bytes(coll))

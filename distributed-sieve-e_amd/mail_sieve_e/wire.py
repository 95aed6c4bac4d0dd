"""Wire-compatible lead and follower for the reference's TCP/EDN protocol.

core.py replaces the reference's socket star with a torch.distributed
rendezvous; that is faster but cannot talk to a reference JVM machine. This
module speaks the reference protocol itself (core.clj:13-205, sieve.clj:118-172),
so a GPU machine can join a ring of reference machines, or lead one:

  lead -> follower, per follower in arrival order (core.clj:160-166):
      "<machine-number>"        Long, 2..P
      "[<lo> <hi>]"             spread-work bounds as Doubles ("[5001.0 9999.0]")
      "1"                       start signal
  machine m while it leads (sieve.clj:131-150), one line per survivor of its chunk:
      "[m j prime]"             j = index in chunk m, prime = its value (Double for m = 1)
      "[m -1 0]"                appoint machine m+1
  lead relay (core.clj:118-134): a line from machine m goes to machines > m;
      the appoint from machine P ends the run
  lead -> all: "0"              kill signal (core.clj:171)

What differs from the reference machine: each GPU machine sieves its whole
chunk on the device as soon as it has its bounds (primes <= sqrt(hi) are
computed on the device, so the incoming [mi ps p] lines are read and dropped,
not marked). The outgoing lines are exactly the reference's, so reference
machines numbered above a GPU machine mark from them as before.
"""
from __future__ import annotations

import os
import queue
import socket
import threading
from typing import Callable, List, Optional, Tuple

import numpy as np

from . import sieve as S

# ---------------------------------------------------------------- EDN lines


def _atom(tok: str):
    if tok == "nil":
        return None
    if tok in ("true", "false"):
        return tok == "true"
    try:
        return int(tok)
    except ValueError:
        return float(tok)


def parse_line(line: str):
    """read-string on one protocol line (core.clj:54): a number, nil/true, or
    a flat vector of numbers. Empty lines are skipped by the reference
    (core.clj:53) and return None here."""
    s = line.strip()
    if not s:
        return None
    if s[0] == "[":
        if s[-1] != "]":
            raise ValueError(f"unterminated vector: {line!r}")
        return [_atom(t) for t in s[1:-1].replace(",", " ").split()]
    return _atom(s)


def java_double_str(v) -> str:
    """Double.toString as Clojure's str prints it: plain "d.d" for
    1e-3 <= |v| < 1e7, computerized scientific "d.dddE<n>" otherwise."""
    f = float(v)
    if f == 0.0:
        return "0.0"
    sign = "-" if f < 0 else ""
    f = abs(f)
    r = repr(f)                                   # shortest round-trip digits
    mant, _, exp = r.partition("e")
    ip, _, fp = mant.partition(".")
    e10 = int(exp) if exp else 0
    if f < 1e-3:
        raise ValueError("only values >= 1e-3 occur on the wire")
    if f < 1e7:                                   # repr is plain "d.d" in this range
        return f"{sign}{ip}.{fp or '0'}"
    digits = (ip + fp).rstrip("0")                # ip has no leading zero for f >= 1
    point = len(ip) - 1 + e10
    return f"{sign}{digits[0]}.{digits[1:] or '0'}E{point}"


def format_bounds(bounds) -> str:
    """str of spread-work's [head tail] pair of Doubles (sieve.clj:24-34)."""
    return f"[{java_double_str(bounds[0])} {java_double_str(bounds[1])}]"


def prime_lines(my_num: int, chunk: S.Chunk) -> bytes:
    """The lines machine my_num sends while it leads (sieve.clj:131-146): one
    [my-num start prime] per survivor in chunk order, then the appoint
    [my-num -1 0] (sieve.clj:148). Chunk 1 holds Doubles (spread-work's 3.0
    head), later chunks Longs (client-start's (mapv int bounds))."""
    if chunk.mask is None:
        raise ValueError("chunk not sieved")
    bits = np.unpackbits(chunk.mask.view(np.uint8), bitorder="little")[: chunk.cs]
    idx = np.flatnonzero(bits)
    vals = chunk.lower + 2 * idx
    if my_num == 1:
        body = [f"[1 {j} {java_double_str(v)}]" for j, v in zip(idx.tolist(), vals.tolist())]
    else:
        body = [f"[{my_num} {j} {v}]" for j, v in zip(idx.tolist(), vals.tolist())]
    body.append(f"[{my_num} -1 0]")
    return ("\n".join(body) + "\n").encode()


class LineChannel:
    """One protocol socket: a reader thread drains it into a queue (the
    reference's read-handler, core.clj:46-58) so the peer never blocks on a
    full TCP buffer; writes are whole lines under a lock (core.clj:40-44)."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.q: "queue.Queue" = queue.Queue()
        self._wlock = threading.Lock()
        self._t = threading.Thread(target=self._read, daemon=True)
        self._t.start()

    _EOF = object()

    def _read(self):
        f = self.sock.makefile("rb")
        try:
            for raw in f:
                line = raw.decode().strip()
                if line:
                    self.q.put(line)
        except OSError:
            pass
        finally:
            self.q.put(self._EOF)

    def get_line(self, timeout: Optional[float] = None) -> Optional[str]:
        """Next non-empty line, None at end of stream. timeout=None waits
        forever, as the reference does (core.clj:54, sieve.clj:156); a finite
        timeout that expires raises RuntimeError."""
        try:
            line = self.q.get(timeout=timeout)
        except queue.Empty:
            raise RuntimeError(f"no protocol line from the peer within {timeout} s") from None
        if line is self._EOF:
            self.q.put(self._EOF)
            return None
        return line

    def get(self, timeout: Optional[float] = None):
        """Next parsed message, None at end of stream (read-string, core.clj:54)."""
        while True:
            line = self.get_line(timeout)
            if line is None:
                return None
            msg = parse_line(line)
            if msg is not None:
                return msg

    def send(self, data) -> None:
        if isinstance(data, str):
            data = (data + "\n").encode()
        with self._wlock:
            self.sock.sendall(data)

    def close(self) -> None:
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()


# --------------------------------------------------------------- the engine

SieveFn = Callable[[int, int], Tuple[np.ndarray, int]]


def gpu_sieve_fn(device: int = 0) -> Tuple[SieveFn, Callable[[], None]]:
    """The product engine: libdse's wheel path on one GPU. Raises when no GPU
    or no libdse.so is present (no CPU fallback)."""
    ctx = S.Context(device=device)

    def fn(g_start: int, nbits: int):
        return ctx.sieve_odd_range(g_start, nbits, want_mask=True)
    return fn, ctx.close


def _sieve_chunk(chunk: S.Chunk, sieve_fn: SieveFn) -> S.Chunk:
    if chunk.cs < 1:
        raise ValueError("empty chunk (find-first-prime would throw, sieve.clj:113)")
    mask, count = sieve_fn(chunk.g_start, chunk.cs)
    chunk.mask, chunk.n_primes = np.ascontiguousarray(mask, dtype=np.uint64), int(count)
    return chunk


def _out_path(out_dir: Optional[str], my_num: int) -> str:
    return os.path.join(out_dir or os.path.expanduser("~"), f"primes{my_num}.txt")


# ------------------------------------------------------------------ follower


def _expect(ch: LineChannel, what: str, timeout_s: Optional[float]):
    msg = ch.get(timeout_s)
    if msg is None:
        raise RuntimeError(f"lead closed the connection before sending {what}")
    return msg


def client_start(host: str, port: int, *, out_dir: Optional[str] = None, sieve_fn: Optional[SieveFn] = None,
                 device: int = 0, timeout_s: Optional[float] = None, write_file: bool = True) -> S.Chunk:
    """core.clj:181-205 client-start, speaking the reference protocol. Like
    the reference, every protocol wait is unbounded by default (a reference
    lead marking prime by prime can take hours); timeout_s bounds them."""
    close = None
    if sieve_fn is None:
        sieve_fn, close = gpu_sieve_fn(device)
    print("connecting to host...", flush=True)
    sock = socket.create_connection((host, port), timeout=timeout_s)
    sock.settimeout(None)  # before the reader starts: a socket timeout there would read as the lead's EOF
    ch = LineChannel(sock)
    try:
        my_num = _expect(ch, "the machine number", timeout_s)   # core.clj:188
        if not isinstance(my_num, int):
            raise RuntimeError(f"expected the machine number, got {my_num!r}")
        bounds = _expect(ch, "the chunk bounds", timeout_s)     # core.clj:189 (mapv int ...)
        if not (isinstance(bounds, list) and len(bounds) == 2):
            raise RuntimeError(f"expected [lo hi] bounds, got {bounds!r}")
        chunk = S.gen_table([int(x) for x in bounds])           # core.clj:190
        start = ch.get(timeout_s)                                 # core.clj:192
        if not start:
            raise RuntimeError("lead closed before the start signal")
        _sieve_chunk(chunk, sieve_fn)                             # the whole chunk, on the GPU
        # sieve.clj:157-172: follow until machine my_num-1 appoints this one.
        while True:
            msg = ch.get(timeout_s)
            if msg is None:
                raise RuntimeError("lead closed before this machine was appointed")
            if isinstance(msg, list) and len(msg) == 3 and int(msg[1]) == -1 and int(msg[0]) == my_num - 1:
                break
        print("Appointed as new lead.\n", flush=True)
        ch.send(prime_lines(my_num, chunk))                       # sieve.clj:139,148
        if write_file:
            S.finish(chunk, my_num, path=_out_path(out_dir, my_num))  # sieve.clj:150
        print("Waiting for kill signal...", flush=True)
        while True:                                               # core.clj:199-200
            msg = ch.get(timeout_s)
            if msg is None or msg == 0:
                break
        return chunk
    finally:
        ch.close()
        if close:
            close()
        print("Done!", flush=True)


# ---------------------------------------------------------------------- lead


def lead_start(num_expected: int, num_primes: int, port: int, *, host: str = "0.0.0.0",
               out_dir: Optional[str] = None, sieve_fn: Optional[SieveFn] = None, device: int = 0,
               timeout_s: Optional[float] = None, write_file: bool = True,
               ready: Optional[threading.Event] = None) -> S.Chunk:
    """core.clj:136-179 lead-start, speaking the reference protocol: accept
    num_expected-1 followers, hand out numbers and bounds, lead with chunk 1,
    relay every follower line to the machines numbered above its sender,
    stop at the appoint from machine P. With P = 1 the reference waits
    forever for an appoint that never comes; here the run ends. Every wait
    (accept, the last appoint) is unbounded by default, as in the reference
    (core.clj:113,165-166); timeout_s bounds them (tests)."""
    P, n = int(num_expected), int(num_primes)
    close = None
    if sieve_fn is None:
        sieve_fn, close = gpu_sieve_fn(device)
    srv = socket.create_server((host, port), reuse_port=False)
    srv.settimeout(timeout_s)
    if ready is not None:
        ready.set()
    conns: List[LineChannel] = []
    try:
        print("Waiting for computers to join...", flush=True)   # core.clj:112
        while len(conns) < P - 1:                                 # arrival order = machine order
            s, _ = srv.accept()
            s.settimeout(None)
            conns.append(LineChannel(s))
        print("# Connected: ", len(conns), flush=True)
        _, chunks = S._spread(n, P)                                # core.clj:151
        lead_chunk = S.gen_table(chunks[0])                        # core.clj:152
        if lead_chunk.cs < 4:
            raise ValueError("chunks of < 4 candidates break finish's 2/3/5/7 hack (sieve.clj:93-96)")
        for mi, c in enumerate(conns):                             # core.clj:154-166
            c.send(f"{mi + 2}\n{format_bounds(chunks[mi + 1])}\n1")

        done = threading.Event()
        errors: List[BaseException] = []
        if P == 1:
            done.set()

        def relay(src: LineChannel):                               # core.clj:118-134
            try:
                while True:
                    line = src.get_line()
                    if line is None:
                        return
                    msg = parse_line(line)
                    if not (isinstance(msg, list) and len(msg) == 3):
                        continue
                    mi, ps = int(msg[0]), int(msg[1])
                    data = (line + "\n").encode()
                    for dst in conns[max(mi - 1, 0):]:
                        dst.send(data)
                    if ps == -1 and mi == P:
                        done.set()
            except BaseException as e:  # noqa: BLE001 - surfaced to the lead thread
                errors.append(e)
                done.set()

        _sieve_chunk(lead_chunk, sieve_fn)                         # sieve.clj:131-146 on the GPU
        lines = prime_lines(1, lead_chunk)
        # Chunk 1's lines reach every follower before any relayed line: the
        # relay threads start only after this broadcast (lines that followers
        # send meanwhile wait in their LineChannel queues), so machine 3 never
        # sees machine 2's lines, or its appoint, ahead of machine 1's primes.
        for c in conns:                                            # send-chan broadcast (core.clj:93)
            c.send(lines)
        threads = [threading.Thread(target=relay, args=(c,), daemon=True) for c in conns]
        for t in threads:
            t.start()
        if write_file:
            S.finish(lead_chunk, 1, path=_out_path(out_dir, 1))    # sieve.clj:150
        print("Waiting for other machines to finish...\n", flush=True)
        if not done.wait(timeout_s):
            raise RuntimeError(f"no appoint from the last machine within {timeout_s} s")
        if errors:
            raise errors[0]
        print("Shutting down server...\n", flush=True)
        for c in conns:                                            # core.clj:171
            c.send("0")
        return lead_chunk
    finally:
        for c in conns:
            c.close()
        srv.close()
        if close:
            close()
        print("Sieve completed!", flush=True)


def main(argv=None) -> int:
    """-main (core.clj:207-212) over the reference wire: 3 args = lead
    (num-comps num-primes port), 2 args = follower (host port). Optional
    --timeout SECONDS bounds every protocol wait (default: wait forever)."""
    import sys
    argv = list(sys.argv[1:] if argv is None else argv)
    usage = "usage: lead: <num-comps> <num-primes> <port> | follower: <host> <port> [--timeout S]"
    timeout_s = None
    if "--timeout" in argv:
        i = argv.index("--timeout")
        try:
            timeout_s = float(argv[i + 1])
            if not timeout_s > 0:
                raise ValueError(argv[i + 1])
        except (IndexError, ValueError):
            print(usage, file=sys.stderr)
            return 2
        del argv[i:i + 2]
    if len(argv) == 3:
        c = lead_start(int(argv[0]), int(argv[1]), int(argv[2]), timeout_s=timeout_s)
        print(f"machine 1: {c.n_primes} odd primes in [{c.lower}, {c.upper})", flush=True)
    elif len(argv) == 2:
        c = client_start(argv[0], int(argv[1]), timeout_s=timeout_s)
        print(f"{c.n_primes} odd primes in [{c.lower}, {c.upper})", flush=True)
    else:
        print(usage, file=sys.stderr)
        return 2
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

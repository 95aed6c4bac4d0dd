"""Debug aid for the wheel kernel: one range, selected phases (DSE_PHASES),
compared with a numpy sieve restricted to the same prime classes.
Phases: 1 = A (61,1024], 2 = B (1024,16384], 4 = L (>16384), 8 = patterns 7..61, 16 = store.
Usage: wheel_debug.py g0 nbits  (runs every phase combination in a subprocess)"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")]
import numpy as np

CLASSES = {1: (61, 1024), 2: (1024, 16384), 4: (16384, 1 << 40)}


def run_one(g0, nb, phases):
    from mail_sieve_e import _dse
    _dse.LIB_PATH = os.environ.get("DSE_LIB", os.path.join(ROOT, "variants", "libdse_knob.so"))  # knob build
    from mail_sieve_e.sieve import Context
    from mail_sieve_e.work import odd_primes_upto
    c = Context(1)
    m, cnt = c.sieve_odd_range(g0, nb)
    bits = np.unpackbits(m.view(np.uint8), bitorder="little")[:nb].astype(bool)
    vals = 3 + 2 * (g0 + np.arange(nb, dtype=np.int64))
    comp = (vals % 3 == 0) & (vals != 3) | (vals % 5 == 0) & (vals != 5)
    for p in odd_primes_upto(int(vals[-1] ** 0.5) + 1):
        if p <= 5:
            continue
        use = (p <= 61 and phases & 8) or any(phases & b and lo < p <= hi for b, (lo, hi) in CLASSES.items())
        if not use:
            continue
        start = max(p * p, ((int(vals[0]) + p - 1) // p) * p) if p > 61 else max(3 * p, ((int(vals[0]) + p - 1) // p) * p)
        if start % 2 == 0:
            start += p
        if start <= vals[-1]:
            comp[(start - int(vals[0])) // 2::p] = True
    ref = ~comp
    bad = np.flatnonzero(bits != ref)
    print(f"phases={phases} nb={nb} gpu_count={cnt} ref_count={int(ref.sum())} bad={bad.size} "
          f"gpu_says_prime={int(bits[bad].sum())} gpu_says_comp={int((~bits[bad]).sum())}", flush=True)
    for b in bad[:8]:
        v = int(vals[b])
        fs = [int(p) for p in odd_primes_upto(5000) if v % p == 0][:3]
        print(f"   bit {b} v {v} v%30={v % 30} factors {fs} gpu {bits[b]}", flush=True)


if __name__ == "__main__":
    g0, nb = int(sys.argv[1]), int(sys.argv[2])
    if len(sys.argv) > 3:
        run_one(g0, nb, int(sys.argv[3]))
        sys.exit(0)
    for ph in (24 | 96, 25 | 96, 26 | 96, 28 | 96, 127):
        env = dict(os.environ, DSE_PHASES=str(ph), DSE_KERNEL="wheel")
        subprocess.run([sys.executable, __file__, str(g0), str(nb), str(ph)], env=env, timeout=120)

"""Profiling aid: compare counts of DSE_CFG variants per phase mask (subprocess per variant)."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = ("import sys; sys.path[:0]=[%r,%r]; from mail_sieve_e.sieve import Context; c=Context(1); "
        "print(c.sieve_odd_range(10**9+7, 3145741, want_mask=False)[1], c.sieve_odd_range(0, 2**19*5+77, want_mask=False)[1])"
        % (ROOT, os.path.join(ROOT, "distributed-sieve-e_amd")))
for ph in [31, 1 | 8 | 16, 2 | 8 | 16, 4 | 8 | 16, 8 | 16, 16]:
    outs = []
    for cfg in ("0", "1"):
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, DSE_CFG=cfg, DSE_PHASES=str(ph)),
                           capture_output=True, text=True, timeout=120)
        outs.append(r.stdout.strip() or r.stderr[-300:])
    print(ph, outs, "SAME" if outs[0] == outs[1] else "DIFF", flush=True)

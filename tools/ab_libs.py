"""A/B of library builds (variants/libdse_<name>.so), each optionally with a
DSE_PHASES mask (knob builds only): `python tools/ab_libs.py name[:phases] ...`.
Interleaved rounds, one bench.py process per run; prints kernel ms. Profiling aid."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = os.environ.get("AB_N", "1e11")
rounds = int(os.environ.get("AB_ROUNDS", "2"))
for rnd in range(rounds):
    for v in sys.argv[1:]:
        name, _, ph = v.partition(":")
        lib = os.path.join(ROOT, "distributed-sieve-e_amd", "mail_sieve_e", "libdse.so") if name == "prod" \
            else os.path.join(ROOT, "variants", f"libdse_{name}.so")
        env = dict(os.environ, DSE_LIB=lib)
        if ph:
            env["DSE_PHASES"] = ph
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "3",
                            "--cpu-baseline", "off", "--n", N], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(v, "FAILED", r.stderr[-400:], flush=True); sys.exit(1)
        j = json.loads(r.stdout.strip().splitlines()[-1])
        print(f"{rnd} {v:24s} kernel_ms={j['roofline']['kernel_ms']:.3f} ok={j['verified']}", flush=True)

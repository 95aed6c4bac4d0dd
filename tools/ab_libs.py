"""A/B of library builds (variants/libdse_<name>.so, or `prod` for the in-tree
library): `python tools/ab_libs.py name ...`. Interleaved rounds, one bench.py
process per run; prints the kernel ms (HIP events) and the step ms. Profiling aid."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = os.environ.get("AB_N", "1e11")
rounds = int(os.environ.get("AB_ROUNDS", "2"))
extra = os.environ.get("AB_ARGS", "").split()
for rnd in range(rounds):
    for name in sys.argv[1:]:
        lib = os.path.join(ROOT, "distributed-sieve-e_amd", "mail_sieve_e", "libdse.so") if name == "prod" \
            else os.path.join(ROOT, "variants", f"libdse_{name}.so")
        env = dict(os.environ, DSE_LIB=lib)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "3",
                            "--cpu-baseline", "off", "--n", N] + extra, env=env, capture_output=True, text=True,
                           timeout=300)
        if r.returncode:
            print(name, "FAILED", r.stderr[-400:], flush=True); sys.exit(1)
        j = json.loads(r.stdout.strip().splitlines()[-1])
        km = j['roofline']['kernel_ms'] if j.get('roofline') else float('nan')
        print(f"{rnd} {name:24s} kernel_ms={km:.3f} step_ms={j['ms_per_step']:.3f} ok={j['verified']}", flush=True)

"""Time the sieve kernel with phases switched off (DSE_PHASES bitmask), one
process per variant is avoided by re-exec-free subprocess runs. Profiling only."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = sys.argv[1] if len(sys.argv) > 1 else "1e11"
variants = {"all": 63, "no_store": 47, "no_small": 55, "only_midA": 1 | 16, "only_midB": 2 | 16,
            "only_coopC": 4 | 16, "only_scatterD": 32 | 16, "only_small": 8 | 16, "only_zero_wb": 16, "nothing": 0}
for name, ph in variants.items():
    env = dict(os.environ, DSE_PHASES=str(ph))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2",
                        "--cpu-baseline", "off", "--n", N], env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(name, "FAILED", r.stderr[-500:]); sys.exit(1)
    j = json.loads(r.stdout.strip().splitlines()[-1])
    print(f"{name:14s} phases={ph:2d} kernel_ms={j['roofline']['kernel_ms']:.3f} step_ms={j['ms_per_step']:.3f}", flush=True)

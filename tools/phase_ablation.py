"""Time the sieve kernel with phases switched off (DSE_PHASES bitmask), one
subprocess per variant. Profiling only. Needs a knob build of the library:
  bash tools/build_variant.sh knob -DDSE_PHASE_KNOB   (-> variants/libdse_knob.so, used via DSE_LIB)"""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = sys.argv[1] if len(sys.argv) > 1 else "1e11"
# wheel kernel phases: 1 = A, 2 = B, 4 = L, 8 = patterns (init), 16 = store, 32 = expand, 64 = unit loop
variants = {"all": 127, "no_store": 111, "only_A": 1 | 120, "only_B": 2 | 120, "only_L": 4 | 120,
            "init_units_expand_store": 120, "init_units_expand": 104, "init_units": 72, "init_expand": 40,
            "init": 8, "nothing": 0, "no_A": 126, "no_B": 125, "no_L": 123, "no_init": 119,
            "no_expand_store": 79}
for name, ph in variants.items():
    env = dict(os.environ, DSE_PHASES=str(ph),
               DSE_LIB=os.environ.get("DSE_LIB", os.path.join(ROOT, "variants", "libdse_knob.so")))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2",
                        "--cpu-baseline", "off", "--n", N], env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(name, "FAILED", r.stderr[-500:]); sys.exit(1)
    j = json.loads(r.stdout.strip().splitlines()[-1])
    print(f"{name:14s} phases={ph:2d} kernel_ms={j['roofline']['kernel_ms']:.3f} step_ms={j['ms_per_step']:.3f}", flush=True)

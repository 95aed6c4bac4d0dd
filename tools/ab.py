"""A/B of env-knob variants, interleaved rounds in separate processes (profiling aid)."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
variants = [dict(kv.split("=", 1) for kv in v.split(",") if kv) for v in sys.argv[1:]] or [{}]
for rnd in range(2):
    for v in variants:
        env = dict(os.environ, **v)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "3",
                            "--cpu-baseline", "off"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(v, "FAILED", r.stderr[-400:]); sys.exit(1)
        j = json.loads(r.stdout.strip().splitlines()[-1])
        print(rnd, v, "kernel_ms=%.3f ok=%s" % (j['roofline']['kernel_ms'], j['verified']), flush=True)

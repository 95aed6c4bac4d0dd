"""bench.py's contract: one JSON line with the BASELINE metric, a roofline and
cpu_baseline object, and pi verified; the N-rank path (broadcast, all-reduce,
max-over-ranks timing) rehearsed with 2 ranks on one GPU over gloo
(DSE_BENCH_REHEARSE=1; the driver's real N-GPU runs use RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _check_line(d: dict, n_gpus: int):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == n_gpus and d["verified"] is True and d["value"] > 0
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-6 * rf["frac"] + 1e-12
    assert 0 < rf["frac"] <= 1
    assert 0 < rf["frac_ds_or"] < rf["frac"] and rf["cycles_per_mark_instr"] > 2.6
    # the world the run formed: one entry per rank
    w = d["world"]
    assert w["size"] == n_gpus and [x["rank"] for x in w["ranks"]] == list(range(n_gpus))
    # every rank's own figures (all-gathered, not only the max), so an N-GPU
    # line can be checked rank by rank; the headline is the max over ranks
    for x in w["ranks"]:
        assert x["step_ms"] > 0 and x["kernel_ms"] > 0 and x["bracketed_ms"] > 0 and x["pipelined_ms"] > 0
        assert x["nbits"] == d["config"]["cs"]
    assert sorted(x["g_start"] for x in w["ranks"]) == [r * d["config"]["cs"] for r in range(n_gpus)]
    assert abs(d["roofline"]["kernel_ms"] - max(x["kernel_ms"] for x in w["ranks"])) < 1e-9 + 1e-9 * d["roofline"]["kernel_ms"]
    # chunk configs broadcast the primes (109 KB at 1e11, the reference's broadcast)
    assert w["base_table"]["path"] == "broadcast" and 0 < w["base_table"]["bytes"] <= 8 << 20
    # the headline is the median of per-step times, each from the call to the counts on the host
    assert d["ms_per_step"] > 0 and d["ms_per_step_bracketed"] > 0 and d["ms_per_step_pipelined"] > 0
    assert abs(d["value"] - d["config"]["N"] / (d["ms_per_step"] / 1e3)) < 1e-6 * d["value"]
    # the line names the library it loaded (the id pmc_build.json records for a profiled build)
    assert d["build"]["libdse"].endswith("libdse.so") and len(d["build"]["libdse_sha256_16"]) == 16


@pytest.mark.gpu
def test_bench_single_gpu_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--n", "1e10", "--steps", "3", "--warmup", "1",
                        "--cpu-baseline", "on", "--cpu-max-n", "1e7"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    _check_line(d, 1)
    cb = d["cpu_baseline"]
    # the reference's lead + 2 followers as threads + the relay thread (P = 3)
    assert cb["cores"] == 4 and cb["value"] > 0 and cb["kind"] == "port"
    assert {(x["N"], x["P"]) for x in cb["runs"]} == {(n, p) for n in (10**4, 10**6, 10**7) for p in (2, 3)}


@pytest.mark.gpu
def test_bench_window_two_rank_rehearsal():
    """--window over 2 ranks on one GPU (gloo): table built on rank 0 and
    broadcast, two slices, count all-reduced == the oracle's window count."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, DSE_BENCH_REHEARSE="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--window", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["verified"] is True and d["pi_full"] == 241272176
    assert d["config"]["P"] == 2 and d["value"] > 0
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and 0 < rf["frac"] <= 1 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    # the window's 203 MB of primes are not broadcast: every rank builds its table
    t = d["world"]["base_table"]
    assert t["path"] == "local" and t["bytes"] > 8 << 20
    assert [x["rank"] for x in d["world"]["ranks"]] == [0, 1] and all(x["kernel_ms"] > 0 for x in d["world"]["ranks"])


@pytest.mark.gpu
def test_bench_window_single_gpu_line():
    """BASELINE config 5 on one GPU: the count verified and an HBM roofline of
    the bucketed pass (8 B per bucket entry, WINDOW_BUCKET_ENTRIES of them)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--window", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    assert d["verified"] is True and d["pi_full"] == 241272176 and d["n_gpus"] == 1
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] <= 1
    assert abs(rf["achieved"] - 8 * 1_208_549_165 / (rf["kernel_ms"] / 1e3) / 1e9) < 1e-6 * rf["achieved"]
    # one rank: nothing to share, the table is built where it is used
    assert d["world"]["base_table"]["path"] == "local"


@pytest.mark.gpu
def test_bench_two_rank_rehearsal():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, DSE_BENCH_REHEARSE="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--N", "1e10", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    _check_line(d, 2)
    assert d["config"]["P"] == 2 and d["pi_full"] == 455052511


@pytest.mark.gpu
def test_bench_single_rank_rccl_line():
    """--rccl-single: the step's dist.broadcast of the primes and dist.all_reduce
    of the counts run through a real 1-rank nccl (RCCL) process group, formed
    by the same init_process_group("nccl", device_id=...) call an N-GPU rank
    makes; pi stays verified and the line names the nccl backend."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--n", "1e10", "--steps", "3", "--warmup", "1",
                        "--cpu-baseline", "off", "--rccl-single"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    _check_line(d, 1)
    assert d["world"]["backend"] == "nccl" and d["world"]["rccl_single"] is True
    assert d["pi_full"] == 455052511


def test_watchdog_names_rank_and_phase():
    """A stuck phase ends the rank with status 3 and its rank, world size and
    phase on stderr (bench.Watchdog), instead of running into the driver's
    time limit. CPU only: no GPU call is made."""
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "w = bench.Watchdog(1, 8, 1.0); w.phase('timed steps'); time.sleep(30)" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "bench.py rank 1/8 in phase 'timed steps': no progress for 1 s" in r.stderr


def test_lib_build_id_is_the_library_sha():
    """bench.lib_build(): the loaded library's path and SHA-256 prefix (CPU only:
    hashing the file, no GPU call)."""
    import hashlib
    sys.path.insert(0, ROOT)
    import bench
    b = bench.lib_build()
    path = os.path.join(ROOT, b["libdse"])
    assert os.path.exists(path)
    assert b["libdse_sha256_16"] == hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]

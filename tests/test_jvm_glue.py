"""JVM drop-in glue: jvm/src/mail_sieve_e/dse.clj binds
include/dse.h through JNA; jvm/dse_replay.c makes the same calls from C
(dse_init -> dse_spread_work -> dse_sieve_chunk -> dse_write_primes_file ->
dse_destroy), the sequence lead-start and client-start would make
(core.clj:151-152,163,192,196; finish at sieve.clj:150). No JDK exists in the
image, so the Clojure file is checked statically and its call sequence is run
through the C replay on the GPU against the golden primes{k}.txt hashes."""
import hashlib
import json
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPLAY = os.path.join(ROOT, "jvm", "dse_replay")
CLJ = os.path.join(ROOT, "jvm", "src", "mail_sieve_e", "dse.clj")
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))


def test_clj_binds_only_declared_symbols():
    header = open(os.path.join(ROOT, "include", "dse.h")).read()
    declared = set(re.findall(r"\b(dse_\w+)\s*\(", header))
    used = set(re.findall(r'\(f "(dse_\w+)"\)', open(CLJ).read()))
    assert used, "no bindings found"
    assert used <= declared, used - declared
    # the replay makes the calls run-machine! makes, in that order
    src = open(os.path.join(ROOT, "jvm", "dse_replay.c")).read()
    body = src[src.index("int main"):]
    order = [m.group(1) for m in re.finditer(r"\b(dse_init|dse_spread_work|dse_sieve_chunk|dse_write_primes_file|"
                                             r"dse_destroy)\(", body)]
    assert order == ["dse_init", "dse_spread_work", "dse_sieve_chunk", "dse_write_primes_file", "dse_destroy"]


def test_replay_built_and_rejects_bad_usage():
    assert os.access(REPLAY, os.X_OK), "jvm/dse_replay not built (make -C jvm, run by __graft_entry__.build)"
    r = subprocess.run([REPLAY, "bogus"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("N,P", [(10_000, 2), (1_000_000, 3)])
def test_replay_files_match_golden(tmp_path, N, P):
    files = {f["my_num"]: f for f in GOLDEN["files"] if f["N"] == N and f["P"] == P}
    assert len(files) == P
    for k in range(1, P + 1):
        args = ["lead", str(N), str(P), str(tmp_path)] if k == 1 else \
               ["client", str(N), str(P), str(k), str(tmp_path)]
        r = subprocess.run([REPLAY] + args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        my_num, count = map(int, r.stdout.split())
        assert my_num == k and count + (1 if k == 1 else 0) == files[k]["nonzero"]
        b = (tmp_path / f"primes{k}.txt").read_bytes()
        assert len(b) == files[k]["bytes"] and hashlib.sha256(b).hexdigest() == files[k]["sha256"], (N, P, k)

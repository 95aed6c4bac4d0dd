"""JVM drop-in glue: jvm/src/mail_sieve_e/dse.clj is a
drop-in for the reference's mail-sieve-e.sieve namespace (spread-work,
gen-table, sieve-e, finish at sieve.clj's arities), so core.clj keeps its
handshake and only swaps its :require (core.clj:6). jvm/dse_replay.c makes
the glue's libdse calls from C in the glue's order (dse_spread_work ->
dse_device_count -> dse_init_device -> dse_sieve_odd_range ->
dse_write_range_file -> dse_destroy) and writes the lead lines the glue puts
on out-channel. No JDK exists in the image, so the Clojure file is checked
statically (read with tests/clj_reader.py) and its call sequence runs through
the C replay on the GPU against the golden primes{k}.txt hashes and the lead
lines of the reference machines restated in oracle/ref_wire.py."""
import hashlib
import json
import os
import re
import subprocess

import pytest

from clj_reader import Form, Str, accepts, defn_arities, read_all, walk

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPLAY = os.path.join(ROOT, "jvm", "dse_replay")
CLJ = os.path.join(ROOT, "jvm", "src", "mail_sieve_e", "dse.clj")
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
CORE_CALLS = json.load(open(os.path.join(ROOT, "tests", "golden", "core_clj_sieve_calls.json")))
REF_CORE = "/root/reference/src/mail_sieve_e/core.clj"  # present in the build container only


def _forms():
    return read_all(open(CLJ).read())


def _header_params():
    """dse_* name -> parameter count, from include/dse.h."""
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "dse.h")).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(dse_\w+)\s*\(([^)]*)\)\s*;", txt):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_clj_reads_and_is_the_namespace():
    forms = _forms()  # raises on unbalanced brackets or an unterminated string
    ns = forms[0]
    assert isinstance(ns, Form) and ns[:2] == ["ns", "mail-sieve-e.dse"]


def test_core_sieve_calls_resolve_at_their_arity():
    """Every s/ call core.clj makes (tests/golden/core_clj_sieve_calls.json:
    spread-work 2 args at :151, gen-table 1 at :152 and :192, sieve-e 5 at
    :163 and :196) and sieve-e's own (finish chunk my-num) resolve to a public
    defn of dse.clj that accepts that many arguments."""
    ar = defn_arities(_forms())
    for c in CORE_CALLS["calls"] + CORE_CALLS["internal"]:
        assert c["name"] in ar, c
        public, arities = ar[c["name"]]
        assert public and accepts(arities, c["args"]), (c, arities)
    assert {c["name"] for c in CORE_CALLS["calls"]} == {"spread-work", "gen-table", "sieve-e"}


def test_core_calls_fixture_matches_reference_source():
    """The committed fixture is what the reference's core.clj holds (checked
    where the reference exists; the GPU box has no /root/reference)."""
    if not os.path.exists(REF_CORE):
        pytest.skip("reference source not present (GPU box)")
    from golden.make_core_calls import sieve_calls
    assert sieve_calls(REF_CORE) == CORE_CALLS["calls"]


def test_clj_binds_declared_symbols_with_their_arity():
    """Every (f "dse_x") the glue invokes names a symbol of include/dse.h and
    passes (object-array [...]) with exactly that function's parameter count."""
    params = _header_params()
    used = 0
    for f in walk(_forms()):
        if not (isinstance(f, Form) and f.kind == "(" and len(f) >= 3 and isinstance(f[0], str)
                and f[0].startswith(".invoke")):
            continue
        target, args = f[1], f[2]
        assert isinstance(target, Form) and target[0] == "f" and isinstance(target[1], Str), f
        name = str(target[1])
        assert name in params, name
        assert isinstance(args, Form) and args[0] == "object-array", f
        n = int(args[1]) if not isinstance(args[1], Form) else len(args[1])
        assert n == params[name], (name, n, params[name])
        used += 1
    assert used >= 7


def test_integration_note_names_only_the_require_swap():
    """The glue's note: the :require swap is the only core.clj edit in the
    reference's range; Long/parseLong and (mapv long ...) only beyond 2^31."""
    head = open(CLJ).read().split("(ns ")[0]
    assert "[mail-sieve-e.sieve :as s]" in head and "[mail-sieve-e.dse :as s]" in head
    assert "and nothing else" in head
    assert "Long/parseLong" in head and "(mapv long" in head


def test_replay_makes_the_glue_calls_in_order():
    src = open(os.path.join(ROOT, "jvm", "dse_replay.c")).read()
    body = src[src.index("int main"):]
    names = ("dse_spread_work", "dse_device_count", "dse_init_device", "dse_sieve_odd_range",
             "dse_write_range_file", "dse_destroy")
    order = [m.group(1) for m in re.finditer(r"\b(" + "|".join(names) + r")\(", body)]
    assert order == list(names)
    # and the glue calls the same entry points
    clj = set(re.findall(r'\(f "(dse_\w+)"\)', open(CLJ).read()))
    assert set(names) <= clj | {"dse_destroy"}


def test_replay_built_and_rejects_bad_usage():
    assert os.access(REPLAY, os.X_OK), "jvm/dse_replay not built (make -C jvm, run by __graft_entry__.build)"
    for args in (["bogus"], ["client", "100", "2", "3", "/tmp"]):
        r = subprocess.run([REPLAY] + args, capture_output=True, text=True, timeout=30)
        assert r.returncode == 2, args


def _reference_lead_lines(N, P):
    """The lines every machine sends while it leads, from the reference
    machines restated in oracle/ref_wire.py run in the race-free order:
    machine m marks its chunk with every earlier lead's [mi ps p] lines
    (sieve.clj:154-166), then leads (sieve.clj:131-148)."""
    from oracle import ref_wire as W
    bounds = W.spread_work(N, P)
    cs = len(range(int(bounds[0][0]), int(bounds[0][1]), 2))
    sent, lines = [], {}
    for m in range(1, P + 1):
        lo, hi = (int(x) for x in bounds[m - 1])
        chunk = [float(v) for v in range(lo, hi, 2)] if m == 1 else list(range(lo, hi, 2))
        coll = bytearray(b"\x01") * cs
        for mi, ps, p in sent:
            W.mark_composites(mi, cs, ps, p, m, coll)
        out = []
        W.lead_body(m, chunk, coll, cs, out.append)
        lines[m] = out
        sent += [tuple(int(float(t)) for t in s[1:-1].split()) for s in out[:-1]]
    return lines


@pytest.mark.gpu
@pytest.mark.parametrize("N,P", [(10_000, 2), (1_000_000, 3)])
def test_replay_files_and_lines_match_reference(tmp_path, N, P):
    files = {f["my_num"]: f for f in GOLDEN["files"] if f["N"] == N and f["P"] == P}
    assert len(files) == P
    want_lines = _reference_lead_lines(N, P)
    for k in range(1, P + 1):
        lines = tmp_path / f"lines{k}.txt"
        args = ["lead", str(N), str(P), str(tmp_path), str(lines)] if k == 1 else \
               ["client", str(N), str(P), str(k), str(tmp_path), str(lines)]
        r = subprocess.run([REPLAY] + args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        my_num, count = map(int, r.stdout.split())
        assert my_num == k and count + (1 if k == 1 else 0) == files[k]["nonzero"]
        b = (tmp_path / f"primes{k}.txt").read_bytes()
        assert len(b) == files[k]["bytes"] and hashlib.sha256(b).hexdigest() == files[k]["sha256"], (N, P, k)
        assert lines.read_text().splitlines() == want_lines[k], (N, P, k)

"""C-ABI boundary (include/dse.h / libdse.so) and the host-side mirror of the
reference interface, on CPU (no GPU compute calls)."""
import hashlib
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dse.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dse_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_survey_abi():
    syms = header_symbols()
    # SURVEY.md 8(b) C ABI the build must export
    for s in ("dse_spread_work", "dse_sieve_chunk", "dse_sieve_all", "dse_sieve_window",
              "dse_write_primes_file", "dse_init", "dse_destroy", "dse_last_error"):
        assert s in syms


def test_library_exports_every_header_symbol():
    from mail_sieve_e import _dse
    L = _dse.lib()
    for s in header_symbols():
        assert hasattr(L, s), f"libdse.so does not export {s}"
        assert s in _dse.SIGNATURES, f"ctypes binding misses {s}"


def test_library_has_gfx950_code():
    from mail_sieve_e import _dse
    blob = open(_dse.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_spread_work_matches_oracle(oracle):
    from mail_sieve_e import sieve as S
    rng = np.random.default_rng(1)
    for _ in range(200):
        n = int(rng.integers(1, 10**13))
        P = int(rng.integers(1, 9))
        cs, bounds = oracle.spread_work(n, P)
        assert S.spread_work(n, P) == [list(b) for b in bounds]
        g, nb = S.tail_range(n, P)
        assert (g, nb) == oracle.tail_range(n, P)
    assert S.spread_work(10_000, 2) == [[3, 5001], [5001, 9999]]


def test_spread_work_rejects_bad_P():
    from mail_sieve_e import _dse
    from mail_sieve_e import sieve as S
    with pytest.raises(_dse.DseError) as e:
        S.spread_work(100, 0)
    assert e.value.code == -1
    assert b"num-comps" in _dse.lib().dse_last_error()


def test_base_limits():
    from mail_sieve_e import _dse
    from mail_sieve_e import sieve as S
    L = _dse.lib()
    assert S.base_limit_for_range(0, (10**11 - 1) // 2) == 316227
    assert S.base_limit_for_range(0, (10**12 - 1) // 2) == 999999
    assert L.dse_base_limit_max() >= 1_000_001
    # table holds pi(1e6) - 1 = 78497 odd primes
    assert S.base_table_bytes(10**6) >= 16 + 12 * 78497


def test_table_broadcast_rule():
    """Chunk configs broadcast the primes (the reference's broadcast,
    sieve.clj:139): 1e11 and 1e12 tables are 109 KB / 314 KB; the 1e18
    window's table (limit 1e9 + 4, 203 MB) is built on every device instead."""
    from mail_sieve_e import sieve as S
    for n in (10**9, 10**10, 10**11, 10**12):
        lim = S.base_limit_for_range(0, (n - 1) // 2)
        assert S.base_table_broadcast_bytes(lim) == S.base_table_prime_bytes(lim) <= 8 << 20
    g = (10**18 + 1 - 3) // 2
    lim = S.base_limit_for_range(g, 10**10 // 2)
    assert lim == 10**9 + 4 and S.base_table_prime_bytes(lim) > 200e6
    assert S.base_table_broadcast_bytes(lim) == 0


def test_no_gpu_init_fails_cleanly():
    from mail_sieve_e import _dse
    L = _dse.lib()
    if L.dse_device_count() > 0:
        pytest.skip("a GPU is visible")
    assert not L.dse_init(1)
    assert b"no HIP device" in L.dse_last_error()


@pytest.mark.parametrize("N,P", [(10_000, 2), (10**6, 3), (2 * 10**7 + 3, 1), (123_457, 5)])
def test_writer_matches_oracle_finish(oracle, tmp_path, N, P):
    """dse_write_primes_file (product) == the oracle's finish (restatement)."""
    from mail_sieve_e import _dse
    cs, masks, _, _ = oracle.sieve(N, P)
    for k in range(P):
        a, b = tmp_path / f"dse{k}.txt", tmp_path / f"ref{k}.txt"
        _dse.check(_dse.lib().dse_write_primes_file(str(a).encode(), k + 1, N, P, _dse.u64p(masks[k])), "write")
        oracle.finish(str(b), k + 1, N, P, masks[k])
        assert a.read_bytes() == b.read_bytes()


def test_writer_survey_hashes(oracle, tmp_path):
    from mail_sieve_e import sieve as S
    cs, masks, _, _ = oracle.sieve(10**6, 3)
    want = ["893331a3af40a499", "7f807e9baa0ff67e", "15254ce843ba8339"]
    for k, (lo, hi) in enumerate(S.spread_work(10**6, 3)):
        ch = S.gen_table([lo, hi])
        ch.mask = masks[k]
        p = S.finish(ch, k + 1, path=str(tmp_path / f"primes{k + 1}.txt"))
        assert hashlib.sha256(open(p, "rb").read()).hexdigest()[:16] == want[k]


def test_writer_rejects_tiny_first_chunk(tmp_path):
    from mail_sieve_e import _dse
    m = np.zeros(1, dtype=np.uint64)
    rc = _dse.lib().dse_write_primes_file(str(tmp_path / "x").encode(), 1, 8, 1, _dse.u64p(m))
    assert rc == -1  # cs = 3 < 4: the 2/3/5/7 hack cannot apply (sieve.clj:93-96)


def test_chunk_primes_and_gen_table(oracle):
    from mail_sieve_e import sieve as S
    cs, masks, _, _ = oracle.sieve(10_000, 2)
    ch = S.gen_table([5001, 9999])
    assert ch.cs == cs == 2499 and ch.g_start == 2499
    ch.mask = masks[1]
    pr = ch.primes()
    assert pr[0] == 5003 and pr[-1] == 9973 and len(pr) == 560
    with pytest.raises(ValueError):
        S.gen_table([4, 10])


def test_product_path_has_no_oracle_dependency():
    """The product (package + library) never imports or links the oracle."""
    pkg = os.path.join(ROOT, "distributed-sieve-e_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")) and "Makefile" not in f:
                txt = open(os.path.join(dirpath, f), errors="replace").read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", txt).replace("no oracle", ""), f
    from mail_sieve_e import _dse
    assert b"liboracle" not in open(_dse.LIB_PATH, "rb").read()

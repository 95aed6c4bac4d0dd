"""Parity of the HIP path (libdse.so on an MI355X) with the oracle.

Small sizes: bit-exact masks/counts/files against the oracle's faithful
restatement of sieve.clj (golden fixtures in tests/golden/golden.json and
live oracle calls). Full sizes (1e9..1e12): mask SHA-256 against golden
fixtures, published pi(10^k), and size-independent properties (chunk masks
concatenate to the P=1 mask; P does not change pi_ref + tail).
"""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def test_golden_sweep_bit_exact(ctx):
    """120 seeded (N, P) cases (seed 0x5EED, N in [20, 1e7], P in 1..8)."""
    for case in GOLDEN["sweep"]:
        N, P = case["N"], case["P"]
        for k in range(P):
            m, c = ctx.sieve_chunk(N, P, k + 1)
            assert c == case["counts"][k], (N, P, k + 1)
            assert sha(m) == case["mask_sha256"][k], (N, P, k + 1)


def test_live_oracle_random_chunks(ctx, oracle):
    rng = np.random.default_rng(0x5EED + 1)
    for _ in range(40):
        N = int(rng.integers(20, 3_000_000))
        P = int(rng.integers(1, 9))
        cs, _ = oracle.spread_work(N, P)
        if cs < 1:
            continue
        _, masks, counts, _ = oracle.sieve(N, P)
        counts_all, pi_ref, pi_full = ctx.sieve_all(N, P)
        assert [int(x) for x in counts_all] == [int(x) for x in counts]
        assert pi_ref == oracle.pi_ref(counts)
        for k in range(P):
            assert np.array_equal(ctx.copy_chunk_mask(N, P, k + 1), masks[k]), (N, P, k)


@pytest.mark.parametrize("g0,nb", [(0, 1), (0, 2), (0, 3), (0, 31), (0, 32), (0, 33), (0, 63), (0, 64),
                                   (0, 65), (0, 127), (0, 128), (0, 129), (5, 7), (29, 70), (31, 1000),
                                   (2**20 - 3, 7), (2**20 - 64, 2**20 + 128), (10**6, 3 * 2**20 + 17),
                                   (123456789, 2**21 - 1), (49_999_999_000, 999)])
def test_ragged_ranges(ctx, oracle, g0, nb):
    """Unaligned starts/lengths, partial words and segments, the small-prime
    self-bits near index 0, p^2 crossing segment boundaries."""
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    m, c = ctx.sieve_odd_range(g0, nb)
    assert c == c_ref
    assert np.array_equal(m, m_ref)


def test_counts_every_start_residue(ctx, oracle):
    """Every odd residue of the range's first value mod 30 (it fixes the plane
    order and the e bits), over more than two segments with a ragged end:
    masks and counts against the oracle. The kernel counts a whole block from
    its raw image words (256 minus the composite bits, expand_segment) and
    only the range's first block and its end from the output words, so a
    block whose bits did not map one-to-one would change the count here."""
    for r in range(15):
        g0 = 10**9 + r
        nb = 2 * 15 * 2**17 + 777 + 31 * r
        m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
        m, c = ctx.sieve_odd_range(g0, nb)
        assert c == c_ref and np.array_equal(m, m_ref), r


def test_random_ranges(ctx, oracle):
    rng = np.random.default_rng(11)
    for _ in range(25):
        g0 = int(rng.integers(0, 5 * 10**10))
        nb = int(rng.integers(1, 5 * 2**20))
        m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
        m, c = ctx.sieve_odd_range(g0, nb)
        assert c == c_ref and np.array_equal(m, m_ref), (g0, nb)


def test_files_byte_exact(ctx, tmp_path):
    from mail_sieve_e import sieve as S
    for f in GOLDEN["files"]:
        N, P, k = f["N"], f["P"], f["my_num"]
        ch = S.gen_table(S.spread_work(N, P)[k - 1])
        S.sieve_e(k, k == 1, None, ch, None, ctx=ctx, path=str(tmp_path / f"primes{k}.txt"))
        b = (tmp_path / f"primes{k}.txt").read_bytes()
        assert (len(b), b.count(b"\n"), hashlib.sha256(b).hexdigest()) == (f["bytes"], f["lines"], f["sha256"])


def test_1e9_mask_golden(ctx):
    g = GOLDEN["big"]["1e9_P1"]
    m, c = ctx.sieve_chunk(g["N"], 1, 1)
    assert c + 1 == g["pi_ref"] == 50_847_534
    assert sha(m) == g["mask_sha256"][0]


@pytest.mark.parametrize("P", [2, 4, 8])
def test_1e10_chunks_golden(ctx, P):
    g = GOLDEN["big"][f"1e10_P{P}"]
    counts, pi_ref, pi_full = ctx.sieve_all(10**10, P)
    assert [int(x) for x in counts] == g["counts"]
    assert pi_ref == pi_full == 455_052_511
    for k in range(P):
        assert sha(ctx.copy_chunk_mask(10**10, P, k + 1)) == g["mask_sha256"][k]


def test_chunks_concatenate_to_single_chunk(ctx):
    """Size-independent property: the P chunk masks, laid end to end, are the
    first P*cs bits of the P=1 mask (N=1e10 with P=8: cs is not a multiple of 64)."""
    N, P = 10**10, 8
    full, _ = ctx.sieve_chunk(N, 1, 1)
    bits_full = np.unpackbits(full.view(np.uint8), bitorder="little")
    ctx.sieve_all(N, P)
    cs = (N - 1) // 2 // P
    for k in range(P):
        mk = ctx.copy_chunk_mask(N, P, k + 1)
        bk = np.unpackbits(mk.view(np.uint8), bitorder="little")
        assert np.array_equal(bk[:cs], bits_full[k * cs:(k + 1) * cs])
        assert not bk[cs:].any()  # tail bits of the last word are zero


def _chunk_sha_resident(ctx, N, P, k):
    """SHA-256 of chunk k's resident mask (dse_copy_chunk_mask): one host copy
    (up to 7.8 GB at 1e12 P=8), hashed in place through its buffer, no second
    copy."""
    m = ctx.copy_chunk_mask(N, P, k)
    h = hashlib.sha256(memoryview(m).cast("B")).hexdigest()
    del m
    return h


@pytest.mark.parametrize("P", [1, 2, 4, 8])
def test_1e11_chunks_golden(ctx, P):
    """The headline config, mask-level: every chunk's resident mask equals
    the golden SHA-256 (tests/golden/make_golden.py --big11: the CPU fast
    sieve, itself equal to the faithful restatement at 1e9 and 1e10)."""
    g = GOLDEN["big"][f"1e11_P{P}"]
    counts, pi_ref, pi_full = ctx.sieve_all(10**11, P)
    assert pi_ref == pi_full == 4_118_054_813 == g["pi_full"]
    assert [int(x) for x in counts] == g["counts"]
    for k in range(P):
        assert _chunk_sha_resident(ctx, 10**11, P, k + 1) == g["mask_sha256"][k], (P, k + 1)


def test_pi_1e12_dropped_tail(ctx):
    """SURVEY.md Gotcha 1: the reference's chunks lose 999999999989. With the
    golden 1e12 P=8 chunk hashes present (make_golden.py --big12), every
    chunk's 7.8 GB mask is checked too."""
    counts, pi_ref, pi_full = ctx.sieve_all(10**12, 8)
    assert pi_ref == 37_607_912_017
    assert pi_full == 37_607_912_018
    g = GOLDEN["big"].get("1e12_P8")
    if g is not None:
        assert [int(x) for x in counts] == g["counts"]
        for k in range(8):
            assert _chunk_sha_resident(ctx, 10**12, 8, k + 1) == g["mask_sha256"][k], k + 1


def test_idempotent(ctx):
    a = ctx.sieve_chunk(10**9, 3, 2)
    b = ctx.sieve_chunk(10**9, 3, 2)
    assert a[1] == b[1] and np.array_equal(a[0], b[0])


def test_window_small(ctx, oracle):
    for lo, hi in [(10**12, 10**12 + 10**7), (2, 100), (1, 2), (4, 4), (999_999_999_989, 10**12)]:
        a = max(lo, 3) | 1
        if hi < a:
            assert ctx.sieve_window(lo, hi) == 0
            continue
        g0, nb = (a - 3) // 2, ((hi if hi & 1 else hi - 1) - a) // 2 + 1
        assert ctx.sieve_window(lo, hi) == oracle.fast_sieve_range(g0, nb, want_mask=False)[1]


def test_device_api_with_torch(ctx):
    """The *_dev_async entry points on torch tensors == the host entry point."""
    import torch
    from mail_sieve_e import sieve as S
    g0, nb = 10**9, 3 * 2**20 + 5
    limit = S.base_limit_for_range(g0, nb)
    table = torch.empty(S.base_table_bytes(limit), dtype=torch.uint8, device="cuda")
    mask = torch.empty((nb + 63) // 64, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    ctx.base_primes_dev_async(limit, table.data_ptr(), table.numel(), sp)
    ctx.sieve_range_dev_async(table.data_ptr(), g0, nb, mask.data_ptr(), cnt.data_ptr(), sp)
    torch.cuda.synchronize()
    m_ref, c_ref = ctx.sieve_odd_range(g0, nb)
    assert int(cnt.item()) == c_ref
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), m_ref)


def test_errors_fail_loudly(ctx):
    from mail_sieve_e import _dse
    with pytest.raises(_dse.DseError):
        ctx.sieve_chunk(10**6, 3, 4)          # my_num outside 1..P
    with pytest.raises(_dse.DseError) as e:
        ctx.sieve_window(2**63, 2**63 + 10**6)    # base primes beyond 2^31
    assert e.value.code == -6


def test_core_lead_single_machine_gpu(tmp_path, oracle):
    """core.lead_start with the HIP engine (P=1: no follower), nccl process group."""
    import socket
    from mail_sieve_e import core
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = core.lead_start(1, 10**6, port, out_dir=str(tmp_path))
    assert (r.my_num, r.count, r.pi_ref, r.pi_full) == (1, 78497, 78498, 78498)
    _, masks, _, _ = oracle.sieve(10**6, 1)
    oracle.finish(str(tmp_path / "ref.txt"), 1, 10**6, 1, masks[0])
    assert (tmp_path / "primes1.txt").read_bytes() == (tmp_path / "ref.txt").read_bytes()


# ---- high-offset window (outside the reference's semantics) ----

def _is_prime_mr(n):
    """Deterministic Miller-Rabin for n < 3.3e24 (first 12 prime bases)."""
    if n < 2:
        return False
    bases = (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37)
    for p in bases:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in bases:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def test_big_base_table(ctx):
    """Two-level base-prime build (limit 1e9 > one-workgroup kernel): sieve of
    [3, 1e9] by the segment kernel + ordered compaction + Barrett factors."""
    import torch
    from mail_sieve_e import sieve as S
    limit = 10**9
    t = torch.zeros(S.base_table_bytes(limit), dtype=torch.uint8, device="cuda")
    ctx.base_primes_dev_async(limit, t.data_ptr(), t.numel(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    hdr = t[:16].cpu().numpy()
    count, cap = int(hdr[:4].view(np.uint32)[0]), int(hdr[4:8].view(np.uint32)[0])
    assert count == 50_847_533  # pi(1e9) - 1 (odd primes)
    P = t[16:16 + 4 * count].cpu().numpy().view(np.uint32)
    assert P[0] == 3 and P[-1] == 999_999_937 and np.all(np.diff(P.astype(np.int64)) > 0)
    moff = (16 + 4 * cap + 7) & ~7
    M = t[moff:moff + 8 * count].cpu().numpy().view(np.uint64)
    n_m = int(np.searchsorted(P, 1 << 20, side="right"))  # Barrett factors exist for p <= 2^20 only
    rng = np.random.default_rng(3)
    for i in rng.integers(0, n_m, 100):
        assert int(M[i]) == (2**64 - 1) // int(P[i])
    for i in rng.integers(0, count, 200):
        assert _is_prime_mr(int(P[i]))


@pytest.mark.parametrize("lo,width", [(4 * 10**12, 10**8), (10**15, 10**7), (10**18, 2 * 10**6)])
def test_window_vs_oracle(ctx, oracle, lo, width):
    g0, nb = ((lo | 1) - 3) // 2, width // 2
    m, c = ctx.sieve_odd_range(g0, nb)
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    assert c == c_ref and np.array_equal(m, m_ref)


def test_window_1e18_miller_rabin(ctx):
    import random
    g0, nb = (10**18 + 1 - 3) // 2, 5 * 10**7
    m, c = ctx.sieve_odd_range(g0, nb)
    bits = np.unpackbits(m.view(np.uint8), bitorder="little")
    rng = random.Random(5)
    idx = [rng.randrange(nb) for _ in range(2000)] + list(np.flatnonzero(bits[:nb])[:2000])
    for j in idx:
        assert bool(bits[j]) == _is_prime_mr(3 + 2 * (g0 + int(j))), j


def test_window_1e18_full(ctx):
    """BASELINE configs[4]: [1e18, 1e18+1e10]. No published count exists; the
    golden value is the oracle's independent CPU count (fast_count_window,
    make_golden.py --window), and additivity over sub-windows holds too."""
    total = ctx.sieve_window(10**18, 10**18 + 10**10)
    assert total == GOLDEN["big"]["window_1e18"]["count"] == 241_272_176
    parts = sum(ctx.sieve_window(10**18 + k * 10**9 + (1 if k else 0), 10**18 + (k + 1) * 10**9) for k in range(10))
    assert parts == total


def test_window_two_contexts_concurrently(ctx):
    """Two contexts (own streams) sieving bucketed windows on one device at
    the same time: each stream has its own bucket scratch."""
    import threading
    from mail_sieve_e.sieve import Context
    wins = [(10**18 + k * 10**9 + (1 if k else 0), 10**18 + (k + 1) * 10**9) for k in range(4)]
    want = [ctx.sieve_window(lo, hi) for lo, hi in wins]
    got, errs = [None] * 4, []

    def work(i):
        try:
            with Context(num_gpus=1) as c:
                for _ in range(3):
                    got[i] = c.sieve_window(*wins[i])
                    assert got[i] == want[i]
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs
    assert got == want


def _odd_primes_upto(n):
    if n < 3:
        return np.zeros(0, dtype=np.int64)
    s = np.ones(n + 1, dtype=bool)
    s[:2] = False
    s[4::2] = False
    for i in range(3, int(n ** 0.5) + 1, 2):
        if s[i]:
            s[i * i::2 * i] = False
    p = np.nonzero(s)[0]
    return p[p > 2]


@pytest.mark.parametrize("limit", [3, 4, 9, 10, 97, 1_000, 316_227, 1_000_003, 1_048_577, 1_048_579, 2_097_153,
                                   2_097_155, 2_457_601])
def test_base_table_primes_exact(ctx, limit):
    """The base table's p[] is every odd prime <= limit, in order, from a
    single odd value up to the largest one-level build (kBaseLimitMax =
    2,457,601; round 6 measured a one-workgroup build of these tables, 79 us
    against 34 us at 1e11, and dropped it)."""
    import torch
    from mail_sieve_e import sieve as S
    t = torch.zeros(S.base_table_bytes(limit), dtype=torch.uint8, device="cuda")
    ctx.base_primes_dev_async(limit, t.data_ptr(), t.numel(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    hdr = t[:16].cpu().numpy()
    count = int(hdr[:4].view(np.uint32)[0])
    want = _odd_primes_upto(limit)
    assert count == len(want) and int(hdr[8:16].view(np.uint64)[0]) == limit
    P = t[16:16 + 4 * count].cpu().numpy().view(np.uint32)
    assert np.array_equal(P.astype(np.int64), want)


@pytest.mark.parametrize("limit", [316_227, 1_000_003, 5_000_011])
def test_table_from_broadcast_primes(ctx, limit):
    """Ranks receive only the primes (dse_base_table_prime_bytes) and finish
    the table locally: same Barrett factors and offsets, same sieve."""
    import torch
    from mail_sieve_e import sieve as S
    dev = torch.device("cuda", 0)
    tbytes, pbytes = S.base_table_bytes(limit), S.base_table_prime_bytes(limit)
    cap = (pbytes - 16) // 4
    m_off = (16 + 4 * cap + 7) & ~7
    a_off = (m_off + 8 * cap + 31) & ~31
    full = torch.empty(tbytes, dtype=torch.uint8, device=dev)
    ctx.base_primes_dev_async(limit, full.data_ptr(), tbytes, 0)
    torch.cuda.synchronize()
    part = torch.full((tbytes,), 0xA5, dtype=torch.uint8, device=dev)
    part[:pbytes] = full[:pbytes]
    ctx.base_table_finish_dev_async(limit, part.data_ptr(), tbytes, 0)
    torch.cuda.synchronize()
    n = int(full[:4].cpu().view(torch.int32)[0])
    P = full[16:16 + 4 * n].cpu().view(torch.int32).numpy()
    n_rows = int(np.searchsorted(P, 1 << 20, side="right"))  # Barrett factors and rows exist for p <= 2^20
    assert torch.equal(full[m_off:m_off + 8 * n_rows], part[m_off:m_off + 8 * n_rows])  # Barrett factors
    assert torch.equal(full[a_off:a_off + 32 * n_rows], part[a_off:a_off + 32 * n_rows])
    g0, nb = (limit * limit) // 2 - 5_000_000, 4_000_000
    outs = []
    for t in (full, part):
        mask = torch.zeros((nb + 63) // 64, dtype=torch.int64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.sieve_range_dev_async(t.data_ptr(), g0, nb, mask.data_ptr(), cnt.data_ptr(), 0)
        torch.cuda.synchronize()
        outs.append((mask.cpu(), int(cnt.item())))
    assert outs[0][1] == outs[1][1] > 0 and torch.equal(outs[0][0], outs[1][0])


@pytest.mark.parametrize("g0,nseg", [(0, 64), (12345, 37), (10**9 + 7, 20), (4 * 10**10, 9)])
def test_table_beyond_range_root(ctx, oracle, g0, nseg):
    """A table built for N=1e12 (primes to 1e6) over ranges whose own roots
    are far smaller: each sixteenth of a range claims large units only up to
    its last prime with p^2 below its end (WheelRange::lcap), so the bound
    moves from piece to piece (64 segments from 0: pieces of 4 segments).
    Masks and counts against the oracle."""
    import torch
    dev = torch.device("cuda", 0)
    limit = 1_000_003
    from mail_sieve_e import sieve as S
    tbytes = S.base_table_bytes(limit)
    table = torch.empty(tbytes, dtype=torch.uint8, device=dev)
    ctx.base_primes_dev_async(limit, table.data_ptr(), tbytes, 0)
    nb = nseg * 1966080 - 4321
    mask = torch.zeros((nb + 63) // 64, dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.sieve_range_dev_async(table.data_ptr(), g0, nb, mask.data_ptr(), cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    assert int(cnt.item()) == c_ref
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), m_ref.view(np.uint64))


@pytest.mark.parametrize("log_kb", [32, 38])
def test_kb_float_quotient_boundary(ctx, oracle, log_kb):
    """The L units take Kb mod p from one float quotient while Kb =
    floor(V/30) < 2^32, from two up to 2^38 and from a 64-bit Barrett
    reduction above: ranges straddling V = 30 * 2^32 and 30 * 2^38
    (segments on both sides) against the oracle."""
    v = 30 * 2**log_kb
    g0 = (v - 3) // 2 - 3 * 1966080 + 12345
    nb = 6 * 1966080 + 777
    m, c = ctx.sieve_odd_range(g0, nb)
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    assert c == c_ref and np.array_equal(m, m_ref)


# ---- bucketed pass (primes > 2^20) ----

def test_bucket_threshold_window_vs_oracle(ctx, oracle):
    """1e13: base primes up to 3.16e6, the ones above 2^20 go through buckets."""
    g0, nb = (10**13 + 1 - 3) // 2, 5 * 10**7
    m, c = ctx.sieve_odd_range(g0, nb)
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    assert c == c_ref and np.array_equal(m, m_ref)


def test_bucket_multi_pass_mask(oracle):
    """Passes of 3 segments (test-only context option bucket_pass_segments):
    the pass boundaries, the per-pass bucket builds and the output offsets,
    bit-exact."""
    from mail_sieve_e import sieve as S
    g0, nb = (10**14 + 12345) // 2 * 1 + 7, 20 * 983040 + 12345  # ragged start and end, 21 segments
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    with S.Context(num_gpus=1) as c3:
        c3.debug_set_option("bucket_pass_segments", 3)
        m, c = c3.sieve_odd_range(g0, nb)
    assert c == c_ref and np.array_equal(m, m_ref)


@pytest.mark.parametrize("split", [20, 23, 25, 63])
def test_bucket_bands_mask(oracle, split):
    """Band split of the bucketed primes (test-only option bucket_split_log2):
    p <= 2^split one-level fill, above it the staged two-level fill. At 1e16
    the bucketed primes run from 2^20 to 1e8 = 2^26.6: all two-level (20),
    two splits inside, all one-level (63); in one pass and in passes of 3
    segments, bit-exact. The production split is covered by every window test."""
    from mail_sieve_e import sieve as S
    g0, nb = 10**16 // 2 + 12345, 20 * 983040 + 777
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    with S.Context(num_gpus=1) as c:
        c.debug_set_option("bucket_split_log2", split)
        m, cnt = c.sieve_odd_range(g0, nb)
        assert cnt == c_ref and np.array_equal(m, m_ref)
        c.debug_set_option("bucket_pass_segments", 3)
        m, cnt = c.sieve_odd_range(g0, nb)
        assert cnt == c_ref and np.array_equal(m, m_ref)


def test_bucket_scratch_freed_with_context():
    """Each context owns its bucketed-pass scratch and dse_destroy frees it:
    creating and destroying contexts that sieve a 1e18 slice must not shrink
    the device's free memory (grow-only global scratch)."""
    import torch
    from mail_sieve_e import sieve as S
    lo = 10**18
    def once():
        with S.Context(num_gpus=1) as c:
            c.sieve_window(lo, lo + 2 * 10**8)
    once()
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(4):
        once()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert free1 >= free0 - (64 << 20), (free0, free1)


def test_debug_option_rejects_unknown(ctx):
    from mail_sieve_e import _dse
    with pytest.raises(_dse.DseError):
        ctx.debug_set_option("no_such_option", 1)
    for name, bad in (("bucket_split_log2", 64), ("bucket_split_log2", -1), ("bucket_pass_segments", -1),
                      ("bucket_cap_divisor", -1), ("bucket_k0_divisor", -1), ("wheel_geometry", 3),
                      ("wheel_geometry", -1), ("scratch_poison", 2), ("scratch_poison", -1)):
        with pytest.raises(_dse.DseError):
            ctx.debug_set_option(name, bad)


def test_bucket_overflow_flag(oracle):
    """A bucketed pass over its entry capacity (forced with the test-only
    option bucket_cap_divisor; the production bound is rigorous) must fail
    loudly: DSE_EINTERNAL from the blocking entry points, bit 63 of the device
    count plus DSE_EINTERNAL from dse_device_status on the async path, and no
    stale flag once the option is cleared."""
    import torch
    from mail_sieve_e import _dse
    from mail_sieve_e import sieve as S
    g0, nb = (10**13 + 1 - 3) // 2, 5 * 10**6
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    with S.Context(num_gpus=1) as c:
        c.debug_set_option("bucket_cap_divisor", 1000)
        with pytest.raises(_dse.DseError) as e:
            c.sieve_odd_range(g0, nb)
        assert e.value.code == -7 and "capacity" in str(e.value)
        with pytest.raises(_dse.DseError) as e:
            c.sieve_window(10**18, 10**18 + 10**7)
        assert e.value.code == -7
        limit = S.base_limit_for_range(g0, nb)
        table = torch.empty(S.base_table_bytes(limit), dtype=torch.uint8, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        sp = torch.cuda.current_stream().cuda_stream
        c.base_primes_dev_async(limit, table.data_ptr(), table.numel(), sp)
        c.sieve_range_dev_async(table.data_ptr(), g0, nb, 0, cnt.data_ptr(), sp)
        torch.cuda.synchronize()
        assert int(cnt.item()) < 0  # bit 63
        with pytest.raises(_dse.DseError) as e:
            c.device_status()
        assert e.value.code == -7
        c.device_status()  # cleared
        c.debug_set_option("bucket_cap_divisor", 0)
        m, cnt2 = c.sieve_odd_range(g0, nb)
        assert cnt2 == c_ref and np.array_equal(m, m_ref)


def test_bucket_overflow_stale_scratch(oracle):
    """an overflowed pass right after a scratch grow, with the
    scratch full of stale bytes (test-only option scratch_poison): the fill
    kernel still zeroes every band-0 region fill and the wheel kernel clamps
    them, so the pass reads only what it wrote -- DSE_EINTERNAL, no fault --
    and the same context is bit-exact afterwards (poisoned scratch, no
    overflow: every pass rewrites what it reads)."""
    from mail_sieve_e import _dse
    from mail_sieve_e import sieve as S
    g0, nb = (10**15 + 1 - 3) // 2, 3 * 10**6
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    with S.Context(num_gpus=1) as c:
        c.debug_set_option("scratch_poison", 1)
        c.debug_set_option("bucket_split_log2", 22)  # both bands in the pass
        c.debug_set_option("bucket_cap_divisor", 1000)
        with pytest.raises(_dse.DseError) as e:
            c.sieve_odd_range(g0, nb)  # first pass of the context: a fresh (grown) scratch
        assert e.value.code == -7
        c.debug_set_option("bucket_cap_divisor", 0)
        m, cnt = c.sieve_odd_range(g0, nb)
        assert cnt == c_ref and np.array_equal(m, m_ref)
        c.debug_set_option("bucket_split_log2", 0)
        m, cnt = c.sieve_odd_range(g0, nb)
        assert cnt == c_ref and np.array_equal(m, m_ref)


@pytest.mark.parametrize("div", [8, 100000])
def test_bucket_spill_list(oracle, div):
    """Band-0 regions shrunk (test-only option bucket_k0_divisor): hits past a
    region's capacity go through the spill list, and masks and counts stay
    exact. div=8 spills a region's tail, 100000 leaves one slot per region (every
    other hit spilled); multi-pass (3-segment passes) with both bands."""
    from mail_sieve_e import sieve as S
    g0, nb = (10**15 + 1 - 3) // 2, 3 * 10**6
    m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
    with S.Context(num_gpus=1) as c:
        c.debug_set_option("bucket_k0_divisor", div)
        m, cnt = c.sieve_odd_range(g0, nb)
        assert cnt == c_ref and np.array_equal(m, m_ref)
        c.debug_set_option("bucket_split_log2", 22)
        c.debug_set_option("bucket_pass_segments", 3)
        g1, nb1 = (10**18 + 1 - 3) // 2, 10**7
        m, cnt = c.sieve_odd_range(g1, nb1)
        m_ref, c_ref = oracle.fast_sieve_range(g1, nb1)
        assert cnt == c_ref and np.array_equal(m, m_ref)


def test_scratch_null_stream_then_host_call(oracle):
    """a bucketed pass on the null stream (dev_async, stream 0)
    followed at once by a host entry point on the same context (its own
    non-blocking stream, the same scratch): the second pass waits for the
    first (event-ordered scratch), both bit-exact."""
    import torch
    from mail_sieve_e import sieve as S
    g0a, nba = (10**15 + 1 - 3) // 2, 3 * 10**7
    g0b, nbb = (10**14 + 1 - 3) // 2, 2 * 10**7
    ra, rb = oracle.fast_sieve_range(g0a, nba), oracle.fast_sieve_range(g0b, nbb)
    with S.Context(num_gpus=1) as c:
        limit = S.base_limit_for_range(g0a, nba)
        table = torch.empty(S.base_table_bytes(limit), dtype=torch.uint8, device="cuda")
        mask = torch.zeros((nba + 63) // 64, dtype=torch.int64, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        for _ in range(3):
            cnt.zero_()
            torch.cuda.synchronize()
            c.base_primes_dev_async(limit, table.data_ptr(), table.numel(), 0)
            c.sieve_range_dev_async(table.data_ptr(), g0a, nba, mask.data_ptr(), cnt.data_ptr(), 0)
            m, cb = c.sieve_odd_range(g0b, nbb)  # no host sync in between
            assert cb == rb[1] and np.array_equal(m, rb[0])
            torch.cuda.synchronize()
            assert int(cnt.item()) == ra[1]
            assert np.array_equal(mask.cpu().numpy().view(np.uint64), ra[0])
        c.device_status()


def test_init_more_devices_than_visible():
    """dse_init(n) with n above the visible devices: DSE_EINVAL, a message
    naming both numbers, no context (the single-process multi-GPU path,
    core.clj:141-147's wait for clients, must refuse rather than hang)."""
    import torch
    from mail_sieve_e import _dse
    from mail_sieve_e import sieve as S
    n = torch.cuda.device_count()
    with pytest.raises(_dse.DseError) as e:
        S.Context(num_gpus=n + 1)
    assert e.value.code == -1
    assert f"asked for {n + 1} GPUs, {n} visible" in str(e.value)


@pytest.mark.parametrize("geometry", [1, 2])
def test_segment_geometries_vs_oracle(oracle, geometry):
    """The full (2^17 periods) and half-size (2^16, dse_wheel_half.hip)
    segment geometries alone (test-only option wheel_geometry), on ragged and
    random ranges, bit-exact against the oracle. The default (0) splits a
    range's last partial round of full segments into half segments; every
    chunk test covers that path."""
    from mail_sieve_e import sieve as S
    rng = np.random.default_rng(0xC0DE + geometry)
    ranges = [(0, 1), (0, 65), (5, 7), (31, 1000), (2**20 - 64, 2**20 + 128), (10**6, 3 * 2**20 + 17),
              (123456789, 2**21 - 1), (49_999_999_000, 999), (0, 300 * 983040 + 12345)]
    ranges += [(int(rng.integers(0, 5 * 10**10)), int(rng.integers(1, 6 * 2**20))) for _ in range(12)]
    with S.Context(num_gpus=1) as c:
        c.debug_set_option("wheel_geometry", geometry)
        for g0, nb in ranges:
            m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
            m, cnt = c.sieve_odd_range(g0, nb)
            assert cnt == c_ref and np.array_equal(m, m_ref), (geometry, g0, nb)


@pytest.mark.parametrize("geometry", [0, 1, 2])
def test_pooled_chunks_vs_oracle(oracle, geometry):
    """Several chunks of one device in one launch (launch_sieve_ranges pools a
    device's chunks and the dropped tail; more than 9 ranges go in batches):
    every chunk mask and count of random (N, P), P up to 20, against the
    oracle, with the segments past the last full round in the half-size
    geometry (0, when it pays), all full (1) or all half (2)."""
    from mail_sieve_e import sieve as S
    rng = np.random.default_rng(0xB10C + geometry)
    cases = [(10**9, 8), (2 * 10**8 + 7, 11), (10**7 + 1, 20)]
    cases += [(int(rng.integers(10**6, 3 * 10**8)), int(rng.integers(1, 21))) for _ in range(6)]
    with S.Context(num_gpus=1) as c:
        c.debug_set_option("wheel_geometry", geometry)
        for N, P in cases:
            cs = (N - 1) // 2 // P
            tail_g, tail_n = oracle.tail_range(N, P)
            counts, pi_ref, pi_full = c.sieve_all(N, P)
            for k in range(P):
                m_ref, c_ref = oracle.fast_sieve_range(k * cs, cs)
                assert int(counts[k]) == c_ref, (geometry, N, P, k)
                assert np.array_equal(c.copy_chunk_mask(N, P, k + 1), m_ref), (geometry, N, P, k)
            t_ref = oracle.fast_sieve_range(tail_g, tail_n, want_mask=False)[1] if tail_n else 0
            assert pi_full - pi_ref == t_ref, (geometry, N, P)


@pytest.mark.parametrize("lo", [17, 18, 20])
def test_bucket_lo_threshold_mask(oracle, lo):
    """The bucket threshold of bucketed ranges (production 2^19; test-only
    option bucket_lo_log2): the primes in (2^lo, 2^20] move between the wheel
    kernel's L units and the band-0 fill; a 1e13 range (base primes up to
    3.2e6) and a 1e16 range (up to 1e8), each in one pass and in passes of 3
    segments, bit-exact against the oracle."""
    from mail_sieve_e import sieve as S
    for g0, nb in (((10**13 + 1 - 3) // 2, 5 * 10**7), (10**16 // 2 + 12345, 20 * 983040 + 777)):
        m_ref, c_ref = oracle.fast_sieve_range(g0, nb)
        with S.Context(num_gpus=1) as c:
            c.debug_set_option("bucket_lo_log2", lo)
            m, cnt = c.sieve_odd_range(g0, nb)
            assert cnt == c_ref and np.array_equal(m, m_ref), (lo, g0)
            c.debug_set_option("bucket_pass_segments", 3)
            m, cnt = c.sieve_odd_range(g0, nb)
            assert cnt == c_ref and np.array_equal(m, m_ref), (lo, g0, 3)
    with S.Context(num_gpus=1) as c:
        from mail_sieve_e import _dse
        for bad in (1, 16, 21):
            with pytest.raises(_dse.DseError):
                c.debug_set_option("bucket_lo_log2", bad)


def test_pooled_and_bucketed_chunks_in_one_call(ctx):
    """One dse_sieve_all call whose chunks take both paths of
    launch_sieve_ranges: N = 1.2e12, P = 8 on one device, chunks
    1-7 (the square root of their largest value below 2^20) pooled into one
    persistent launch, chunk 8 through the bucketed pass, issued inline before
    the pooled launch on the same stream with the same count slots. Every
    chunk's count, and the masks of chunk 7 (pooled, last of the launch) and
    chunk 8 (bucketed), equal the single-range path (dse_sieve_odd_range, one
    range per call); pi_ref + the tail equals the one-range count of [3, N]."""
    N, P = 12 * 10**11, 8
    cs = (N - 1) // 2 // P
    counts, pi_ref, pi_full = ctx.sieve_all(N, P)
    import math
    assert math.isqrt(3 + 2 * (7 * cs - 1)) <= 2**20 < math.isqrt(3 + 2 * (8 * cs - 1))
    for k in (7, 8):
        m, c = ctx.sieve_odd_range((k - 1) * cs, cs)
        assert int(counts[k - 1]) == c, k
        assert np.array_equal(ctx.copy_chunk_mask(N, P, k), m), k
        del m
    for k in range(1, 7):
        _, c = ctx.sieve_odd_range((k - 1) * cs, cs, want_mask=False)
        assert int(counts[k - 1]) == c, k
    _, whole = ctx.sieve_odd_range(0, (N - 1) // 2, want_mask=False)
    assert pi_full == 1 + whole
    assert pi_ref == 1 + sum(int(x) for x in counts)

"""Generate tests/golden/golden.json from the CPU oracle (oracle/dse_oracle.c).

Run from the repo root:  python tests/golden/make_golden.py [--big]

Every value here comes from the faithful restatement of sieve.clj (ref_*),
except the N >= 1e10 mask hashes, which come from the independent fast
segmented sieve (fast_*) after it was checked against ref_* at 1e9. The
reference itself cannot run in this image (Clojure/JVM absent), so these are
restatement outputs, cross-checked in tests/test_oracle.py against published
pi(10^k), sympy and the SURVEY.md section 4 table.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as o  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def sweep(seed: int = 0x5EED, n_cases: int = 120):
    """Seeded (N, P) sweep, N in [20, 1e7], P in [1, 8], cs >= 4."""
    rng = np.random.default_rng(seed)
    cases = []
    while len(cases) < n_cases:
        lo_exp = rng.uniform(np.log10(20), 7)
        N = int(10 ** lo_exp)
        P = int(rng.integers(1, 9))
        cs, _ = o.spread_work(N, P)
        if cs < 4:
            continue
        cs, masks, counts, msgs = o.sieve(N, P)
        cases.append({"N": N, "P": P, "cs": cs, "counts": [int(c) for c in counts],
                      "pi_ref": o.pi_ref(counts), "mask_sha256": [sha(m) for m in masks],
                      "prime_messages": int(msgs)})
    return cases


def files():
    out = []
    import tempfile
    for N, P in [(10_000, 2), (1_000_000, 3)]:
        cs, masks, counts, _ = o.sieve(N, P)
        for k in range(P):
            with tempfile.NamedTemporaryFile(delete=False) as f:
                path = f.name
            o.finish(path, k + 1, N, P, masks[k])
            b = open(path, "rb").read()
            os.unlink(path)
            out.append({"N": N, "P": P, "my_num": k + 1, "bytes": len(b), "lines": b.count(b"\n"),
                        "sha256": hashlib.sha256(b).hexdigest(), "nonzero": int(counts[k]) + (1 if k == 0 else 0)})
    return out


def big(include_1e10: bool):
    res = {}
    t = time.time()
    cs, masks, counts, msgs = o.sieve(10**9, 1)
    m_fast, c_fast = o.fast_sieve_range(0, cs)
    assert np.array_equal(m_fast, masks[0]) and c_fast == int(counts[0]), "fast sieve disagrees with ref at 1e9"
    res["1e9_P1"] = {"N": 10**9, "P": 1, "cs": cs, "counts": [int(counts[0])], "pi_ref": o.pi_ref(counts),
                     "mask_sha256": [sha(masks[0])], "source": "ref_sieve (faithful) == fast_sieve_range"}
    print(f"1e9 done in {time.time() - t:.1f}s", flush=True)
    if include_1e10:
        for P in (2, 4, 8):
            t = time.time()
            N = 10**10
            cs, _ = o.spread_work(N, P)
            entry = {"N": N, "P": P, "cs": cs, "counts": [], "mask_sha256": [], "source": "fast_sieve_range"}
            for k in range(P):
                m, c = o.fast_sieve_range(k * cs, cs)
                entry["counts"].append(int(c))
                entry["mask_sha256"].append(sha(m))
            g, nb = o.tail_range(N, P)
            _, ct = o.fast_sieve_range(g, nb, want_mask=False)
            entry["pi_ref"] = 1 + sum(entry["counts"])
            entry["pi_full"] = entry["pi_ref"] + int(ct)
            res[f"1e10_P{P}"] = entry
            print(f"1e10 P={P} done in {time.time() - t:.1f}s", flush=True)
    return res


def chunk_hash(g0: int, nbits: int, piece: int = 1 << 30):
    """SHA-256 of the odd-only mask of indices [g0, g0+nbits) (ceil(nbits/64)
    LE uint64 words, bits past nbits zero) and its popcount, streamed through
    fast_sieve_range in pieces of `piece` bits (a multiple of 64), so the
    whole mask never sits in memory."""
    assert piece % 64 == 0
    h = hashlib.sha256()
    cnt = 0
    off = 0
    while off < nbits:
        nb = min(piece, nbits - off)
        m, c = o.fast_sieve_range(g0 + off, nb)
        h.update(m.view(np.uint8))
        cnt += int(c)
        off += nb
    return h.hexdigest(), cnt


def big_streamed(N: int, Ps) -> dict:
    """Per-chunk mask SHA-256 and counts of (N, P) runs, streamed (SURVEY 8(d)
    headline and 1e12 configs: masks of 6.25 GB per P at 1e11, 62.5 GB at 1e12)."""
    res = {}
    for P in Ps:
        t = time.time()
        cs, _ = o.spread_work(N, P)
        entry = {"N": N, "P": P, "cs": cs, "counts": [], "mask_sha256": [],
                 "source": "fast_sieve_range (streamed), checked against ref_sieve at 1e9 and 1e10"}
        for k in range(P):
            hx, c = chunk_hash(k * cs, cs)
            entry["counts"].append(c)
            entry["mask_sha256"].append(hx)
        g, nb = o.tail_range(N, P)
        _, ct = o.fast_sieve_range(g, nb, want_mask=False)
        entry["pi_ref"] = 1 + sum(entry["counts"])
        entry["pi_full"] = entry["pi_ref"] + int(ct)
        res[f"1e{len(str(N)) - 1}_P{P}"] = entry
        print(f"N={N:.0e} P={P} done in {time.time() - t:.1f}s pi_full={entry['pi_full']}", flush=True)
    return res


def ref_check_1e10(g: dict) -> None:
    """The faithful restatement (ref_sieve) at N=1e10, P=2/4/8 must reproduce
    the fast sieve's golden chunk hashes: pins fast_sieve_range, which alone
    reaches 1e11 and 1e12, to the restatement at 1e10 as well as 1e9."""
    for P in (2, 4, 8):
        t = time.time()
        e = g["big"][f"1e10_P{P}"]
        cs, masks, counts, _ = o.sieve(10**10, P)
        assert [int(c) for c in counts] == e["counts"], P
        assert [sha(m) for m in masks] == e["mask_sha256"], P
        del masks
        e["source"] = "ref_sieve (faithful) == fast_sieve_range"
        print(f"1e10 P={P}: ref_sieve == fast_sieve_range ({time.time() - t:.1f}s)", flush=True)


def window(g: dict) -> None:
    lo, hi = 10**18, 10**18 + 10**10
    t = time.time()
    c = o.count_window(lo, hi)
    g["big"]["window_1e18"] = {"lo": lo, "hi": hi, "count": c,
                               "source": "fast_count_window (OpenMP CPU sieve, independent of the GPU path)"}
    print(f"window [1e18, 1e18+1e10]: {c} ({time.time() - t:.1f}s)", flush=True)


def main():
    """Default: regenerate the small fixtures (sweep, files, 1e9). Flags add or
    refresh sections of the existing golden.json in place:
      --big      1e10 P=2/4/8 (fast sieve, in memory)
      --ref1e10  check the 1e10 entries with the faithful restatement
      --big11    1e11 P=1/2/4/8 (streamed)
      --big12    1e12 P=8 (streamed, ~10 min on 8 cores)
      --window   the [1e18, 1e18+1e10] count"""
    flags = set(sys.argv[1:])
    incremental = flags & {"--ref1e10", "--big11", "--big12", "--window"}
    if incremental and os.path.exists(OUT):
        g = json.load(open(OUT))
    else:
        g = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/dse_oracle.c",
             "sweep_seed": "0x5EED", "sweep": sweep(), "files": files(), "big": big("--big" in flags)}
    if "--ref1e10" in flags:
        ref_check_1e10(g)
    if "--big11" in flags:
        g["big"].update(big_streamed(10**11, (1, 2, 4, 8)))
    if "--big12" in flags:
        g["big"].update(big_streamed(10**12, (8,)))
    if "--window" in flags:
        window(g)
    with open(OUT, "w") as f:
        json.dump(g, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()

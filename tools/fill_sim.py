"""Lane efficiency of the band-0 fill walk (bucket_fill_wg) at the window [1e18, 1e18+1e10] for chunk
schedules: hits / (64 x wave iterations) of the divergent per-round walks, over sampled waves (CPU only,
profiling aid): python tools/fill_sim.py [waves]."""
import numpy as np, sys, math
lo = 10**18
span_seg = 30 << 17
nseg = -(-10**10 // span_seg)
V0 = lo  # approx
# band-0 primes 2^19 < p <= 2^28
def primes_upto(n):
    s = np.ones(n // 2 + 1, dtype=bool); s[0] = False
    for i in range(3, int(n**0.5) + 1, 2):
        if s[i // 2]: s[i * i // 2::i] = False
    return 2 * np.nonzero(s)[0] + 1
P = primes_upto(1 << 28)
P = P[P > (1 << 19)].astype(np.int64)
print("band-0 primes", len(P), "nseg", nseg, file=sys.stderr)
T = np.array([sum(1 for m in range(1, r + 1) if math.gcd(m, 30) == 1) for r in range(30)], dtype=np.int64)
def F(x):  # m in [1, x] coprime to 30
    return 8 * (x // 30) + T[x % 30]
stride = 1024 * 256
rng = np.random.default_rng(1)
waves = rng.choice(4096, size=int(sys.argv[1]) if len(sys.argv) > 1 else 128, replace=False)
def run(sched, RG=16):
    it = 0; hits = 0; visits = 0
    nR = -(-len(P) // stride)
    for w in waves:
        j = w * 64 + np.arange(64)
        for R in range(nR):
            g = R // RG
            C = sched(g)
            jj = (stride - 1 - j) if (R & 1) else j
            i = R * stride + jj
            ok = i < len(P)
            if not ok.any(): continue
            p = P[np.minimum(i, len(P) - 1)]
            nch = -(-nseg // C)
            a = V0 + np.arange(nch, dtype=np.int64)[:, None] * (C * span_seg)
            b = np.minimum(a + C * span_seg, V0 + nseg * span_seg)
            a = np.maximum(a, p[None, :] * p[None, :])
            m0 = -(-a // p[None, :]); m1 = (b - 1) // p[None, :]
            n = np.where(m1 >= m0, F(m1) - F(m0 - 1), 0) * ok[None, :]
            it += n.max(axis=1).sum(); hits += n.sum(); visits += nch
    return it, hits, visits
for name, sched in [("c32", lambda g: 32), ("c16g1", lambda g: 16 << min(3, g)), ("c16g2", lambda g: 16 << min(3, 2 * g)),
                    ("c8", lambda g: 8), ("c64", lambda g: 64), ("c128", lambda g: 128), ("c4096", lambda g: 4096),
                    ("c16,64,256,1024", lambda g: [16, 64, 256, 1024][min(g, 3)])]:
    it, h, v = run(sched)
    print(f"{name:18s} iterations {it:>10d}  hits {h:>10d}  lane eff {h / (64 * it):.3f}  (r, chunk) visits {v * 16:>8d}")

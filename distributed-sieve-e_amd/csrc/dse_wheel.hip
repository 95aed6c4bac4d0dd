// dse_wheel.hip -- mod-30 wheel segmented sieve for gfx950 (MI355X).
//
// Same contract as the odd-only kernel (dse_kernels.hip): bit j of the caller's
// range stands for the odd value 3+2(g_start+j), the reference's element j of its
// chunk vector (sieve.clj:9-13), and a set bit = prime. Only the LDS image
// differs: multiples of 3 and 5 are never stored, so the marking loops (the
// replacement of sieve.clj:36-71's index walk) touch 8/15 of the words the
// odd-only image needs, and one 128 KiB segment covers 3,932,160 integers.
//
// Geometry. V0 = v_start - 1 (even); segment s covers the integers
// [Vs, Vs + 30*2^17) with Vs = V0 + s*30*2^17, which is exactly output bits
// [s*1966080, (s+1)*1966080) -- a whole number of words, so no output word is
// shared by two segments. The 8 odd residues rho_0 < ... < rho_7 in [1,29]
// with gcd(V0 + rho, 30) = 1 define the planes: plane i bit k <-> the value
// Vs + rho_i + 30k, i.e. output bit 15k + (rho_i - 1)/2 of the segment.
//
// LDS image: plane i is split into 8 columns of LS = 2^14 periods; column
// C = 8i + c holds periods [c*LS, (c+1)*LS) of plane i, 32 per word, and word
// (row r, column C) sits at r*64 + C. The bank of a word is C mod 32 whatever
// its row, so 32 lanes in 32 distinct columns never conflict.
//
// Per segment, one 1024-thread workgroup:
//   1. init: every word = the OR of the patterns of 7..61 (register shifts);
//   2. mark (ds_or_b32), units handed out through an LDS counter:
//      - A (61 < p <= LS/16): one prime per wave, lane L walks column L;
//      - B (LS/16 < p <= LS): 8 primes x 8 planes per wave; lane (prime j,
//        plane i) walks its plane's 8 columns diagonally (column (j+t) mod 8 at
//        step t), so a half-wave touches 32 distinct columns at every step;
//      - L (p > LS): one prime per lane, its 8 planes in a lane-rotated order,
//        starts from the table's wheel offsets with one Barrett reduction;
//   3. expand: lane reads one row of its column in all 8 planes, transposes the
//      8x32 bits into 32 period bytes, maps each through a 256-entry LDS table
//      to the 15 odd slots of its period, packs 480 output bits, fixes the
//      small primes 3..61, masks the range end, popcounts, stores.
// See DESIGN.md section 4 for the rooflines.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dse_internal.h"

namespace dse {
namespace {

constexpr uint32_t kPhaseMidA = 1, kPhaseMidB = 2, kPhaseLarge = 4, kPhaseSmall = 8, kPhaseStore = 16;
constexpr uint32_t kPhaseAll = 31;

constexpr uint32_t KP = 1u << kWheelLogKP;  // periods per segment (per plane)
constexpr uint32_t LOG_LS = 14;
constexpr uint32_t LS = 1u << LOG_LS;       // periods per column
constexpr uint32_t ROWS = LS / 32;          // 512 words per column
constexpr uint32_t NT = 1024;
constexpr uint32_t NW = NT / 64;
constexpr uint32_t TA = LS / 16;            // A/B threshold
constexpr uint32_t kMidCap = 1920;          // odd primes in (61, LS]: 1882
constexpr uint32_t kOutWordsPerSeg = (uint32_t)(kWheelOutBits / 32);  // 61440

constexpr int kNQ = 15;
constexpr uint32_t kQ[kNQ] = {7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61};
constexpr uint32_t kQMax = 61;

constexpr uint64_t pat64(uint32_t q) {
  uint64_t v = 0;
  for (uint32_t k = 0; k < 64; k += q) v |= 1ull << k;
  return v;
}
constexpr uint32_t inv30_const(uint32_t q) {
  for (uint32_t x = 1; x < q; ++x)
    if ((30 * x) % q == 1) return x;
  return 0;
}

struct WheelArgs {
  uint64_t V0;         // v_start - 1
  uint64_t nbits;      // odd candidates in the range
  uint64_t KB0;        // floor(V0 / 30)
  uint64_t rho_pack;   // rho_i in bits [5i, 5i+5)
  uint32_t iota_pack;  // absolute residue index of plane i in bits [3i, 3i+3)
  uint32_t e_bits;     // bit i: floor((V0 + rho_i)/30) = KB0 + 1
  uint32_t fix0;       // output word 0 bits of the primes 3..61 inside the range
  uint32_t phases;
  uint8_t v0q[kNQ];    // V0 mod q
};

__device__ __forceinline__ void lds_or(uint32_t* a, uint32_t v) {
  __hip_atomic_fetch_or(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// x mod p for x < 2^63 with m = floor((2^64-1)/p).
__host__ __device__ __forceinline__ uint32_t mod_barrett(uint64_t x, uint32_t p, uint64_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t q = __umul64hi(x, m);
#else
  uint64_t q = (uint64_t)(((unsigned __int128)x * m) >> 64);
#endif
  uint64_t r = x - q * p;
  if (r >= p) r -= p;
  if (r >= p) r -= p;
  return (uint32_t)r;
}

__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// t mod p, t < 2^24
__device__ __forceinline__ uint32_t mod_small(uint32_t t, uint32_t p, float invp) {
  uint32_t q = (uint32_t)((float)t * invp);
  int32_t r = (int32_t)(t - q * p);
  r = r < 0 ? r + (int32_t)p : r;
  r = r >= (int32_t)p ? r - (int32_t)p : r;
  return (uint32_t)r;
}

// ceil(t / p), t < 2^24
__device__ __forceinline__ uint32_t div_ceil_small(uint32_t t, uint32_t p, float invp) {
  uint32_t q = (uint32_t)((float)t * invp);
  q = q * p > t ? q - 1 : q;
  q = (q + 1) * p <= t ? q + 1 : q;  // q = floor(t/p)
  return q + (q * p != t ? 1u : 0u);
}

// floor(t / p), t < 2^24
__device__ __forceinline__ uint32_t div_small(uint32_t t, uint32_t p, float invp) {
  uint32_t q = (uint32_t)((float)t * invp);
  q = q * p > t ? q - 1 : q;
  q = (q + 1) * p <= t ? q + 1 : q;
  return q;
}

// x*y mod p for x, y < p <= 2^14
__device__ __forceinline__ uint32_t mulmod_small(uint32_t x, uint32_t y, uint32_t p, float invp) {
  const uint32_t xy = x * y;
  uint32_t q = (uint32_t)((float)xy * invp);
  int32_t r = (int32_t)(xy - q * p);
  r = r < 0 ? r + (int32_t)p : r;
  r = r < 0 ? r + (int32_t)p : r;
  r = r >= (int32_t)p ? r - (int32_t)p : r;
  r = r >= (int32_t)p ? r - (int32_t)p : r;
  return (uint32_t)r;
}

// 30^{-1} mod p for p coprime to 30: (p*a + 1)/30 with p*a = -1 (mod 30);
// a = 2*nibble + 1, nibble indexed by (p mod 30)/2.
__host__ __device__ __forceinline__ uint64_t inv30_of(uint64_t p) {
  constexpr uint64_t T = (14ull << 0) | (8ull << 12) | (9ull << 20) | (11ull << 24) | (3ull << 32) | (5ull << 36) |
                         (6ull << 44) | (0ull << 56);
  const uint32_t r = (uint32_t)(p % 30u);
  const uint64_t a = 2 * ((T >> (4 * (r >> 1))) & 15) + 1;
  return (p * a + 1) / 30;
}

// First k >= 0 with p | Vs + rho + 30k, given Xs = Vs mod p (p in (61, 2^14]).
__device__ __forceinline__ uint32_t plane_first(uint32_t Xs, uint32_t rho, uint32_t p, uint32_t inv30,
                                                float invp) {
  uint32_t t = Xs + rho;
  t = t >= p ? t - p : t;
  const uint32_t u = t ? p - t : 0u;
  return mulmod_small(u, inv30, p, invp);
}

// First k >= start with k = kp (mod p); kp < p, start < 2^23.
__device__ __forceinline__ uint32_t first_at_or_after(uint32_t kp, uint32_t start, uint32_t p, float invp) {
  if (start <= kp) return kp;
  return kp + p * div_ceil_small(start - kp, p, invp);
}

// Smallest plane index k whose value Vs + rho + 30k is >= p^2, given D = p^2 - Vs > 0.
__device__ __forceinline__ uint32_t kmin_for(uint32_t D, uint32_t rho) {
  return D > rho ? (D - rho + 29u) / 30u : 0u;
}

// 8 diagonal column steps of one lane's prime with compile-time hit counts:
// NU unconditional marks and NX value-predicated ones per column; at the wrap
// from column 7 back to column 0 the offset restarts at the plane start O0.
template <int NU, int NX>
__device__ __forceinline__ void diag_walk(uint32_t* __restrict__ seg, uint32_t off, uint32_t p, uint32_t cb,
                                          uint32_t c, uint32_t O0) {
#pragma unroll 2
  for (uint32_t t = 0; t < 8; ++t) {
    uint32_t* colp = seg + cb + c;
#pragma unroll
    for (int h = 0; h < NU; ++h) {
      lds_or(colp + ((off >> 5) << 6), 1u << (off & 31));
      off += p;
    }
#pragma unroll
    for (int h = 0; h < NX; ++h) {
      const bool hit = off < LS;
      const uint32_t o = hit ? off : 0u;
      lds_or(colp + ((o >> 5) << 6), hit ? 1u << (o & 31) : 0u);
      off = hit ? off + p : off;
    }
    off -= LS;
    c = (c + 1) & 7;
    off = c == 0 ? O0 : off;
  }
}

template <int U>
__device__ __forceinline__ void diag_dispatch(uint32_t n_u, uint32_t n_x, uint32_t* __restrict__ seg, uint32_t off,
                                              uint32_t p, uint32_t cb, uint32_t c, uint32_t O0) {
  if constexpr (U <= 15) {
    if (n_u == U) {
      if (n_x == 1) diag_walk<U, 1>(seg, off, p, cb, c, O0);
      else diag_walk<U, 2>(seg, off, p, cb, c, O0);
      return;
    }
    diag_dispatch<U + 1>(n_u, n_x, seg, off, p, cb, c, O0);
  }
}

// 8x8 bit-matrix transpose: byte i bit j <-> byte j bit i.
__device__ __forceinline__ uint64_t transpose8(uint64_t x) {
  uint64_t t;
  t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x ^= t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x ^= t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  x ^= t ^ (t << 28);
  return x;
}

__global__ __launch_bounds__(NT) void wheel_segments_kernel(const void* __restrict__ table, WheelArgs wa,
                                                            uint32_t* __restrict__ out,
                                                            unsigned long long* __restrict__ count_out) {
  __shared__ __attribute__((aligned(16))) uint32_t seg[KP * 8 / 32];
  __shared__ uint64_t s_mid_m[kMidCap];
  __shared__ uint32_t s_mid_p[kMidCap];
  __shared__ uint32_t s_lut[256];
  __shared__ uint32_t s_ctr;
  __shared__ uint32_t s_thr[3];
  __shared__ unsigned long long s_wave_cnt[NW];

  const TableHeader* th = reinterpret_cast<const TableHeader*>(table);
  const uint32_t np = th->count;
  const uint32_t* __restrict__ P = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + 16);
  const uint64_t* __restrict__ M =
      reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(table) + table_m_offset(th->cap));
  const uint32_t* __restrict__ A =
      reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + table_a_offset(th->cap));

  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t phases = wa.phases;

  if (tid == 0) {
    // first index with p > 61, with p > TA, with p > LS (capped by the LDS stage)
    uint32_t lo = 0, hi = np;
    while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (P[mid] <= kQMax) lo = mid + 1; else hi = mid; }
    s_thr[0] = lo;
    hi = np;
    while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (P[mid] <= TA) lo = mid + 1; else hi = mid; }
    s_thr[1] = lo;
    hi = np;
    while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (P[mid] <= LS) lo = mid + 1; else hi = mid; }
    s_thr[2] = min(lo, s_thr[0] + kMidCap);
  }
  if (tid < 256) {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
      const uint32_t rho = (uint32_t)(wa.rho_pack >> (5 * i)) & 31u;
      if (tid & (1u << i)) v |= 1u << ((rho - 1) >> 1);
    }
    s_lut[tid] = v;
  }
  __syncthreads();
  const uint32_t i_mid0 = s_thr[0], i_midB = s_thr[1], i_mid1 = s_thr[2];
  for (uint32_t i = tid; i < i_mid1 - i_mid0; i += NT) {
    s_mid_p[i] = P[i_mid0 + i];
    s_mid_m[i] = M[i_mid0 + i];
  }
  // work units: S1 = nA single mid primes + nB diagonal units (8 primes each),
  // S2 = nL large units (64 primes each); S1 and S2 interleaved
  const uint32_t nA = i_midB - i_mid0;
  const uint32_t n_mid = i_mid1 - i_mid0;
  const uint32_t nB = (i_mid1 - i_midB + 7) / 8;
  const uint32_t nL = (np - i_mid1 + 63) / 64;
  const uint32_t nS1 = nA + nB, nS2 = nL;
  const uint32_t nI = min(nS1, nS2);
  const uint32_t n_units = nS1 + nS2;

  const uint64_t out_words = 2ull * ((wa.nbits + 63) / 64);  // 32-bit words of the caller's mask
  const uint64_t nseg = (wa.nbits + kWheelOutBits - 1) / kWheelOutBits;
  unsigned long long my_count = 0;

  for (uint64_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const uint64_t Vs = wa.V0 + s * kWheelSpan;  // segment base value
    const uint64_t Vend = Vs + kWheelSpan;

    // ---- 1. init: small-prime patterns (7..61) -------------------------
    {
      const uint32_t C = lane, pl = lane >> 3, c = lane & 7;
      const uint32_t rho = (uint32_t)(wa.rho_pack >> (5 * pl)) & 31u;
      const uint32_t r0 = wave * (ROWS / NW);              // 32 rows per wave
      const uint32_t k0 = c * LS + 32 * r0;                // first period of the lane's words
      uint32_t res[kNQ];
#pragma unroll
      for (int j = 0; j < kNQ; ++j) {
        const uint32_t q = kQ[j];
        // (Vs + rho + 30 k0) mod q, Vs = V0 + s*W
        const uint32_t wq = (uint32_t)(kWheelSpan % q);
        const uint32_t sq = (uint32_t)(s % q);
        const uint32_t x = ((uint32_t)wa.v0q[j] + sq * wq + rho + (30u * k0) % q) % q;
        const uint32_t u = x ? q - x : 0u;
        res[j] = (u * inv30_const(q)) % q;                 // first k >= k0 with q | value, minus k0
      }
      const bool on = phases & kPhaseSmall;
#pragma unroll 2
      for (uint32_t r = 0; r < ROWS / NW; r += 2) {
        uint64_t w = 0;
#pragma unroll
        for (int j = 0; j < kNQ; ++j) {
          const uint32_t q = kQ[j];
          const uint32_t d = 64 % q;
          w |= pat64(q) << res[j];
          res[j] = res[j] >= d ? res[j] - d : res[j] + q - d;
        }
        if (!on) w = 0;
        seg[(r0 + r) * 64 + C] = (uint32_t)w;
        seg[(r0 + r + 1) * 64 + C] = (uint32_t)(w >> 32);
      }
      if (tid == 0) s_ctr = 0;
    }
    __syncthreads();

    // ---- 2. mark -------------------------------------------------------
    for (;;) {
      uint32_t u = 0;
      if (lane == 0) u = atomicAdd(&s_ctr, 1u);
      u = __builtin_amdgcn_readlane(u, 0);
      if (u >= n_units) break;
      bool in_s1;
      uint32_t k;
      if (u < 2 * nI) { in_s1 = !(u & 1); k = u >> 1; }
      else { in_s1 = nS1 > nS2; k = u - nI; }

      if (in_s1 && k < nA) {
        if (!(phases & kPhaseMidA)) continue;
        // one prime per wave; lane L = column L = (plane L>>3, column L&7)
        const uint32_t p = __builtin_amdgcn_readfirstlane(s_mid_p[k]);
        const uint64_t p2 = (uint64_t)p * p;
        if (p2 >= Vend) continue;
        const uint64_t m = s_mid_m[k];
        const uint32_t Xs = mod_barrett(Vs, p, m);
        const float invp = fast_rcp((float)p);
        const uint32_t pl = lane >> 3, c = lane & 7;
        const uint32_t rho = (uint32_t)(wa.rho_pack >> (5 * pl)) & 31u;
        const uint32_t kp = plane_first(Xs, rho, p, (uint32_t)inv30_of(p), invp);
        uint32_t* const colp = seg + lane;
        if (p2 <= Vs) {
          const uint32_t cm = mod_small(c * LS, p, invp);
          uint32_t off = kp >= cm ? kp - cm : kp + p - cm;
          const uint32_t n_full = div_small(LS, p, invp);
#pragma unroll 4
          for (uint32_t h = 0; h < n_full; ++h) {
            lds_or(colp + ((off >> 5) << 6), 1u << (off & 31));
            off += p;
          }
          if (off < LS) lds_or(colp + ((off >> 5) << 6), 1u << (off & 31));
        } else {
          const uint32_t kmin = kmin_for((uint32_t)(p2 - Vs), rho);
          const uint32_t kf = first_at_or_after(kp, max(kmin, c * LS), p, invp);
          for (uint32_t off = kf - c * LS; off < LS; off += p) lds_or(colp + ((off >> 5) << 6), 1u << (off & 31));
        }
      } else if (in_s1) {
        if (!(phases & kPhaseMidB)) continue;
        // 8 primes x 8 planes: half-wave g takes planes 4g..4g+3; lane
        // (prime jp, plane pl) walks columns jp, jp+1, ... (mod 8)
        const uint32_t j0 = nA + (k - nA) * 8;
        const uint32_t nj = min(8u, n_mid - j0);
        const uint32_t pfirst = __builtin_amdgcn_readfirstlane(s_mid_p[j0]);
        if ((uint64_t)pfirst * pfirst >= Vend) continue;
        const uint32_t l = lane & 31;
        const uint32_t pl = 4 * (lane >> 5) + (l & 3), jp = l >> 2;
        const bool valid = jp < nj;
        const uint32_t p = valid ? s_mid_p[j0 + jp] : pfirst;
        const uint64_t m = s_mid_m[valid ? j0 + jp : j0];
        const float invp = fast_rcp((float)p);
        const uint32_t rho = (uint32_t)(wa.rho_pack >> (5 * pl)) & 31u;
        const uint32_t Xs = mod_barrett(Vs, p, m);
        const uint32_t kp = plane_first(Xs, rho, p, (uint32_t)inv30_of(p), invp);
        const uint64_t p2 = (uint64_t)p * p;
        uint32_t O0, off;
        const uint32_t cstart = jp * LS;
        const bool slow = p2 > Vs;
        if (!slow) {
          O0 = kp;
          const uint32_t cm = mod_small(cstart, p, invp);
          off = kp >= cm ? kp - cm : kp + p - cm;
        } else {
          const uint32_t kmin = p2 >= Vend ? KP : kmin_for((uint32_t)(p2 - Vs), rho);
          O0 = first_at_or_after(kp, kmin, p, invp);
          off = first_at_or_after(kp, max(kmin, cstart), p, invp) - cstart;
        }
        const uint32_t pmin = pfirst;
        const uint32_t pmax = __builtin_amdgcn_readfirstlane(s_mid_p[j0 + nj - 1]);
        const bool any_slow = __builtin_amdgcn_ballot_w64(slow) != 0;
        const uint32_t n_u = any_slow ? 0u : div_small(LS, pmax, fast_rcp((float)pmax));
        const uint32_t n_x = div_ceil_small(LS, pmin, fast_rcp((float)pmin)) - n_u;
        const uint32_t cb = 8 * pl;
        // lanes past the batch end mark nothing (their unconditional marks would
        // land in another prime's columns)
        if (!valid) {
        } else if (n_u >= 1 && n_u <= 15 && n_x >= 1 && n_x <= 2) {
          diag_dispatch<1>(n_u, n_x, seg, off, p, cb, jp, O0);
        } else {
          uint32_t c = jp;
          for (uint32_t t = 0; t < 8; ++t) {
            uint32_t* colp = seg + cb + c;
            for (uint32_t h = 0; h < n_u; ++h) {
              lds_or(colp + ((off >> 5) << 6), 1u << (off & 31));
              off += p;
            }
            for (uint32_t h = 0; h < n_x; ++h) {
              const bool hit = off < LS;
              const uint32_t o = hit ? off : 0u;
              lds_or(colp + ((o >> 5) << 6), hit ? 1u << (o & 31) : 0u);
              off = hit ? off + p : off;
            }
            off -= LS;
            c = (c + 1) & 7;
            off = c == 0 ? O0 : off;
          }
        }
      } else {
        if (!(phases & kPhaseLarge)) continue;
        // 64 primes > LS, one per lane, planes in a lane-rotated order
        const uint32_t base = i_mid1 + k * 64;
        const uint32_t p0 = __builtin_amdgcn_readfirstlane(P[base]);
        if ((uint64_t)p0 * p0 >= Vend) continue;
        const uint32_t il = base + lane;
        const bool ok = il < np;
        const uint32_t p = ok ? P[il] : 0x7FFFFFFFu;
        const uint64_t m = ok ? M[il] : 1ull;
        const uint64_t p2 = (uint64_t)p * p;
        const bool live = ok && p2 < Vend;
        const bool slow = p2 > Vs;
        const uint32_t D = slow && live ? (uint32_t)(p2 - Vs) : 0u;
        const uint64_t Kb = wa.KB0 + s * (uint64_t)KP;
        const uint32_t Kbm = ok ? mod_barrett(Kb, p, m) : 0u;
        const float invp = fast_rcp((float)p);
        const uint32_t pmax = __builtin_amdgcn_readlane(p, 63);
        const bool none = __builtin_amdgcn_ballot_w64(!live || slow) != 0;
        const uint32_t n_min = (none || pmax >= KP) ? 0u : div_small(KP - pmax, pmax, fast_rcp((float)pmax));
        uint32_t av[8];
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
          const uint32_t pl = (q + lane) & 7;
          av[q] = live ? A[8ull * il + ((wa.iota_pack >> (3 * pl)) & 7u)] : 0u;
        }
        if (live) {
#pragma unroll
          for (uint32_t q = 0; q < 8; ++q) {
            const uint32_t pl = (q + lane) & 7;
            const uint32_t e = (wa.e_bits >> pl) & 1u;
            int32_t kr = (int32_t)av[q] - (int32_t)Kbm - (int32_t)e;
            kr = kr < 0 ? kr + (int32_t)p : kr;
            kr = kr < 0 ? kr + (int32_t)p : kr;
            uint32_t kk = (uint32_t)kr;
            if (slow) {
              const uint32_t rho = (uint32_t)(wa.rho_pack >> (5 * pl)) & 31u;
              const uint32_t kmin = kmin_for(D, rho);
              if (kmin > kk) {
                const uint32_t d = kmin - kk;  // < 2^18
                uint32_t qd = (uint32_t)((float)d * invp);
                while (qd * p < d) ++qd;
                while (qd > 0 && (qd - 1) * p >= d) --qd;
                kk += qd * p;
              }
            }
            uint32_t* const pb = seg + 8 * pl;
#pragma unroll 2
            for (uint32_t h = 0; h < n_min; ++h) {
              lds_or(pb + ((kk >> 5) & (ROWS - 1)) * 64 + (kk >> LOG_LS), 1u << (kk & 31));
              kk += p;
            }
            for (; kk < KP; kk += p) lds_or(pb + ((kk >> 5) & (ROWS - 1)) * 64 + (kk >> LOG_LS), 1u << (kk & 31));
          }
        }
      }
    }
    __syncthreads();

    // ---- 3. expand to odd-only bits, count, store ------------------------
    {
      const uint32_t c = lane >> 3, a8 = lane & 7;
      const uint64_t seg_word0 = s * (uint64_t)kOutWordsPerSeg;
#pragma unroll 1
      for (uint32_t t = 0; t < ROWS / (NW * 8); ++t) {
        const uint32_t row = 8 * ((ROWS / (NW * 8)) * wave + t) + a8;
        const uint32_t* rp = seg + row * 64 + c;
        uint32_t Pw[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) Pw[j] = ~rp[8 * ((j + a8) & 7)];  // plane (j + a8) & 7, 1 = prime
        // un-rotate: plane i = Pw[(i - a8) & 7]
#pragma unroll
        for (uint32_t b = 1; b < 8; b <<= 1) {
          uint32_t T[8];
#pragma unroll
          for (uint32_t i = 0; i < 8; ++i) T[i] = (a8 & b) ? Pw[(i - b) & 7] : Pw[i];
#pragma unroll
          for (uint32_t i = 0; i < 8; ++i) Pw[i] = T[i];
        }
        uint32_t o[15];
#pragma unroll
        for (int w = 0; w < 15; ++w) o[w] = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
          uint32_t lo = 0, hi = 0;
#pragma unroll
          for (uint32_t i = 0; i < 4; ++i) {
            lo |= ((Pw[i] >> (8 * q)) & 0xFFu) << (8 * i);
            hi |= ((Pw[i + 4] >> (8 * q)) & 0xFFu) << (8 * i);
          }
          const uint64_t x = transpose8((uint64_t)lo | ((uint64_t)hi << 32));
#pragma unroll
          for (uint32_t bb = 0; bb < 8; ++bb) {
            const uint32_t e = s_lut[(uint32_t)(x >> (8 * bb)) & 0xFFu];
            const uint32_t pos = 15 * (8 * q + bb);
            o[pos >> 5] |= e << (pos & 31);
            if ((pos & 31) > 17) o[(pos >> 5) + 1] |= e >> (32 - (pos & 31));
          }
        }
        const uint64_t w0 = seg_word0 + 15ull * (c * ROWS + row);  // caller's 32-bit word index
        if (s == 0 && c == 0 && row == 0) o[0] |= wa.fix0;
        const uint64_t bit0 = 32ull * w0;
        if (bit0 + 480 > wa.nbits) {
#pragma unroll
          for (int w = 0; w < 15; ++w) {
            const uint64_t b = bit0 + 32ull * w;
            o[w] = b >= wa.nbits ? 0u : (wa.nbits - b >= 32 ? o[w] : o[w] & ((1u << (wa.nbits - b)) - 1u));
          }
        }
#pragma unroll
        for (int w = 0; w < 15; ++w) my_count += (unsigned long long)__popc(o[w]);
        if (out && (phases & kPhaseStore)) {
          if (w0 + 15 <= out_words) {
#pragma unroll
            for (int w = 0; w < 15; ++w) out[w0 + w] = o[w];
          } else {
#pragma unroll
            for (int w = 0; w < 15; ++w)
              if (w0 + w < out_words) out[w0 + w] = o[w];
          }
        }
      }
    }
    __syncthreads();
  }

#pragma unroll
  for (int o = 32; o > 0; o >>= 1) my_count += __shfl_xor(my_count, o);
  if (lane == 0) s_wave_cnt[wave] = my_count;
  __syncthreads();
  if (tid == 0) {
    unsigned long long t = 0;
    for (uint32_t w = 0; w < NW; ++w) t += s_wave_cnt[w];
    if (t) atomicAdd(count_out, t);
  }
}

// a[8i+j] = first k >= 0 with p | R30[j] + 30k, for every table prime >= 7.
__global__ void wheel_offsets_kernel(void* __restrict__ table) {
  const TableHeader* h = reinterpret_cast<const TableHeader*>(table);
  const uint32_t n = h->count == 0xFFFFFFFFu ? 0u : h->count;
  const uint32_t* P = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + 16);
  const uint64_t* M = reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(table) + table_m_offset(h->cap));
  uint32_t* A = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(table) + table_a_offset(h->cap));
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t p = P[i];
    if (p < 7) {
#pragma unroll
      for (int j = 0; j < 8; ++j) A[8ull * i + j] = 0;
      continue;
    }
    const uint64_t m = M[i];
    const uint64_t inv = inv30_of(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t t = kR30[j] % p;
      const uint32_t u = t ? p - t : 0u;
      A[8ull * i + j] = mod_barrett((uint64_t)u * inv, p, m);
    }
  }
}

}  // namespace

hipError_t launch_wheel_offsets(void* table, int num_cus, hipStream_t stream) {
  hipLaunchKernelGGL(wheel_offsets_kernel, dim3(4 * (uint32_t)num_cus), dim3(256), 0, stream, table);
  return hipGetLastError();
}

hipError_t launch_sieve_range_wheel(const void* table, uint64_t g_start, uint64_t nbits, uint32_t* out,
                                    unsigned long long* count, int num_cus, hipStream_t stream) {
  if (nbits == 0) return hipSuccess;
  static const uint32_t phases = [] {
    const char* e = getenv("DSE_PHASES");  // profiling-only ablation knob
    return e ? (uint32_t)strtoul(e, nullptr, 0) & kPhaseAll : kPhaseAll;
  }();
  WheelArgs wa{};
  const uint64_t v_start = 3 + 2 * g_start;
  wa.V0 = v_start - 1;
  wa.nbits = nbits;
  wa.KB0 = wa.V0 / 30;
  const uint32_t v0m = (uint32_t)(wa.V0 % 30);
  uint32_t n = 0;
  for (uint32_t rho = 1; rho < 30; rho += 2) {
    const uint32_t r = (v0m + rho) % 30;
    if (r % 3 == 0 || r % 5 == 0) continue;
    uint32_t iota = 0;
    while (kR30[iota] != r) ++iota;
    wa.rho_pack |= (uint64_t)rho << (5 * n);
    wa.iota_pack |= iota << (3 * n);
    if (v0m + rho >= 30) wa.e_bits |= 1u << n;
    ++n;
  }
  if (n != 8) return hipErrorInvalidValue;
  // primes 3..61 inside the range: the wheel drops 3 and 5, the patterns mark 7..61 themselves
  constexpr uint32_t small[] = {3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61};
  for (uint32_t v : small)
    if (v >= v_start && (v - v_start) / 2 < nbits) wa.fix0 |= 1u << ((v - v_start) / 2);
  for (int j = 0; j < kNQ; ++j) wa.v0q[j] = (uint8_t)(wa.V0 % kQ[j]);
  wa.phases = phases;
  const uint64_t nseg = (nbits + kWheelOutBits - 1) / kWheelOutBits;
  const uint64_t grid = nseg < (uint64_t)num_cus ? nseg : (uint64_t)num_cus;
  hipLaunchKernelGGL(wheel_segments_kernel, dim3((uint32_t)grid), dim3(NT), 0, stream, table, wa, out, count);
  return hipGetLastError();
}

// Kernel choice: the wheel kernel for base primes up to kWheelMaxPrime (every
// configured N up to 4.4e12), the odd-only kernel above (high-offset windows).
hipError_t launch_sieve_range(const void* table, uint64_t g_start, uint64_t nbits, uint32_t* out,
                              unsigned long long* count, int num_cus, hipStream_t stream) {
  if (nbits == 0) return hipSuccess;
  static const int force = [] {
    const char* e = getenv("DSE_KERNEL");  // profiling-only: "odd" or "wheel"
    if (!e) return 0;
    return e[0] == 'o' ? 1 : e[0] == 'w' ? 2 : 0;
  }();
  const uint64_t vmax = 3 + 2 * (g_start + nbits - 1);
  uint64_t r = (uint64_t)__builtin_sqrt((double)vmax);
  while (r * r > vmax) --r;
  while ((r + 1) * (r + 1) <= vmax) ++r;
  const bool wheel = force ? force == 2 : r <= kWheelMaxPrime;
  return wheel ? launch_sieve_range_wheel(table, g_start, nbits, out, count, num_cus, stream)
               : launch_sieve_range_odd(table, g_start, nbits, out, count, num_cus, stream);
}

}  // namespace dse

// dse_kernels.hip -- gfx950 (MI355X) kernels for the chunked odd-only sieve.
//
// Replaces the reference's per-prime serial loop (sieve.clj:118-172:
// find-next-non-zero -> broadcast [mi ps p] -> mark-composites' lazy index walk
// with assoc! ... 0) by an LDS-resident segmented sieve. Bit j of a range
// stands for the odd value 3+2(g_start+j), exactly the reference's element j of
// its chunk vector (sieve.clj:9-13); a set bit in the output = "element still
// non-zero" = prime.
//
// Per 2^20-candidate segment, one 1024-thread workgroup (one per CU, 128 KiB LDS):
//   1. zero the LDS segment (ds_write_b128);
//   2. mark composites with ds_or_b32, work handed out dynamically to waves:
//      - "mid" primes 61 < p <= LS: one prime per wave, lane L walks its own
//        column L (a contiguous LS-bit sub-segment stored in LDS bank L mod 32),
//        so every wave-instruction is bank-conflict-free;
//      - "large" primes p > LS: one prime per lane, <= SEG/p hits each;
//   3. write back: lane L reads 4 rows of its column (conflict-free), ORs in the
//      register patterns of the primes 3..61, inverts, masks the range end,
//      popcounts, stores 16 B; the block count goes to one 64-bit atomic.
// See DESIGN.md for the LDS layout and the rooflines.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "dse_internal.h"

namespace dse {
namespace {

constexpr uint32_t kPhaseMidA = 1, kPhaseMidB = 2, kPhaseLarge = 4, kPhaseSmall = 8, kPhaseStore = 16,
                   kPhaseScatter = 32;
constexpr uint32_t kPhaseAll = 63;

constexpr int kNumSmall = 17;
constexpr uint32_t kSmall[kNumSmall] = {3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61};

constexpr uint64_t pat64(uint32_t q) {
  uint64_t v = 0;
  for (uint32_t k = 0; k < 64; k += q) v |= 1ull << k;
  return v;
}
// Bits at the odd indices (q-3)/2 of the small primes themselves: their own
// pattern marks them, the reference keeps them (they are primes).
constexpr uint64_t small_self_bits() {
  uint64_t v = 0;
  for (int i = 0; i < kNumSmall; ++i) v |= 1ull << ((kSmall[i] - 3) / 2);
  return v;
}

__device__ __forceinline__ void lds_or(uint32_t* a, uint32_t v) {
  __hip_atomic_fetch_or(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// x mod p for x < 2^63 with m = floor((2^64-1)/p).
__device__ __forceinline__ uint32_t mod_barrett(uint64_t x, uint32_t p, uint64_t m) {
  uint64_t q = __umul64hi(x, m);
  uint64_t r = x - q * p;
  if (r >= p) r -= p;
  if (r >= p) r -= p;
  return (uint32_t)r;
}

// t mod p for t/p < 2^16, t < 2^24, via a float reciprocal and one fix-up.
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }  // ~1 ulp; users correct

__device__ __forceinline__ uint32_t mod_small(uint32_t t, uint32_t p, float invp) {
  uint32_t q = (uint32_t)((float)t * invp);
  int32_t r = (int32_t)(t - q * p);
  r = r < 0 ? r + (int32_t)p : r;
  r = r >= (int32_t)p ? r - (int32_t)p : r;
  return (uint32_t)r;
}


// Per-column marking of one mid prime (p <= LS) in the fast case (p^2 at or
// before the segment): lane L = column L starts at the first multiple at or
// after G + L*LS. A = (G - g0) mod p, c = LS mod p (both wave-uniform).
template <uint32_t LS>
__device__ __forceinline__ void mark_column(uint32_t* __restrict__ col, uint32_t lane, uint32_t p, uint32_t A,
                                            uint32_t c, float invp) {
  const uint32_t d = mod_small(A + lane * c, p, invp);  // (G + L*LS - g0) mod p
  uint32_t off = d ? p - d : 0;
  // every lane has floor(LS/p) hits, some one more: uniform loop + one predicated
  const uint32_t n_full = (uint32_t)((float)(LS - c) * invp + 0.5f);
#pragma unroll 4
  for (uint32_t k = 0; k < n_full; ++k) {
    lds_or(col + ((off >> 5) << 6), 1u << (off & 31));
    off += p;
  }
  if (off < LS) lds_or(col + ((off >> 5) << 6), 1u << (off & 31));
}

// Slow case (p^2 inside or after this segment's start): per-lane offsets.
template <uint32_t LS>
__device__ __forceinline__ void mark_column_slow(uint32_t* __restrict__ col, uint32_t lane, uint32_t p, uint64_t m,
                                                 uint64_t g0, uint64_t G) {
  const uint64_t GL = G + (uint64_t)lane * LS;
  uint32_t off;
  if (g0 >= GL) {
    const uint64_t t = g0 - GL;
    off = t >= LS ? LS : (uint32_t)t;
  } else {
    const uint32_t d = mod_barrett(GL - g0, p, m);
    off = d ? p - d : 0;
  }
  for (; off < LS; off += p) lds_or(col + ((off >> 5) << 6), 1u << (off & 31));
}


// floor(t / p) for t < 2^24 via a float reciprocal, corrected.
__device__ __forceinline__ uint32_t div_small(uint32_t t, uint32_t p, float invp) {
  uint32_t q = (uint32_t)((float)t * invp);
  const uint32_t qp = q * p;
  q = qp > t ? q - 1 : q;
  q = (q + 1) * p <= t ? q + 1 : q;
  return q;
}


// 16 diagonal column steps of one lane's prime with compile-time hit counts:
// NU unconditional marks and NX value-predicated ones (OR 0 into the lane's
// own column when past the column end) per column; no inner-loop control.
template <uint32_t LS, int NU, int NX>
__device__ __forceinline__ void diag_walk(char* __restrict__ segb, uint32_t off, uint32_t p, uint32_t c4,
                                          uint32_t O0, bool valid) {
#pragma unroll 2
  for (uint32_t t = 0; t < 16; ++t) {
#pragma unroll
    for (int h = 0; h < NU; ++h) {
      lds_or(reinterpret_cast<uint32_t*>(segb + (((off >> 5) << 8) | c4)), 1u << (off & 31));
      off += p;
    }
#pragma unroll
    for (int h = 0; h < NX; ++h) {
      const bool hit = off < LS;
      const uint32_t o = hit ? off : 0u;
      lds_or(reinterpret_cast<uint32_t*>(segb + (((o >> 5) << 8) | c4)), hit ? 1u << (o & 31) : 0u);
      off = hit ? off + p : off;
    }
    off -= LS;
    c4 = (c4 + 4) & 255;
    off = (c4 == 0 && valid) ? O0 : off;  // wrapped from column 63 to column 0
  }
}

template <uint32_t LS, int U>
__device__ __forceinline__ void diag_dispatch(uint32_t n_u, uint32_t n_x, char* __restrict__ segb, uint32_t off,
                                              uint32_t p, uint32_t c4, uint32_t O0, bool valid) {
  if constexpr (U <= 15) {
    if (n_u == U) {
      if (n_x == 1) diag_walk<LS, U, 1>(segb, off, p, c4, O0, valid);
      else diag_walk<LS, U, 2>(segb, off, p, c4, O0, valid);
      return;
    }
    diag_dispatch<LS, U + 1>(n_u, n_x, segb, off, p, c4, O0, valid);
  }
}

// mid primes staged in LDS: odd primes in (61, LS] (16384: 1882, 8192: 1009)
template <uint32_t LS>
constexpr uint32_t max_mid() { return LS >= 16384 ? 1920u : LS >= 8192 ? 1024u : 512u; }

template <int LOG_SEG, int NT>
__global__ __launch_bounds__(NT) void sieve_segments_kernel(const void* __restrict__ table,
                                                           uint64_t g_start, uint64_t nbits,
                                                           uint32_t* __restrict__ out,
                                                           unsigned long long* __restrict__ count_out,
                                                           uint32_t phases) {
  constexpr uint32_t SEG = 1u << LOG_SEG;      // odd candidates per segment
  constexpr uint32_t LOG_LS = LOG_SEG - 6;
  constexpr uint32_t LS = 1u << LOG_LS;        // candidates per column (64 columns)
  constexpr uint32_t ROWS = LS / 32;           // 32-bit words per column
  constexpr uint32_t NW = NT / 64;
  constexpr uint32_t ROWS_PER_WAVE = ROWS / NW;
  constexpr uint32_t TA = LS / 16;             // mid primes <= TA: one per grab (>= 16 hits per column)
  static_assert(ROWS_PER_WAVE % 4 == 0, "write-back handles 4 rows per step");

  __shared__ __attribute__((aligned(16))) uint32_t seg[SEG / 32];
  constexpr uint32_t kMaxMid = max_mid<LS>();
  __shared__ uint64_t s_mid_m[kMaxMid];
  __shared__ uint32_t s_mid_p[kMaxMid];
  __shared__ uint32_t s_ctr;
  __shared__ uint32_t s_thr[4];
  __shared__ unsigned long long s_wave_cnt[NW];

  const TableHeader* th = reinterpret_cast<const TableHeader*>(table);
  const uint32_t np = th->count;
  const uint32_t* __restrict__ P = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + 16);
  const uint64_t* __restrict__ M =
      reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(table) + table_m_offset(th->cap));

  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  if (tid == 0) {
    // first index with p > kSmallMax, with p > TA, with p > LS
    uint32_t lo = 0, hi = np;
    while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (P[mid] <= (uint32_t)kSmallMax) lo = mid + 1; else hi = mid; }
    s_thr[0] = lo;
    hi = np;
    while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (P[mid] <= TA) lo = mid + 1; else hi = mid; }
    s_thr[1] = lo;
    hi = np;
    while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (P[mid] <= LS) lo = mid + 1; else hi = mid; }
    s_thr[2] = min(lo, s_thr[0] + kMaxMid);  // anything beyond the LDS stage goes to the large path
    lo = s_thr[2];
    hi = np;
    while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (P[mid] <= 4 * LS) lo = mid + 1; else hi = mid; }
    s_thr[3] = lo;
  }
  __syncthreads();
  const uint32_t i_mid0 = s_thr[0], i_midA = s_thr[1], i_mid1 = s_thr[2];
  for (uint32_t i = tid; i < i_mid1 - i_mid0; i += NT) {
    s_mid_p[i] = P[i_mid0 + i];
    s_mid_m[i] = M[i_mid0 + i];
  }
  // Work units, handed out dynamically. S1 = LDS-issue-bound: nA single mid
  // primes (p <= TA, one per wave), then nB diagonal units (64 mid primes x 16
  // columns). S2 = large primes: nC cooperative units (64 primes in (LS, 4LS],
  // a lane per hit), then nD scatter units (256 primes > 4LS, 4 per lane).
  // S1 and S2 are interleaved so that waves waiting on global loads overlap
  // waves marking.
  const uint32_t i_big = s_thr[3];
  const uint32_t nA = i_midA - i_mid0;
  const uint32_t nBb = (i_mid1 - i_midA + 63) / 64;  // batches of 64
  const uint32_t nB = nBb * 4;                       // x 4 column quarters
  const uint32_t nC = (i_big - i_mid1 + 63) / 64;
  const uint32_t nD = (np - i_big + 255) / 256;
  const uint32_t nS1 = nA + nB, nS2 = nC + nD;
  const uint32_t nI = min(nS1, nS2);  // interleaved pairs
  const uint32_t n_units = nS1 + nS2;
  const uint32_t n_mid = i_mid1 - i_mid0;

  const uint64_t out_words = 2ull * ((nbits + 63) / 64);  // 32-bit words of the caller's mask
  const uint64_t nseg = (nbits + SEG - 1) / SEG;
  unsigned long long my_count = 0;
  uint32_t* const col = seg + lane;
  char* const segb = reinterpret_cast<char*>(seg);

  for (uint64_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const uint64_t G = g_start + s * SEG;  // global odd index of segment bit 0
    const uint64_t seg_end = G + SEG;

    // ---- 1. zero -------------------------------------------------------
    {
      uint4* s4 = reinterpret_cast<uint4*>(seg);
#pragma unroll
      for (uint32_t i = tid; i < SEG / 128; i += NT) s4[i] = make_uint4(0u, 0u, 0u, 0u);
      if (tid == 0) s_ctr = 0;
    }
    __syncthreads();

    // ---- 2. mark -------------------------------------------------------
    for (;;) {
      uint32_t u = 0;
      if (lane == 0) u = atomicAdd(&s_ctr, 1u);
      u = __builtin_amdgcn_readlane(u, 0);
      if (u >= n_units) break;
      // map u -> (list, index)
      bool in_s1;
      uint32_t k;
      if (u < 2 * nI) { in_s1 = !(u & 1); k = u >> 1; }
      else { in_s1 = nS1 > nS2; k = u - nI; }
      if (in_s1 && k < nA) {
        if (!(phases & kPhaseMidA)) continue;
        // one mid prime (p <= TA) for the whole wave, lane L = column L
        const uint32_t p = s_mid_p[k];
        const uint64_t m = s_mid_m[k];
        const uint64_t g0 = ((uint64_t)p * p - 3) >> 1;  // index of p^2
        if (g0 >= seg_end) continue;
        if (g0 <= G) {
          const float invp = fast_rcp((float)p);
          mark_column<LS>(col, lane, p, mod_barrett(G - g0, p, m), mod_small(LS, p, invp), invp);
        } else {
          mark_column_slow<LS>(col, lane, p, m, g0, G);
        }
      } else if (in_s1) {
        if (!(phases & kPhaseMidB)) continue;
        // 64 mid primes x 16 columns, lane j = prime j, walked diagonally: at
        // step t lane j is in column (j+16q+t) mod 64, so every ds_or hits a
        // distinct column (bank = column mod 32) and the column-to-column
        // hand-over of the offset is free.
        const uint32_t kb = k - nA, q = kb & 3;
        const uint32_t j0 = nA + (kb >> 2) * 64;
        const uint32_t nj = min(64u, n_mid - j0);
        if ((((uint64_t)s_mid_p[j0] * s_mid_p[j0] - 3) >> 1) >= seg_end) continue;
        const bool valid = lane < nj;
        const uint32_t p = valid ? s_mid_p[j0 + lane] : 0x7FFFFFFFu;
        uint32_t O0 = SEG;  // first hit at or after G, relative to G (SEG: none)
        if (valid) {
          const uint64_t g0 = ((uint64_t)p * p - 3) >> 1;
          if (g0 <= G) {
            const uint32_t A = mod_barrett(G - g0, p, s_mid_m[j0 + lane]);
            O0 = A ? p - A : 0;
          } else if (g0 < seg_end) {
            O0 = (uint32_t)(g0 - G);
          }
        }
        const float invp = fast_rcp((float)p);
        const uint32_t c0 = (lane + 16 * q) & 63;
        const uint32_t cstart = c0 * LS;
        uint32_t off;
        if (O0 >= cstart) off = O0 - cstart;
        else { const uint32_t d = mod_small(cstart - O0, p, invp); off = d ? p - d : 0; }
        // a lane past p^2 with off < p has floor(LS/p)..ceil(LS/p) hits per
        // column: n_u unconditional marks + n_x value-predicated ones (OR 0)
        const uint32_t pmin = __builtin_amdgcn_readlane(p, 0);
        const uint32_t pmax = __builtin_amdgcn_readlane(p, nj - 1);
        const bool any_slow = __builtin_amdgcn_ballot_w64(valid && O0 >= p) != 0;
        const uint32_t n_u = any_slow ? 0u : div_small(LS, pmax, fast_rcp((float)pmax));
        const uint32_t n_x = div_small(LS + pmin - 1, pmin, fast_rcp((float)pmin)) - n_u;
        uint32_t c4 = c0 << 2;  // byte offset of the current column
        // lanes past the batch end do no marks at all (their unconditional
        // marks would address outside the segment)
        if (!valid) {
        } else if (n_u >= 1 && n_u <= 15 && n_x >= 1 && n_x <= 2) {
          diag_dispatch<LS, 1>(n_u, n_x, segb, off, p, c4, O0, valid);
        } else {
          for (uint32_t t = 0; t < 16; ++t) {
            for (uint32_t h = 0; h < n_u; ++h) {
              lds_or(reinterpret_cast<uint32_t*>(segb + (((off >> 5) << 8) | c4)), 1u << (off & 31));
              off += p;
            }
            for (uint32_t h = 0; h < n_x; ++h) {
              const bool hit = off < LS;
              const uint32_t o = hit ? off : 0u;
              lds_or(reinterpret_cast<uint32_t*>(segb + (((o >> 5) << 8) | c4)), hit ? 1u << (o & 31) : 0u);
              off = hit ? off + p : off;
            }
            off -= LS;
            c4 = (c4 + 4) & 255;
            off = (c4 == 0 && valid) ? O0 : off;  // wrapped from column 63 to column 0
          }
        }
      } else if (k < nC) {
        if (!(phases & kPhaseLarge)) continue;
        // 64 primes in (LS, 4LS]: < 64 hits each per segment, at most one per
        // column. One prime per wave (p <= 2LS) or per half-wave, lane = hit
        // index: a half-wave's hits lie in distinct columns, so a bank (two
        // columns) sees at most two of them.
        const uint32_t i = i_mid1 + k * 64 + lane;
        const bool ok = i < i_big;
        const uint32_t pl = ok ? P[i] : 0u;
        uint32_t bl = SEG;
        if (ok) {
          const uint64_t g0 = ((uint64_t)pl * pl - 3) >> 1;
          if (g0 < seg_end) {
            if (g0 >= G) bl = (uint32_t)(g0 - G);
            else { const uint32_t d = mod_barrett(G - g0, pl, M[i]); bl = d ? pl - d : 0; }
          }
        }
        const uint32_t nj = min(64u, i_big - (i_mid1 + k * 64));
        const bool two = __builtin_amdgcn_readlane(pl, 0) > 2 * LS;  // sorted: the whole batch > 2LS
        if (!two) {
          for (uint32_t j = 0; j < nj; ++j) {
            const uint32_t p = __builtin_amdgcn_readlane(pl, j);
            const uint32_t b0 = __builtin_amdgcn_readlane(bl, j);
            const uint32_t b = b0 + lane * p;
            const uint32_t o = b & (LS - 1);
            if (b < SEG) lds_or(seg + ((o >> 5) << 6) + (b >> LOG_LS), 1u << (o & 31));
          }
        } else {
          const uint32_t hl = lane & 31;
          for (uint32_t j = 0; j < nj; j += 2) {
            const uint32_t pa = __builtin_amdgcn_readlane(pl, j), ba = __builtin_amdgcn_readlane(bl, j);
            const uint32_t jb = j + 1 < nj ? j + 1 : j;
            const uint32_t pb = __builtin_amdgcn_readlane(pl, jb), bbv = __builtin_amdgcn_readlane(bl, jb);
            const bool lo_half = lane < 32;
            const uint32_t p = lo_half ? pa : pb;
            const uint32_t b = (lo_half ? ba : (j + 1 < nj ? bbv : SEG)) + hl * p;
            const uint32_t o = b & (LS - 1);
            if (b < SEG) lds_or(seg + ((o >> 5) << 6) + (b >> LOG_LS), 1u << (o & 31));
          }
        }
      } else {
        if (!(phases & kPhaseScatter)) continue;
        // 256 primes > 4LS, 4 per lane, scattered anywhere in the segment
        const uint32_t base = i_big + (k - nC) * 256;
        uint32_t pr[4], b[4];
        uint64_t mr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t i = base + r * 64 + lane;
          pr[r] = i < np ? P[i] : 1u;
          mr[r] = i < np ? M[i] : 0ull;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t p = pr[r];
          const uint64_t g0 = ((uint64_t)p * p - 3) >> 1;
          uint32_t bb = SEG;
          if (p > 1 && g0 < seg_end) {
            if (g0 >= G) bb = (uint32_t)(g0 - G);
            else { const uint32_t d = mod_barrett(G - g0, p, mr[r]); bb = d ? p - d : 0; }
          }
          b[r] = bb;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t p = pr[r];
          uint32_t bb = b[r];
          // hits per lane differ little between neighbouring primes: run the
          // wave-wide minimum without exec-mask churn, then the remainder
          // every lane with its first hit bb < p <= pmax has > (SEG-pmax)/pmax
          // hits; any other lane (table end, p^2 inside or past the segment)
          // forces the divergent loop. No cross-lane reduction: a ds_bpermute
          // would wait for all of this wave's outstanding ds_or.
          const uint32_t pmax = __builtin_amdgcn_readlane(p, 63);
          const bool none = __builtin_amdgcn_ballot_w64(bb >= p) != 0;
          // (primes above SEG hit a segment at most once: divergent loop only)
          const uint32_t n_min = (none || pmax > SEG) ? 0u : div_small(SEG - pmax, pmax, fast_rcp((float)pmax));
#pragma unroll 2
          for (uint32_t h = 0; h < n_min; ++h) {
            const uint32_t o = bb & (LS - 1);
            lds_or(seg + ((o >> 5) << 6) + (bb >> LOG_LS), 1u << (o & 31));
            bb += p;
          }
          for (; bb < SEG; bb += p) {
            const uint32_t o = bb & (LS - 1);
            lds_or(seg + ((o >> 5) << 6) + (bb >> LOG_LS), 1u << (o & 31));
          }
        }
      }
    }
    __syncthreads();

    // ---- 3. write back ---------------------------------------------------
    {
      const uint32_t r0 = wave * ROWS_PER_WAVE;
      const uint32_t w0 = lane * ROWS + r0;               // natural 32-bit word in segment
      const uint64_t X0 = G + 32ull * w0;                 // global odd index of that word's bit 0
      // residue of the next multiple of each small prime q, relative to X0:
      // multiples of q have odd index == (q-3)/2 (mod q)
      uint32_t res[kNumSmall];
#pragma unroll
      for (int k = 0; k < kNumSmall; ++k) {
        const uint32_t q = kSmall[k];
        const uint32_t xm = (uint32_t)(X0 % q);
        const uint32_t cq = (q - 3) / 2;
        res[k] = (cq + q - xm) % q;
      }
      const uint64_t pos0 = s * SEG + 32ull * w0;         // position in the caller's range
#pragma unroll 2
      for (uint32_t r = 0; r < ROWS_PER_WAVE; r += 4) {
        const uint32_t* src = seg + (r0 + r) * 64 + lane;
        uint64_t lo = (uint64_t)src[0] | ((uint64_t)src[64] << 32);
        uint64_t hi = (uint64_t)src[128] | ((uint64_t)src[192] << 32);
#pragma unroll
        for (int k = 0; k < kNumSmall; ++k) {
          if (!(phases & kPhaseSmall)) break;
          const uint32_t q = kSmall[k];
          const uint32_t d64 = 64 % q;
          uint32_t t = res[k];
          lo |= pat64(q) << t;
          t = t >= d64 ? t - d64 : t + q - d64;
          hi |= pat64(q) << t;
          t = t >= d64 ? t - d64 : t + q - d64;
          res[k] = t;
        }
        const uint64_t X = X0 + 32ull * r;
        if (X < 64) lo &= ~(small_self_bits() >> X);
        lo = ~lo;
        hi = ~hi;
        const uint64_t pos = pos0 + 32ull * r;
        if (pos + 128 > nbits) {
          lo = pos >= nbits ? 0 : (nbits - pos >= 64 ? lo : lo & ((1ull << (nbits - pos)) - 1));
          hi = pos + 64 >= nbits ? 0 : (nbits - pos - 64 >= 64 ? hi : hi & ((1ull << (nbits - pos - 64)) - 1));
        }
        my_count += (unsigned long long)(__popcll(lo) + __popcll(hi));
        if (out && (phases & kPhaseStore)) {
          const uint64_t wi = pos >> 5;
          if (wi + 4 <= out_words) {
            *reinterpret_cast<uint4*>(out + wi) =
                make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
          } else {
            if (wi + 0 < out_words) out[wi + 0] = (uint32_t)lo;
            if (wi + 1 < out_words) out[wi + 1] = (uint32_t)(lo >> 32);
            if (wi + 2 < out_words) out[wi + 2] = (uint32_t)hi;
            if (wi + 3 < out_words) out[wi + 3] = (uint32_t)(hi >> 32);
          }
        }
      }
    }
    __syncthreads();
  }

  // ---- block count -> one 64-bit atomic --------------------------------
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

// ---------------------------------------------------------------------------
// Big base-prime tables (limit above kBaseLimitMax, e.g. 1e9 for the 1e18
// window): sieve [3, limit] with the segment kernel itself, then compact the
// prime bits into an ordered table. Scratch lives in the table's m[] region,
// which is only written at the very end.
// ---------------------------------------------------------------------------
constexpr uint32_t kCompactWordsPerThread = 2;
constexpr uint32_t kCompactThreads = 256;
constexpr uint32_t kCompactBlockWords = kCompactWordsPerThread * kCompactThreads;  // 512 words

__global__ __launch_bounds__(kCompactThreads) void compact_count_kernel(const uint64_t* __restrict__ mask,
                                                                        uint64_t words,
                                                                        uint32_t* __restrict__ block_sums) {
  __shared__ uint32_t s_part[kCompactThreads / 64];
  const uint64_t w0 = (uint64_t)blockIdx.x * kCompactBlockWords + threadIdx.x * kCompactWordsPerThread;
  uint32_t c = 0;
#pragma unroll
  for (uint32_t k = 0; k < kCompactWordsPerThread; ++k)
    if (w0 + k < words) c += __popcll(mask[w0 + k]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < kCompactThreads / 64; ++w) t += s_part[w];
    block_sums[blockIdx.x] = t;
  }
}

// exclusive scan of block sums in place; total -> table header count
__global__ __launch_bounds__(1024) void compact_scan_kernel(uint32_t* __restrict__ block_sums, uint32_t nblocks,
                                                            void* __restrict__ table, uint32_t cap, uint64_t limit) {
  __shared__ uint32_t s_scan[1024];
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (nblocks + 1023) / 1024;
  const uint32_t b0 = tid * per, b1 = min(nblocks, b0 + per);
  uint32_t sum = 0;
  for (uint32_t b = b0; b < b1; ++b) sum += block_sums[b];
  s_scan[tid] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    const uint32_t x = tid >= o ? s_scan[tid - o] : 0;
    __syncthreads();
    s_scan[tid] += x;
    __syncthreads();
  }
  uint32_t run = s_scan[tid] - sum;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t v = block_sums[b];
    block_sums[b] = run;
    run += v;
  }
  if (tid == 1023) {
    TableHeader* h = reinterpret_cast<TableHeader*>(table);
    const uint32_t total = s_scan[1023];
    h->count = total <= cap ? total : 0xFFFFFFFFu;
    h->cap = cap;
    h->limit = limit;
  }
}

__global__ __launch_bounds__(kCompactThreads) void compact_write_kernel(const uint64_t* __restrict__ mask,
                                                                        uint64_t words,
                                                                        const uint32_t* __restrict__ block_offs,
                                                                        uint32_t* __restrict__ P, uint32_t cap) {
  __shared__ uint32_t s_scan[kCompactThreads];
  const uint32_t tid = threadIdx.x;
  const uint64_t w0 = (uint64_t)blockIdx.x * kCompactBlockWords + tid * kCompactWordsPerThread;
  uint64_t v[kCompactWordsPerThread];
  uint32_t c = 0;
#pragma unroll
  for (uint32_t k = 0; k < kCompactWordsPerThread; ++k) {
    v[k] = w0 + k < words ? mask[w0 + k] : 0ull;
    c += __popcll(v[k]);
  }
  s_scan[tid] = c;
  __syncthreads();
  for (uint32_t o = 1; o < kCompactThreads; o <<= 1) {
    const uint32_t x = tid >= o ? s_scan[tid - o] : 0;
    __syncthreads();
    s_scan[tid] += x;
    __syncthreads();
  }
  uint32_t pos = block_offs[blockIdx.x] + s_scan[tid] - c;
#pragma unroll
  for (uint32_t k = 0; k < kCompactWordsPerThread; ++k) {
    uint64_t x = v[k];
    while (x) {
      const uint32_t b = __ffsll((long long)x) - 1;
      x &= x - 1;
      if (pos < cap) P[pos] = (uint32_t)(3 + 2 * ((w0 + k) * 64 + b));
      ++pos;
    }
  }
}

// ---------------------------------------------------------------------------
// Base primes up to kBaseLimitMax: many workgroups each sieve a slice of the
// odd values 3..limit in LDS by the odd primes q <= sqrt(limit) (each
// workgroup finds them by trial division: q <= 1568) and write the slice as
// prime bits; the ordered compaction above then builds p[].
// ---------------------------------------------------------------------------
constexpr uint32_t kBaseMaskThreads = 256;
constexpr uint32_t kBaseMaskMaxWords = 128;  // u64 words per workgroup slice

__global__ __launch_bounds__(kBaseMaskThreads) void base_mask_kernel(uint64_t limit, uint64_t* __restrict__ mask,
                                                                     uint32_t words, uint32_t wpw) {
  __shared__ uint32_t bm[2 * kBaseMaskMaxWords];
  const uint32_t tid = threadIdx.x;
  const uint32_t nb = (uint32_t)((limit - 3) / 2 + 1);  // odd values 3..limit
  const uint32_t w0 = blockIdx.x * wpw;
  const uint32_t nw = min(wpw, words - w0);
  for (uint32_t i = tid; i < 2 * nw; i += kBaseMaskThreads) bm[i] = 0;
  __syncthreads();
  const uint32_t g_lo = 64 * w0, g_hi = min(64 * (w0 + nw), nb);  // odd indices of this slice
  for (uint32_t t = tid;; t += kBaseMaskThreads) {
    const uint32_t q = 3 + 2 * t;
    if ((uint64_t)q * q > limit) break;
    bool pr = true;
    for (uint32_t d = 3; d * d <= q; d += 2)
      if (q % d == 0) { pr = false; break; }
    if (!pr) continue;
    // odd multiples v = q*m >= max(q^2, 3 + 2 g_lo): index (v - 3)/2, stride q
    const uint64_t vlo = 3 + 2ull * g_lo;
    uint64_t v = (uint64_t)q * q;
    if (v < vlo) {
      v = (vlo + q - 1) / q * q;
      if (!(v & 1)) v += q;
    }
    for (uint32_t g = (uint32_t)((v - 3) >> 1); g < g_hi; g += q) {
      const uint32_t r = g - g_lo;
      atomicOr(&bm[r >> 5], 1u << (r & 31));
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < nw; i += kBaseMaskThreads) {
    uint64_t v = ~((uint64_t)bm[2 * i] | ((uint64_t)bm[2 * i + 1] << 32));
    const uint32_t gb = 64 * (w0 + i);
    if (gb + 64 > nb) v = gb >= nb ? 0 : v & ((1ull << (nb - gb)) - 1);
    mask[w0 + i] = v;
  }
}

}  // namespace

hipError_t launch_base_primes(uint64_t limit, void* table, uint32_t cap, hipStream_t stream) {
  if (limit > kBaseLimitMax) return hipErrorInvalidValue;
  if (limit < 3) {  // no odd primes: empty table
    TableHeader h{0, cap, limit};
    return hipMemcpyAsync(table, &h, sizeof(h), hipMemcpyHostToDevice, stream);
  }
  // scratch carved from the table's m[]/a[] region (written last): [mask][block sums]
  char* mreg = reinterpret_cast<char*>(table) + table_m_offset(cap);
  const uint64_t nb = (limit - 3) / 2 + 1;
  const uint32_t words = (uint32_t)((nb + 63) / 64);
  uint64_t* mask = reinterpret_cast<uint64_t*>(mreg);
  const uint32_t nblocks = (words + kCompactBlockWords - 1) / kCompactBlockWords;
  uint32_t* sums = reinterpret_cast<uint32_t*>(mreg + ((words * 8ull + 255) & ~255ull));
  if ((uint64_t)(reinterpret_cast<char*>(sums + nblocks) - mreg) > 40ull * cap) return hipErrorInvalidValue;
  const uint32_t wpw = std::max<uint32_t>((words + 255) / 256, 1u);
  if (wpw > kBaseMaskMaxWords) return hipErrorInvalidValue;
  const uint32_t grid = (words + wpw - 1) / wpw;
  hipLaunchKernelGGL(base_mask_kernel, dim3(grid), dim3(kBaseMaskThreads), 0, stream, limit, mask, words, wpw);
  hipLaunchKernelGGL(compact_count_kernel, dim3(nblocks), dim3(kCompactThreads), 0, stream, mask, (uint64_t)words,
                     sums);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, stream, sums, nblocks, table, cap, limit);
  uint32_t* P = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(table) + 16);
  hipLaunchKernelGGL(compact_write_kernel, dim3(nblocks), dim3(kCompactThreads), 0, stream, mask, (uint64_t)words,
                     sums, P, cap);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_wheel_offsets(table, 256, stream);  // m[] and a[]
}


hipError_t launch_base_primes_big(uint64_t limit, void* table, uint32_t cap, int num_cus, hipStream_t stream) {
  if (limit <= kBaseLimitMax) return launch_base_primes(limit, table, cap, stream);
  if (limit > kBigBaseLimitMax) return hipErrorInvalidValue;
  // scratch carved from the m[] region: [mask][level-0 table][block sums][count]
  char* mreg = reinterpret_cast<char*>(table) + table_m_offset(cap);
  const uint64_t nb = (limit - 3) / 2 + 1;            // odd values 3..limit
  const uint64_t words = (nb + 63) / 64;
  uint64_t* mask = reinterpret_cast<uint64_t*>(mreg);
  const uint64_t lim0 = [&] {                          // isqrt(limit)
    uint64_t r = (uint64_t)__builtin_sqrt((double)limit);
    while (r * r > limit) --r;
    while ((r + 1) * (r + 1) <= limit) ++r;
    return r;
  }();
  const uint32_t cap0 = (uint32_t)(1.26 * (double)lim0 / __builtin_log((double)(lim0 > 100 ? lim0 : 100))) + 64;
  char* t0 = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(mreg) + words * 8 + 255) & ~(uintptr_t)255);
  const uint64_t t0_bytes = (table_bytes_for_cap(cap0) + 255) & ~255ull;
  const uint32_t nblocks = (uint32_t)((words + kCompactBlockWords - 1) / kCompactBlockWords);
  uint32_t* sums = reinterpret_cast<uint32_t*>(t0 + t0_bytes);
  unsigned long long* cnt = reinterpret_cast<unsigned long long*>(sums + ((nblocks + 63) & ~63u));
  if ((uint64_t)(reinterpret_cast<char*>(cnt + 1) - mreg) > 40ull * cap) return hipErrorInvalidValue;
  hipError_t e = launch_base_primes(lim0, t0, cap0, stream);
  if (e != hipSuccess) return e;
  if ((e = hipMemsetAsync(cnt, 0, sizeof(*cnt), stream)) != hipSuccess) return e;
  if ((e = launch_sieve_range(t0, 0, nb, reinterpret_cast<uint32_t*>(mask), cnt, num_cus, stream)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(compact_count_kernel, dim3(nblocks), dim3(kCompactThreads), 0, stream, mask, words, sums);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, stream, sums, nblocks, table, cap, limit);
  uint32_t* P = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(table) + 16);
  hipLaunchKernelGGL(compact_write_kernel, dim3(nblocks), dim3(kCompactThreads), 0, stream, mask, words, sums, P,
                     cap);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return launch_wheel_offsets(table, num_cus, stream);  // m[] and a[]
}

hipError_t launch_sieve_range_odd(const void* table, uint64_t g_start, uint64_t nbits, uint32_t* out,
                                  unsigned long long* count, int num_cus, hipStream_t stream) {
  if (nbits == 0) return hipSuccess;
  constexpr uint64_t SEG = 1ull << kLogSeg;
  const uint64_t nseg = (nbits + SEG - 1) / SEG;
  const uint64_t grid = nseg < (uint64_t)num_cus ? nseg : (uint64_t)num_cus;
  static const uint32_t phases = [] {
    const char* e = getenv("DSE_PHASES");  // profiling-only ablation knob
    return e ? (uint32_t)strtoul(e, nullptr, 0) : kPhaseAll;
  }();
  static const int cfg = [] {
    const char* e = getenv("DSE_CFG");  // profiling-only: 0 = 2^20 x 1 WG/CU, 1 = 2^19 x 2 WG/CU
    return e ? atoi(e) : 0;
  }();
  if (cfg == 1) {
    constexpr uint64_t SEG1 = 1ull << 19;
    const uint64_t nseg1 = (nbits + SEG1 - 1) / SEG1;
    const uint64_t grid1 = nseg1 < 2ull * num_cus ? nseg1 : 2ull * num_cus;
    hipLaunchKernelGGL((sieve_segments_kernel<19, 512>), dim3((uint32_t)grid1), dim3(512), 0, stream, table,
                       g_start, nbits, out, count, phases);
  } else {
    hipLaunchKernelGGL((sieve_segments_kernel<kLogSeg, kThreads>), dim3((uint32_t)grid), dim3(kThreads), 0,
                       stream, table, g_start, nbits, out, count, phases);
  }
  return hipGetLastError();
}

}  // namespace dse

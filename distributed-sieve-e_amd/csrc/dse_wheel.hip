// dse_wheel.hip -- mod-30 wheel segmented sieve for gfx950 (MI355X).
//
// Bit j of the caller's range stands for the odd value 3+2(g_start+j), the
// reference's element j of its chunk vector (sieve.clj:9-13); a set bit =
// prime. The marking loops replace sieve.clj:36-71's index walk; multiples of
// 3 and 5 are never stored in LDS, so they touch 8/15 of the words an odd-only
// image needs.
//
// Geometry. V0 = v_start - 1 (even); segment s covers the integers
// [Vs, Vs + W), W = 30*KP, Vs = V0 + s*W (KP = 2^17 periods), exactly output
// bits [s*15*KP, (s+1)*15*KP) -- a whole number of words, so no output word is
// shared by two segments. The 8 odd residues rho_0 < ... < rho_7 in [1,29]
// with gcd(V0 + rho, 30) = 1 define the planes: plane i bit k <-> the value
// Vs + rho_i + 30k, i.e. output bit 15k + (rho_i - 1)/2 of the segment.
//
// LDS image (128 KiB), word-interleaved: block R (periods 32R .. 32R+31)
// is 8 consecutive words, one per plane, so the word of (plane i, period k)
// is 8 (k >> 5) + i and its byte address (k & ~31) | 4i -- one v_and_or from
// a period index, and an image of 2^17 periods is 2^17 bytes. The bank of a
// ds_or_b32 (dword address mod 32) is 8 ((k >> 5) mod 4) + i, so a mark
// pattern is conflict-free when the lanes on one plane in a 32-lane group sit
// in distinct blocks mod 4; two lanes per bank cost nothing extra (the
// instruction's transfer takes 2 LDS cycles per group anyway).
//
// One workgroup of 1024 threads per CU, segments blockIdx.x + t*gridDim.x.
// Per segment:
//   1. mark (ds_or_b32), units taken from one LDS counter:
//      A  (79 < p <= TA): one prime per wave; lane (plane i, c = 0..7) takes
//         the hits n of its plane with n mod 256 in [32c, 32c+32), by class
//         n mod 256: a class's hits sit 256p periods apart, same bit, so each
//         further mark is one v_add; the 4 lanes of a plane in a half-wave
//         are 32p periods apart, i.e. in blocks c*p mod 4: distinct banks;
//      B1 (TA < p <= TB1): one prime per half-wave; lane (plane i, j = 0..3)
//         takes the hits n with n mod 128 in [32j, 32j+32), in order (3 VALU
//         per mark), again 32p periods apart: conflict-free;
//      B2 (TB1 < p <= TB): 8 primes x 8 planes per wave, lane (prime, plane)
//         walks its plane's hits in order;
//      L  (p > TB): one prime per lane, its 8 planes in a lane-rotated order,
//         starts from the table's wheel offsets with one reduction;
//   2. expand: lane reads one block (two ds_read_b128), transposes the 8x32
//      bits into 32 period bytes, maps each through a 256-entry LDS table to
//      the 15 odd slots of its period (composite bits in, prime slots out),
//      packs 480 output bits, fixes the small primes 3..79, masks the range
//      end, popcounts, stores; then each wave inits (patterns of 7..61) the
//      blocks it expanded, for the next segment.
// See DESIGN.md section 4 for the rooflines.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <array>
#include <vector>

#include "dse_internal.h"

namespace dse {
namespace {

constexpr uint32_t KP = 1u << kWheelLogKP;  // periods per segment (per plane)
constexpr uint32_t BLOCKS = KP / 32;        // 32-period blocks (8 words each)
constexpr uint32_t IMG_WORDS = 8 * BLOCKS;  // one segment image
constexpr uint32_t IMG_BYTES = 4 * IMG_WORDS;
static_assert(IMG_BYTES == KP, "a period index is its block's byte address");
// The image sits at the top of the workgroup's LDS, bytes [kImgOff, kImgOff +
// IMG_BYTES) (WheelLds): mark addresses are image-relative (a period index |
// its plane's offset) and every ds_or adds kImgOff in its offset field. A
// mark at a period k >= KP (past the segment) thus lands at or beyond the end
// of the allocation, where the LDS drops it (microbench/lds_oor_bench.hip);
// nothing lives above the image. So marks that may fall past the segment's
// end are issued unconditionally, without a compare and exec masking.
#define DSE_IMG_OFF_S "32768"
constexpr uint32_t kImgOff = 32768;
#define DSE_STR2(x) #x
#define DSE_STR(x) DSE_STR2(x)
constexpr uint32_t NT = 1024;
constexpr uint32_t NW = NT / 64;            // waves; every wave marks, expands and inits
static_assert(BLOCKS % (64 * NW) == 0, "expansion blocks");
#ifndef DSE_TA
#define DSE_TA 96
#endif
#ifndef DSE_WHEEL_HALF_TU
#define DSE_WHEEL_HALF_TU 0  // 1: compiled by dse_wheel_half.hip with 2^16 periods per segment
#endif
#ifndef DSE_WHEEL_PLAIN_TU
#define DSE_WHEEL_PLAIN_TU 0  // 1: compiled by dse_wheel_plain.hip: the no-bucket kernel only
#endif
#define DSE_WHEEL_MAIN_TU (!DSE_WHEEL_HALF_TU && !DSE_WHEEL_PLAIN_TU)
#ifndef DSE_HALF_SEG_COST
#define DSE_HALF_SEG_COST 0.68
#endif
#ifndef DSE_LAUNCH_COST
#define DSE_LAUNCH_COST 0.1
#endif
constexpr uint32_t TA = DSE_TA;             // A/B1 threshold
#ifndef DSE_TB1
#define DSE_TB1 640
#endif
constexpr uint32_t TB1 = DSE_TB1;           // B1/B2 threshold
#ifndef DSE_TB
#define DSE_TB 1536
#endif
constexpr uint32_t TB = DSE_TB;             // B2/L threshold
static_assert(TA <= 256 && TA < TB1 && TB1 <= TB && TB <= KP / 8, "unit thresholds");
static_assert(KP / (128 * (TA + 1)) <= 10 && KP / (32 * (TB1 + 1)) <= 10, "class_marks_k covers K <= 10");
constexpr uint32_t kMidCap = TB >= 16384 ? 1920 : TB >= 8192 ? 1040 : TB >= 4096 ? 580 : 320;  // >= odd primes in (61, TB]
constexpr uint32_t kOutWordsPerSeg = (uint32_t)(kWheelOutBits / 32);  // 30720

constexpr uint32_t kQMax = 79;  // the pattern primes are 7..79

constexpr uint32_t inv30_const(uint32_t q) {
  for (uint32_t x = 1; x < q; ++x)
    if ((30 * x) % q == 1) return x;
  return 0;
}
// Init tables: the 15 small primes in 7 groups G with period M_G = prod(G).
// U_G[y] = 1 iff some q in G divides y. Plane i period k holds the value
// Vs + rho_i + 30k, and q | Vs + rho_i + 30k <=> q | k + c_G with
// c_G = (Vs + rho_i) * 30^{-1} mod M_G (gcd(30, M_G) = 1), so every plane
// reads the same bit string at its own offset. A lane inits kInitRun
// consecutive periods of one column: 33 dwords of each string from its bit
// offset o, read as 9 aligned ds_read_b128 from the copy of the string that
// is shifted by (o >> 5) & 3 dwords (4 copies), so every read is aligned
// whatever o is; word r = alignbit(U[d0 + r + 1], U[d0 + r], o & 31).
#ifndef DSE_BK_GRID
#define DSE_BK_GRID 1024  // band-0 fill workgroups (columns)
#endif
#ifndef DSE_BK_UNIT_BATCHES
#define DSE_BK_UNIT_BATCHES 4
#endif
// 7..61 in 7 groups until round 4; 67..79 as two more groups (1e11 -0.3%, 1e12
// -0.7%: the init reads of two more strings cost less than A units for 4 primes)
constexpr int kNG = 9;
constexpr uint32_t kGQ[kNG][3] = {{7, 11, 13}, {17, 19, 1}, {23, 29, 1}, {31, 37, 1}, {41, 43, 1},
                                  {47, 53, 1}, {59, 61, 1}, {67, 71, 1}, {73, 79, 1}};
constexpr uint32_t gmod(int g) { return kGQ[g][0] * kGQ[g][1] * kGQ[g][2]; }
constexpr uint32_t kInitWords = IMG_WORDS / NT;  // words one lane inits per segment (one plane of a block run)
constexpr uint32_t kInitRun = 32 * kInitWords;    // their periods
constexpr uint32_t kExpandBlocks = BLOCKS / NW;   // blocks one wave expands (and inits) per segment
// ds_read_b128 per lane and group (+1: a staggered run's one word more, read as one more pass)
constexpr uint32_t kInitBlocks = kInitRun / 128 + 2;
// dwords per group string and copy: the reads reach dword d0 + 4 kInitBlocks - 1, d0 < M_G/32 + 1
constexpr uint32_t gdw(int g) { return ((gmod(g) + 32 * (4 * kInitBlocks + 1) + 127) / 128) * 4; }
constexpr uint32_t gbase(int g) { return g == 0 ? 0u : gbase(g - 1) + gdw(g - 1); }
constexpr uint32_t kGDW = gbase(kNG);  // dwords per copy (620)
constexpr uint32_t kGInv30[kNG] = {inv30_const(gmod(0)), inv30_const(gmod(1)), inv30_const(gmod(2)),
                                   inv30_const(gmod(3)), inv30_const(gmod(4)), inv30_const(gmod(5)),
                                   inv30_const(gmod(6)), inv30_const(gmod(7)), inv30_const(gmod(8))};

// The init tables, built at compile time (a launch copies them into LDS):
// copy k, group g, dword gbase(g) + j = bits [32 (j + k), 32 (j + k) + 32) of U_g.
struct InitTables {
  uint32_t w[4 * kGDW];
};
constexpr InitTables make_init_tables() {
  InitTables t{};
  for (int g = 0; g < kNG; ++g) {
    for (uint32_t j = 0; j < gdw(g) + 3; ++j) {  // dword j of U_g
      uint32_t v = 0;
      for (uint32_t b = 0; b < 32; ++b) {
        const uint32_t y = 32 * j + b;
        const bool hit = y % kGQ[g][0] == 0 || y % kGQ[g][1] == 0 || (kGQ[g][2] > 1 && y % kGQ[g][2] == 0);
        v |= (uint32_t)hit << b;
      }
      for (uint32_t k = 0; k < 4; ++k)
        if (j >= k && j - k < gdw(g)) t.w[k * kGDW + gbase(g) + (j - k)] = v;
    }
  }
  return t;
}
__device__ const InitTables g_init_tables = make_init_tables();

constexpr uint32_t kLPieces = 16;  // pieces of a range with their own large-prime bound

// One odd-index range of a launch: its segments are [seg0, seg0 + its
// segment count) of the launch's list (WheelArgs::nseg in all).
struct WheelRange {
  uint64_t V0;         // v_start - 1
  uint64_t nbits;      // odd candidates in the range
  uint64_t KB0;        // floor(V0 / 30)
  uint64_t rho_pack;   // rho_i in bits [5i, 5i+5)
  uint32_t* out;       // the range's mask (32-bit words), or null
  unsigned long long* count;  // incremented by the range's prime count (device)
  uint32_t pl_pack;    // plane of absolute residue R30[j] in bits [3j, 3j+3)
  uint32_t e_iota;     // bit j: floor((V0 + rho)/30) = KB0 + 1 for the plane of R30[j]
  uint64_t fix;        // output words 0, 1: bits of the primes 3..kQMax inside the range
  uint32_t seg0;       // first segment of the range in the launch
  uint16_t v0g[kNG];   // V0 mod M_G (init tables)
  // Large units past the live primes of a segment only load operands to skip
  // them: segment s of the range needs table indices below
  // lcap[min(s >> lsh, kLPieces - 1)] (>= the odd primes with p^2 < its end)
  uint32_t lsh;
  uint32_t lcap[kLPieces];
};
// Ranges per launch: several chunks of one device (dse_sieve_all with P >
// devices, and the dropped tail) go to one persistent launch, so no chunk's
// partial last round of segments leaves the CUs idle and no host launch
// latency sits between chunks.
constexpr uint32_t kMaxRanges = 9;

struct WheelArgs {
  WheelRange r[kMaxRanges];
  uint32_t nranges;    // 1..kMaxRanges (1 with bucketed primes)
  uint32_t nseg;       // segments of all ranges
  uint32_t nthr[5];    // odd primes <= kQMax (79), TA, TB1, TB, kWheelMaxPrime (table indices of the unit lists)
  // Bucketed hits of the primes > 2^kBucketLoLog, or the bucket_lo_log2 option (bk_start null: none), as
  // entries (bucket_entry):
  const uint32_t* bk_entries;  // band 1: segment s owns [bk_start[s], bk_start[s+1])
  const uint32_t* bk_start;
  const uint32_t* bk_reg0;     // band 0: segment s, column b: bk_n0[s * kBucketGrid + b] entries
  const uint32_t* bk_n0;       //   from bk_reg0 + (b * nseg + s) * bk_k0
  const unsigned long long* bk_spill;  // band-0 hits past their region: segment << 32 | entry,
  const uint32_t* bk_nspill;           //   *bk_nspill of them (normally none)
  uint64_t bk_spill_cap;               //   (at most this many stored)
  uint32_t bk_k0;              // band-0 region capacity (0: no band 0 in the pass)
};
static_assert(sizeof(WheelArgs) <= 4096, "kernel arguments");
// wheel_segments_kernel(table, wa): wa follows the 8-byte table pointer in the
// kernel-argument segment
constexpr uint32_t kWaOffset = 8;
static_assert(alignof(WheelArgs) <= 8, "kernel argument layout");

// 32-bit LDS byte address of a __shared__ pointer.
__device__ __forceinline__ uint32_t lds_addr(const uint32_t* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)p;
}

// Every mark is issued as asm: the compiler's waitcnt pass does not see it,
// so callers drain lgkmcnt before a barrier (lds_drain); and it does not
// unroll loops around it, so runs are unrolled by hand.
__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Keeps a value opaque to the optimiser (loop strength reduction splits a
// marking offset into several induction variables; lane-derived constants get
// hoisted out of the segment loop and spilled).
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}

constexpr uint32_t kBlockMask = ~31u;  // period index -> its block's byte address
#ifndef DSE_FAKE_CF_L
#define DSE_FAKE_CF_L 0
#endif
// profiling knockout (DSE_FAKE_CF_L): the L marks' blocks forced to lane-distinct banks (wrong marks)
constexpr uint32_t kBlockMaskL = DSE_FAKE_CF_L ? ~127u : kBlockMask;
#ifndef DSE_FAKE_CF_INIT
#define DSE_FAKE_CF_INIT 0
#endif
#ifndef DSE_SHORT_TAIL
#define DSE_SHORT_TAIL 16
#endif
// MODE-0 L sets whose tail after the n_min run is at most this many steps mark
// it unconditionally (past the segment: dropped) instead of in mark_tail's loop
constexpr uint32_t kShortTail = DSE_SHORT_TAIL;
// Odd primes <= TB: the table index where the L list (and its sets of 64
// primes) starts whenever the table reaches past TB.
constexpr uint32_t odd_primes_upto(uint32_t x) {
  uint32_t c = 0;
  for (uint32_t v = 3; v <= x; v += 2) {
    bool pr = true;
    for (uint32_t d = 3; d * d <= v; d += 2)
      if (v % d == 0) { pr = false; break; }
    c += pr;
  }
  return c;
}
constexpr uint32_t kL0 = odd_primes_upto(TB);
// The marking plan of a set of 64 large primes pmin..pmax (unit_L), fixed by
// the primes and the segment geometry, so the table carries it (pl[] words
// p | plan << 20, wheel_offsets_kernel) instead of each set deriving it per
// segment with two divisions (~40 instructions): bits 0-1 MODE (2: pmin > KP,
// one mark per plane; 1: pmin > KP/2, two; 0: runs), bit 2 a tail loop
// follows the run, bits 3.. the run length: ceil(KP / pmin) (every lane's hit
// count is at most that; the marks past the segment are dropped), or
// floor(KP / pmax) (every lane's minimum) when the two differ by more than
// kShortTail.
constexpr uint32_t kLPrimeMask = 0x800FFFFFu;  // pl[] word -> p (bit 31: lane past the table end)
static_assert(kWheelMaxPrime <= (1u << 20), "pl[] words: the L primes (odd, <= kWheelMaxPrime) are below 2^20");
__host__ __device__ constexpr uint32_t l_plan(uint32_t pmin, uint32_t pmax, uint32_t kp) {
  if (pmin > kp) return 2;
  if (pmin > kp / 2) return 1;
  const uint32_t n_min = pmax >= kp ? 0u : kp / pmax;
  const uint32_t n_all = (kp + pmin - 1) / pmin;
  return n_all - n_min <= kShortTail ? n_all << 3 : 4u | n_min << 3;
}
static_assert(l_plan(TB + 2, TB + 2, 1u << 17) < (1u << 12), "the plan fits 12 bits");
static_assert(odd_primes_upto(kQMax) + kMidCap >= kL0, "the L list starts at kL0 whenever it exists");

// Mark period k (< KP) of the plane whose byte base is pb4 (image + 4 plane):
// address (k & ~31) | pb4 in one v_and_or, bit 1 << (k & 31) (the shift reads
// the low 5 bits itself). 2 VALU.
__device__ __forceinline__ void mark_k(uint32_t pb4, uint32_t k, uint32_t one) {
  uint32_t a, b;
  asm volatile(
      "v_and_or_b32 %0, %2, %3, %4\n\t"
      "v_lshlrev_b32 %1, %2, %5\n\t"
      "ds_or_b32 %0, %1 offset:" DSE_IMG_OFF_S
      : "=&v"(a), "=&v"(b)
      : "v"(k), "s"(kBlockMask), "v"(pb4), "v"(one)
      : "memory");
}

// mark_k and advance k by p, in one asm block (written as mark_k + an add,
// the loop-carried index costs a v_mov per mark). 3 VALU.
__device__ __forceinline__ void mark_k_step(uint32_t pb4, uint32_t& k, uint32_t p, uint32_t one) {
  uint32_t a, b;
  asm volatile(
      "v_and_or_b32 %0, %2, %3, %4\n\t"
      "v_lshlrev_b32 %1, %2, %6\n\t"
      "ds_or_b32 %0, %1 offset:" DSE_IMG_OFF_S "\n\t"
      "v_add_u32 %2, %2, %5"
      : "=&v"(a), "=&v"(b), "+v"(k)
      : "s"(kBlockMask), "v"(pb4), "v"(p), "v"(one)
      : "memory");
}

// Four mark_k_steps in one asm block. Between two asm blocks the compiler
// puts a wait state (s_nop 0, or a filler) whenever the second reads a VGPR
// the first wrote -- it cannot see that no instruction in them needs one --
// so back-to-back mark_k_steps cost an s_nop per mark.
__device__ __forceinline__ void mark_k_step4(uint32_t pb4, uint32_t& k, uint32_t p, uint32_t one) {
  uint32_t a0, b0, a1, b1;
  asm volatile(
      "v_and_or_b32 %0, %4, %5, %6\n\t"
      "v_lshlrev_b32 %1, %4, %8\n\t"
      "v_add_u32 %4, %4, %7\n\t"
      "ds_or_b32 %0, %1 offset:" DSE_IMG_OFF_S "\n\t"
      "v_and_or_b32 %2, %4, %5, %6\n\t"
      "v_lshlrev_b32 %3, %4, %8\n\t"
      "v_add_u32 %4, %4, %7\n\t"
      "ds_or_b32 %2, %3 offset:" DSE_IMG_OFF_S "\n\t"
      "v_and_or_b32 %0, %4, %5, %6\n\t"
      "v_lshlrev_b32 %1, %4, %8\n\t"
      "v_add_u32 %4, %4, %7\n\t"
      "ds_or_b32 %0, %1 offset:" DSE_IMG_OFF_S "\n\t"
      "v_and_or_b32 %2, %4, %5, %6\n\t"
      "v_lshlrev_b32 %3, %4, %8\n\t"
      "v_add_u32 %4, %4, %7\n\t"
      "ds_or_b32 %2, %3 offset:" DSE_IMG_OFF_S
      : "=&v"(a0), "=&v"(b0), "=&v"(a1), "=&v"(b1), "+v"(k)
      : "s"(kBlockMask), "v"(pb4), "v"(p), "v"(one)
      : "memory");
}


// n unconditional marks k, k + p, ... (by 4: three SALU of loop control per
// mark otherwise); returns the index after the run.
__device__ __forceinline__ uint32_t mark_run(uint32_t pb4, uint32_t k, uint32_t p, uint32_t n, uint32_t one) {
  uint32_t h = 0;
  for (; h + 4 <= n; h += 4) mark_k_step4(pb4, k, p, one);
  for (; h < n; ++h) mark_k_step(pb4, k, p, one);
  return k;
}

// The rest of a lane's walk: k, k + p, ... while k < KP, as one asm loop
// that narrows exec as lanes finish (v_cmpx) and restores it once: 4 VALU
// and one branch per step (the compiler's loop keeps a mask of finished
// lanes: 2 more SALU per step; 1e11 -0.3%). All exec writes are inside the
// block. The branches only decide whether to run another step: exec only
// narrows, every mark is predicated by the exec the v_cmpx left, and a step
// run with an empty exec changes nothing, so even a branch that read exec
// from before the v_cmpx could not mark anything wrong, only run one empty
// step (and k grows by p every step, so the loop ends).
__device__ __forceinline__ void mark_tail(uint32_t pb4, uint32_t k, uint32_t p, uint32_t one) {
  uint64_t sv;
  uint32_t a, b;
  asm volatile(
      "s_mov_b64 %3, exec\n\t"
      "v_cmpx_gt_u32_e32 vcc, %5, %2\n\t"
      "s_cbranch_execz 2f\n"
      "1:\n\t"
      "v_and_or_b32 %0, %2, %6, %7\n\t"
      "v_lshlrev_b32 %1, %2, %8\n\t"
      "v_add_u32 %2, %2, %4\n\t"
      "ds_or_b32 %0, %1 offset:" DSE_IMG_OFF_S "\n\t"
      "v_cmpx_gt_u32_e32 vcc, %5, %2\n\t"
      "s_cbranch_execnz 1b\n"
      "2:\n\t"
      "s_mov_b64 exec, %3"
      : "=&v"(a), "=&v"(b), "+v"(k), "=&s"(sv)
      : "v"(p), "s"(KP), "s"(kBlockMask), "v"(pb4), "v"(one)
      : "memory", "vcc");
}

// ds_or_b32 at a precomputed LDS byte address.
__device__ __forceinline__ void mark_at(uint32_t a, uint32_t bit) {
  asm volatile("ds_or_b32 %0, %1 offset:" DSE_IMG_OFF_S : : "v"(a), "v"(bit) : "memory");
}

// The hits k + (r + 32 t) p, r = 0..31, t < K, of a lane that walks one
// plane from k with step p: class r's hits sit D = 32 S p periods apart (S =
// 1 for a lane that takes consecutive hits, 4 for B1's lanes, which take 32
// of every 128), so they share their bit and their byte addresses step by D
// (a period index is its block's byte address): 3 VALU of setup per class,
// then one v_add per mark (mark_k_step: 3 VALU per mark).
template <int K>
__device__ __forceinline__ void class_marks(uint32_t pb4, uint32_t k, uint32_t p, uint32_t D, uint32_t one) {
#pragma unroll 1
  for (uint32_t r = 0; r < 32; ++r) {
    uint32_t a, b;
    asm volatile(
        "v_and_or_b32 %0, %2, %3, %4\n\t"
        "v_lshlrev_b32 %1, %2, %5\n\t"
        "ds_or_b32 %0, %1 offset:" DSE_IMG_OFF_S
        : "=&v"(a), "=&v"(b)
        : "v"(k), "s"(kBlockMask), "v"(pb4), "v"(one)
        : "memory");
#pragma unroll
    for (int t = 1; t < K; ++t) {
      a += D;
      mark_at(a, b);
    }
    k = opaque(k + p);
  }
}
// K wave-uniform in 1..10 (B1: floor(KP / 128 pmax), B2: floor(KP / 32
// pmax); 0: nothing)
__device__ __forceinline__ void class_marks_k(uint32_t K, uint32_t pb4, uint32_t k, uint32_t p, uint32_t D,
                                              uint32_t one) {
  switch (K) {
    case 0: return;
    case 1: class_marks<1>(pb4, k, p, D, one); return;
    case 2: class_marks<2>(pb4, k, p, D, one); return;
    case 3: class_marks<3>(pb4, k, p, D, one); return;
    case 4: class_marks<4>(pb4, k, p, D, one); return;
    case 5: class_marks<5>(pb4, k, p, D, one); return;
    case 6: class_marks<6>(pb4, k, p, D, one); return;
    case 7: class_marks<7>(pb4, k, p, D, one); return;
    case 8: class_marks<8>(pb4, k, p, D, one); return;
    case 9: class_marks<9>(pb4, k, p, D, one); return;
    case 10: class_marks<10>(pb4, k, p, D, one); return;
    default: __builtin_unreachable();
  }
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

// (x & m) | (y & ~m): v_bfi_b32
// (the compiler rewrites the C form into v_and + v_bitop3 pairs)
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(x), "v"(y));
  return r;
}

// Transpose the 8 x 8 bit matrix in each byte column q of W[0..7] (row i =
// W[i] byte q): afterwards W[j] byte q bit i = old W[i] byte q bit j. Three
// rounds of block swaps between rows i and i + s (blocks of s bits), 4 VALU
// per swap: the upper s bits of row i's blocks trade places with the lower s
// bits of row i + s's.
template <int S>
__device__ __forceinline__ void bit_block_swap(uint32_t& a, uint32_t& b) {
  constexpr uint32_t m = S == 4 ? 0x0F0F0F0Fu : S == 2 ? 0x33333333u : 0x55555555u;
  const uint32_t x = a, y = b;
  b = bfi(m, x >> S, y);
  a = bfi(~m, y << S, x);
}
__device__ __forceinline__ void bit_block_swaps(uint32_t (&W)[8]) {
  bit_block_swap<4>(W[0], W[4]); bit_block_swap<4>(W[1], W[5]);
  bit_block_swap<4>(W[2], W[6]); bit_block_swap<4>(W[3], W[7]);
  bit_block_swap<2>(W[0], W[2]); bit_block_swap<2>(W[1], W[3]);
  bit_block_swap<2>(W[4], W[6]); bit_block_swap<2>(W[5], W[7]);
  bit_block_swap<1>(W[0], W[1]); bit_block_swap<1>(W[2], W[3]);
  bit_block_swap<1>(W[4], W[5]); bit_block_swap<1>(W[6], W[7]);
}

// ---- work units of the mark phase ----------------------------------------

// A, by hit class: lane (plane, c) owns the hits n of its plane with n mod
// 256 = 32c + r, r = 0..31; class r's hits k0 + 256p t share their bit and
// their byte addresses step by the wave-uniform 256p, so after 3 VALU of class
// setup each further mark is one v_add. k0 = kp + (32c + r) p < 256p, so
// every class has K = floor(KP / 256p) or K + 1 hits: K + 1 marks, the last
// dropped past the image (address >= IMG_BYTES, see kImgOff). k = the class-0
// hit of the lane.
template <int K>
__device__ __forceinline__ void a_classes(uint32_t pb4, uint32_t k, uint32_t p, uint32_t one) {
  const uint32_t D = p << 8;  // 256 p periods = bytes
#pragma unroll 1
  for (uint32_t r = 0; r < 32; ++r) {
    uint32_t a, bit;
    asm volatile(
        "v_and_or_b32 %0, %2, %3, %4\n\t"
        "v_lshlrev_b32 %1, %2, %5"
        : "=&v"(a), "=&v"(bit)
        : "v"(k), "s"(kBlockMask), "v"(pb4), "v"(one));
#pragma unroll
    for (int t = 0; t < K; ++t) {
      mark_at(a, bit);
      a += D;
    }
    mark_at(a, bit);  // past the image (a >= IMG_BYTES): dropped
    k = opaque(k + p);
  }
}

// Vs mod p of the staged mid primes, carried from segment to segment: a
// workgroup's next segment starts G W integers later (G workgroups), so the
// unit that uses x[i] for this segment leaves (x[i] + inc[i]) mod p there,
// inc[i] = G W mod p. `have`: x holds this segment's residues (the
// workgroup's previous segment was of the same range and every mid unit ran
// in it); otherwise a 64-bit Barrett reduction (the workgroup's first
// segment, a range change, segments below TB^2).
struct MidRes {
  uint32_t* x;
  const uint32_t* inc;
  bool have;
};
__device__ __forceinline__ uint32_t mid_residue(const MidRes& mr, uint32_t i, uint32_t p, uint64_t m, uint64_t Vs,
                                                bool writer) {
  const uint32_t xs = mr.have ? mr.x[i] : mod_barrett(Vs, p, m);
  if (writer) {
    const uint32_t t = xs + mr.inc[i];
    mr.x[i] = min(t, t - p);
  }
  return xs;
}

// A: one mid prime (kQMax < p <= TA) per wave; lane (plane L & 7, c = L >> 3).
// Lanes 0-31 have c = 0..3: a plane's four lanes mark 32p periods apart at
// every step (same class r, same t), i.e. in blocks c p (mod 4) apart -- four
// distinct banks for odd p.
__device__ __forceinline__ void unit_A(uint32_t img0, uint32_t pi, uint64_t m, const MidRes& mr, uint32_t idx,
                                       uint64_t Vs, uint64_t rho_pack, uint32_t lane, uint32_t one) {
  const uint32_t p = pi & 0xFFFFu, inv30 = pi >> 16;  // wave-uniform
  const uint64_t p2 = (uint64_t)p * p;
  const uint32_t Xs = __builtin_amdgcn_readfirstlane(mid_residue(mr, idx, p, m, Vs, lane == 0));
  const float invp = fast_rcp((float)p);
  const uint32_t pl = lane & 7, c = lane >> 3;
  const uint32_t rho = (uint32_t)(rho_pack >> (5 * pl)) & 31u;
  const uint32_t kp = plane_first(Xs, rho, p, inv30, invp);
  const uint32_t pb4 = img0 + 4 * pl;
  const uint32_t k = kp + 32 * c * p;                   // class 0 of the lane: hit n = 32c
  if (p2 <= Vs) {
    switch (KP / (256 * p)) {  // K (wave-uniform): 2..6 for kQMax < p <= TA (1..3 for the half geometry)
      case 1: a_classes<1>(pb4, k, p, one); return;
      case 2: a_classes<2>(pb4, k, p, one); return;
      case 3: a_classes<3>(pb4, k, p, one); return;
      case 4: a_classes<4>(pb4, k, p, one); return;
      case 5: a_classes<5>(pb4, k, p, one); return;
      case 6: a_classes<6>(pb4, k, p, one); return;
      case 7: a_classes<7>(pb4, k, p, one); return;
      default: __builtin_unreachable();
    }
  }
  // p^2 inside the segment (its first segments only): the lane's hits with
  // k >= kmin, one at a time
  const uint32_t kmin = kmin_for((uint32_t)(p2 - Vs), rho);
  for (uint32_t r = 0; r < 32; ++r)
    for (uint32_t kk = k + r * p; kk < KP; kk += 256 * p)
      if (kk >= kmin) mark_k(pb4, kk, one);
}

// B1: two mid primes (TA < p <= TB1), one per half-wave; lane (plane L & 7,
// j = (L >> 3) & 3) owns the hits n with n mod 128 in [32j, 32j + 32), in
// order: 32 marks k, k + p, ... then a jump of 96p. The four lanes of a plane
// are 32p periods apart: distinct banks, as in A. The blocks of 128 hits
// every lane fills are marked class by class (class_marks); the rest in
// order with wave-uniform counts, the marks past the segment dropped.
__device__ __forceinline__ void unit_B1(uint32_t img0, const uint32_t* __restrict__ s_mid_p,
                                        const uint64_t* __restrict__ s_mid_m, const MidRes& mr, uint32_t j0,
                                        uint32_t nj, uint64_t Vs, uint64_t rho_pack, uint32_t lane, uint32_t one) {
  const uint32_t h = lane >> 5, pl = lane & 7, j = (lane >> 3) & 3;
  if (h >= nj) return;  // the unit's second half-wave when the list ends
  const uint32_t pi = s_mid_p[j0 + h];
  const uint32_t p = pi & 0xFFFFu, inv30 = pi >> 16;
  const uint64_t m = s_mid_m[j0 + h];
  const float invp = fast_rcp((float)p);
  const uint32_t rho = (uint32_t)(rho_pack >> (5 * pl)) & 31u;
  const uint32_t kp = plane_first(mid_residue(mr, j0 + h, p, m, Vs, (lane & 31) == 0), rho, p, inv30, invp);
  const uint32_t pb4 = img0 + 4 * pl;
  uint32_t k = kp + 32 * j * p;                          // hit n = 32j
  const uint64_t p2 = (uint64_t)p * p;
  if (p2 > Vs) {  // p^2 inside the segment: one at a time from kmin
    const uint32_t kmin = kmin_for((uint32_t)min(p2 - Vs, (uint64_t)0xFFFFFFFFu), rho);
    for (; k < KP; k += 96 * p)
      for (uint32_t r = 0; r < 32 && k < KP; ++r, k += p)
        if (k >= kmin) mark_k(pb4, k, one);
    return;
  }
  // blocks every lane of the wave fills: n < 128 (t + 1) <= floor(KP / pmax)
  const uint32_t pmax = __builtin_amdgcn_readlane(p, nj == 2 ? 32 : 0);  // the list ascends
  // class by class (hits 32j + r + 128t, t < tf: 128p periods apart, one
  // bit): 1 VALU per mark where walking them takes 3 (1e11: -0.9%)
  const uint32_t tf = (KP / pmax) / 128;  // wave-uniform (a scalar division)
  class_marks_k(tf, pb4, k, p, 128 * p, one);
  k += tf * (128 * p);
  // the rest: every hit index n of either prime is below n_all = ceil(KP /
  // pmin) (kp < p), so in each further block of 128 hits lane j marks hits
  // base + 32j + r, r < min(32, n_all - base), in order; the ones past the
  // segment are dropped (kImgOff). Wave-uniform counts, no per-lane loop.
  const uint32_t pmin = __builtin_amdgcn_readfirstlane(p);
  const uint32_t n_all = __builtin_amdgcn_readfirstlane(div_ceil_small(KP, pmin, fast_rcp((float)pmin)));
  for (uint32_t base = 128 * tf; base < n_all; base += 128) {
    mark_run(pb4, k, p, min(32u, n_all - base), one);
    k += 128 * p;
  }
}

// B2: 8 mid primes (TB1 < p <= TB) x 8 planes; lane (prime L >> 3, plane
// L & 7) marks its plane's hits: n_u unconditional marks for every lane (the
// first 32 floor(n_u / 32) class by class), then the rest and the tail up to
// ceil(KP / pmin) hits as one run (the marks past the segment dropped). A
// plane's lanes hold different primes, so their banks collide at random (the
// L pattern).
__device__ __forceinline__ void unit_B2(uint32_t img0, const uint32_t* __restrict__ s_mid_p,
                                        const uint64_t* __restrict__ s_mid_m, const MidRes& mr, uint32_t j0,
                                        uint32_t nj, uint64_t Vs, uint64_t Vend, uint64_t rho_pack, uint32_t lane,
                                        uint32_t one) {
  const uint32_t pl = lane & 7, jp = lane >> 3;
  const bool valid = jp < nj;
  const uint32_t pi = s_mid_p[valid ? j0 + jp : j0];
  const uint32_t p = pi & 0xFFFFu, inv30 = pi >> 16;
  const uint64_t m = s_mid_m[valid ? j0 + jp : j0];
  const float invp = fast_rcp((float)p);
  const uint32_t rho = (uint32_t)(rho_pack >> (5 * pl)) & 31u;
  uint32_t k = plane_first(mid_residue(mr, valid ? j0 + jp : j0, p, m, Vs, valid && pl == 0), rho, p, inv30, invp);
  const uint64_t p2 = (uint64_t)p * p;
  const bool slow = p2 > Vs;
  if (slow) k = p2 >= Vend ? KP : first_at_or_after(k, kmin_for((uint32_t)(p2 - Vs), rho), p, invp);
  const uint32_t pmax = __builtin_amdgcn_readfirstlane(s_mid_p[j0 + nj - 1]) & 0xFFFFu;
  const bool any_slow = __builtin_amdgcn_ballot_w64(slow) != 0;
  const uint32_t n_u = any_slow ? 0u : KP / pmax;  // every lane has >= floor(KP / p) of them (k < p)
  const uint32_t pb4 = img0 + 4 * pl;
  // lanes past the batch end mark nothing (their unconditional marks would
  // land in another prime's plane)
  if (!valid) return;
  // the first 32 K of the n_u unconditional hits class by class (hits r +
  // 32t, t < K: 32p periods apart, one bit), the rest in order
  const uint32_t K = n_u / 32;
  class_marks_k(K, pb4, k, p, 32 * p, one);
  k += K * (32 * p);
  if (any_slow) {
    mark_tail(pb4, mark_run(pb4, k, p, n_u - 32 * K, one), p, one);
    return;
  }
  // every lane has fewer than n_all = ceil(KP / pmin) hits (k < p): the rest
  // as one run, the marks past the segment dropped (kImgOff)
  const uint32_t pmin = __builtin_amdgcn_readfirstlane(s_mid_p[j0]) & 0xFFFFu;
  const uint32_t n_all = __builtin_amdgcn_readfirstlane(div_ceil_small(KP, pmin, fast_rcp((float)pmin)));
  mark_run(pb4, k, p, n_all - 32 * K, one);
}

// Operands of one large unit, loaded ahead of use. The table row of prime i
// holds its 8 wheel offsets rotated by i mod 8, so lane L (i = 64u + L) reads
// a[(q + L) & 7] at position q with two aligned 16-byte loads.
struct LargeOps {
  uint32_t p;
  uint64_t m;
  uint32_t a[8];
};

__device__ __forceinline__ void load_L(LargeOps& o, const uint32_t* __restrict__ P, const uint64_t* __restrict__ M,
                                       const uint32_t* __restrict__ A, uint32_t il, uint32_t np, bool need_m) {
  const uint32_t ic = min(il, np - 1);  // past the table end: load the last row, mark nothing
  // p | plan << 20 (table pl[]); past the table end bit 31 marks the lane dead
  // (a load under exec into the preset register: a select after an
  // unconditional load would wait for the load right here)
  o.p = il < np ? *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(P) + (ic << 2)) : 0xFFFFFFFFu;
  o.m = need_m ? M[ic] : 0ull;  // the Barrett factor: only for Kb >= 2^38 (unit_L); 1e12: -1.9%
  // 32-bit byte offset from the table's base (one VALU, no 64-bit address math)
  const uint4* row = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(A) + (ic << 5));
  const uint4 lo = row[0], hi = row[1];
  o.a[0] = lo.x; o.a[1] = lo.y; o.a[2] = lo.z; o.a[3] = lo.w;
  o.a[4] = hi.x; o.a[5] = hi.y; o.a[6] = hi.z; o.a[7] = hi.w;
}

// Operand registers whose contents are dead: left undefined (an empty asm
// that "writes" them), so the compiler keeps no copy of what they held.
__device__ __forceinline__ void undef_ops(LargeOps& o) {
  asm volatile("" : "=v"(o.p), "=v"(o.m), "=v"(o.a[0]), "=v"(o.a[1]), "=v"(o.a[2]), "=v"(o.a[3]), "=v"(o.a[4]),
               "=v"(o.a[5]), "=v"(o.a[6]), "=v"(o.a[7]));
}

// Mark a bucketed hit: entry = LDS word index << 5 | bit (bucket_entry), so
// the address is img0 + (e >> 5) * 4 and the bit 1 << (e & 31) (the shift
// reads the low 5 bits itself): 3 VALU.
__device__ __forceinline__ void mark_entry(uint32_t img0, uint32_t e, uint32_t one) {
  uint32_t a, b;
  asm volatile(
      "v_lshrrev_b32 %0, 3, %2\n\t"
      "v_and_or_b32 %0, %0, -4, %4\n\t"
      "v_lshlrev_b32 %1, %2, %3\n\t"
      "ds_or_b32 %0, %1 offset:" DSE_IMG_OFF_S
      : "=&v"(a), "=&v"(b)
      : "v"(e), "v"(one), "v"(img0)
      : "memory");
}

// Kb mod p by float quotients (unit_L): p > TB bounds the quotients.
constexpr uint64_t kQuotBits = 22;                                 // Kb < 2^32: q < 2^32 / (TB + 1) < 2^22
constexpr uint64_t kQuotErr38 = (1ull << (38 - 22)) / (TB + 1) + 1;  // Kb < 2^38: |q error| < 2^16 / (TB + 1) + 1
static_assert((1ull << 32) / (TB + 1) < (1ull << kQuotBits), "Kb < 2^32: float quotient within 1 (and < 2^24 for __umul24)");
static_assert((kQuotErr38 + 2) * kWheelMaxPrime < (1ull << 31), "Kb < 2^38: the rest Kb - q p must be exact in int32");
static_assert(kWheelMaxPrime < (1ull << 23), "__mul24 / __umul24 operands and float-exact p");
static_assert((uint64_t)(kWheelMaxPrime + 1) * (kWheelMaxPrime + 1) / 30 < (1ull << 38),
              "ranges without bucketed primes never need the Barrett path (unit_L<false>)");

// L: 64 large primes (p > TB), one per lane; at step q lane L handles the
// absolute residue (q + L) & 7 (a half-wave spreads over all 8 planes). The
// per-plane hit count is at most ceil(KP / pmin): units whose primes all
// exceed KP (resp. KP/2) take one (two) predicated marks per plane, no loop.
// Per-segment, per-lane constants of the L units: at step q the lane handles
// absolute residue (q + i) & 7, whose plane byte base (pb) and -e (ne) are
// the same for every unit of the segment.
struct PlaneSteps {
  uint32_t pb[8];
  uint32_t ne[8];
  uint32_t one;  // 1 in a VGPR (shl1)
};

// Plane start (a - Kb - e) mod p = min(t, t + p), t = a + (-Kb mod p) + (-e)
// as one v_add3 (left to itself the compiler forms a - (kbm + e): 4 VALU).
__device__ __forceinline__ uint32_t plane_start(uint32_t a, uint32_t nKbm, uint32_t ne, uint32_t p) {
  uint32_t t, u;
  asm("v_add3_u32 %0, %2, %3, %4\n\t"
      "v_add_u32 %1, %0, %5\n\t"
      "v_min_u32 %0, %0, %1"
      : "=&v"(t), "=&v"(u)
      : "v"(a), "v"(nKbm), "v"(ne), "v"(p));
  return t;
}

// Branch-free body of an L unit whose 64 primes are all live and past p^2
// (the common case): the mark count per plane is decided once per unit.
// MODE 2: pmin > KP, one mark per plane; MODE 1: pmin > KP/2, two; MODE 0:
// n_min unconditional marks per plane and a short loop for the rest. Marks
// past the segment's end are dropped by the LDS (kImgOff), so MODE 1/2 and
// short MODE-0 tails need no compare and no exec masking.
// MODE 1/2: four planes per asm block, each a plane start (a - Kb - e) mod p
// and its NM = 1 or 2 marks kk, kk + p: 5 VALU + one ds_or per mark (round
// 5 predicated each mark with v_cmpx and restored exec after each plane: 2
// instructions more per plane and one per block). One block of four planes,
// not one per plane: between two asm blocks the compiler places an s_nop when
// the second reads a VGPR the first wrote.
#define DSE_PLANE_START(A, NE)                                       \
  "v_add3_u32 %0, " A ", %15, " NE "\n\t" /* t = a - Kb mod p - e */ \
  "v_add_u32 %1, %0, %16\n\t"                                        \
  "v_min_u32 %0, %0, %1\n\t" /* kk = (a - Kb - e) mod p */
#define DSE_PLANE_MARK(PB)               \
  "v_and_or_b32 %1, %0, %17, " PB "\n\t" \
  "v_lshlrev_b32 %2, %0, %18\n\t"        \
  "ds_or_b32 %1, %2 offset:" DSE_IMG_OFF_S "\n\t"
#define DSE_PLANE_NEXT "v_add_u32 %0, %0, %16\n\t"
template <int NM>
__device__ __forceinline__ void start_marks4(const uint32_t* a, const uint32_t* ne, const uint32_t* pb, uint32_t nKbm,
                                             uint32_t p, uint32_t one) {
  uint32_t t, u, b;
  if (NM == 1)
    asm volatile(
        DSE_PLANE_START("%3", "%7") DSE_PLANE_MARK("%11")
        DSE_PLANE_START("%4", "%8") DSE_PLANE_MARK("%12")
        DSE_PLANE_START("%5", "%9") DSE_PLANE_MARK("%13")
        DSE_PLANE_START("%6", "%10") DSE_PLANE_MARK("%14")
        : "=&v"(t), "=&v"(u), "=&v"(b)
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(ne[0]), "v"(ne[1]), "v"(ne[2]), "v"(ne[3]), "v"(pb[0]),
          "v"(pb[1]), "v"(pb[2]), "v"(pb[3]), "v"(nKbm), "v"(p), "s"(kBlockMaskL), "v"(one)
        : "memory");
  else
    asm volatile(
        DSE_PLANE_START("%3", "%7") DSE_PLANE_MARK("%11") DSE_PLANE_NEXT DSE_PLANE_MARK("%11")
        DSE_PLANE_START("%4", "%8") DSE_PLANE_MARK("%12") DSE_PLANE_NEXT DSE_PLANE_MARK("%12")
        DSE_PLANE_START("%5", "%9") DSE_PLANE_MARK("%13") DSE_PLANE_NEXT DSE_PLANE_MARK("%13")
        DSE_PLANE_START("%6", "%10") DSE_PLANE_MARK("%14") DSE_PLANE_NEXT DSE_PLANE_MARK("%14")
        : "=&v"(t), "=&v"(u), "=&v"(b)
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(ne[0]), "v"(ne[1]), "v"(ne[2]), "v"(ne[3]), "v"(pb[0]),
          "v"(pb[1]), "v"(pb[2]), "v"(pb[3]), "v"(nKbm), "v"(p), "s"(kBlockMaskL), "v"(one)
        : "memory");
}

#ifndef DSE_LOCKSTEP
#define DSE_LOCKSTEP 1
#endif
// One mark in each of the 8 planes, k[q] += p: 32 instructions in one block
// (two scratch pairs alternate, as in mark_k_step4, so a ds_or's operands are
// not rewritten by the next instruction).
#define DSE_MARK8_ONE(A, B, K, PB)                   \
  "v_and_or_b32 " A ", " K ", %21, " PB "\n\t"     \
  "v_lshlrev_b32 " B ", " K ", %22\n\t"             \
  "v_add_u32 " K ", " K ", %20\n\t"                 \
  "ds_or_b32 " A ", " B " offset:" DSE_IMG_OFF_S "\n\t"
__device__ __forceinline__ void mark8(uint32_t (&k)[8], const uint32_t* pb, uint32_t p, uint32_t one) {
  uint32_t a0, b0, a1, b1;
  asm volatile(DSE_MARK8_ONE("%0", "%1", "%4", "%12") DSE_MARK8_ONE("%2", "%3", "%5", "%13")
                   DSE_MARK8_ONE("%0", "%1", "%6", "%14") DSE_MARK8_ONE("%2", "%3", "%7", "%15")
                       DSE_MARK8_ONE("%0", "%1", "%8", "%16") DSE_MARK8_ONE("%2", "%3", "%9", "%17")
                           DSE_MARK8_ONE("%0", "%1", "%10", "%18") DSE_MARK8_ONE("%2", "%3", "%11", "%19")
               : "=&v"(a0), "=&v"(b0), "=&v"(a1), "=&v"(b1), "+v"(k[0]), "+v"(k[1]), "+v"(k[2]), "+v"(k[3]),
                 "+v"(k[4]), "+v"(k[5]), "+v"(k[6]), "+v"(k[7])
               : "v"(pb[0]), "v"(pb[1]), "v"(pb[2]), "v"(pb[3]), "v"(pb[4]), "v"(pb[5]), "v"(pb[6]), "v"(pb[7]),
                 "v"(p), "s"(kBlockMaskL), "v"(one)
               : "memory");
}

// MODE 0: n_run marks per plane (TAIL false: n_min + the tail, the ones past
// the segment dropped), or n_run = n_min marks and a loop for the rest (TAIL
// true: sets whose primes spread over a wide range of hit counts).
template <int MODE, bool TAIL = false>
__device__ __forceinline__ void unit_L_fast(const LargeOps& o, uint32_t p, uint32_t nKbm, const PlaneSteps& ps,
                                            uint32_t n_run) {
  if (MODE != 0) {
    constexpr int NM = MODE == 2 ? 1 : 2;  // marks per plane
    start_marks4<NM>(o.a, ps.ne, ps.pb, nKbm, p, ps.one);
    start_marks4<NM>(o.a + 4, ps.ne + 4, ps.pb + 4, nKbm, p, ps.one);
    return;
  }
#if DSE_LOCKSTEP
  if (!TAIL) {
    // all 8 planes in lockstep: one asm block marks hit h of every plane, so
    // the loop control is paid once per 8 marks (the plane starts take the
    // operand row's registers)
    uint32_t kk[8];
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) kk[q] = plane_start(o.a[q], nKbm, ps.ne[q], p);
#pragma unroll 1
    for (uint32_t h = 0; h < n_run; ++h) mark8(kk, ps.pb, p, ps.one);
    return;
  }
#endif
#pragma unroll
  for (uint32_t q = 0; q < 8; ++q) {
    const uint32_t kk = plane_start(o.a[q], nKbm, ps.ne[q], p);
    const uint32_t pb4 = ps.pb[q];
    const uint32_t k = mark_run(pb4, kk, p, n_run, ps.one);
    if (TAIL) mark_tail(pb4, k, p, ps.one);
  }
}

// BARRETT: the launch may hold Kb >= 2^38 (values above 8.2e12, only with
// bucketed primes: the ranges without them end below (2^20 + 1)^2 < 2^40, so
// Kb < 2^36 there and the instantiation keeps no Barrett factors in its
// operand registers)
template <bool BARRETT>
__device__ __forceinline__ void unit_L(const LargeOps& o, uint64_t Vs, uint64_t Vend, uint64_t Kb,
                                       const PlaneSteps& ps, uint32_t pl_rot, const uint64_t* rho_pack_p,
                                       uint32_t sqrt_vs) {
  const uint32_t p = o.p & kLPrimeMask;  // the prime (>= 2^31: a lane past the table end)
  const float invp = fast_rcp((float)p);
  // Kb mod p. While Kb < 2^32 (values below 1.29e11; wave-uniform) a float
  // quotient is within one of the true one: its relative error is below
  // 2^-22 (Kb rounded to float 2^-24, the rcp 2^-23, the product 2^-24) and
  // q < 2^32 / p < 2^22 for p > TB (kQuotBits), so |error| < 1, and the
  // truncation adds at most one more: Kb - q p is in (-p, 2p), corrected by
  // two unsigned min steps; the 64-bit Barrett reduction covers Kb >= 2^38.
  uint32_t kbm;
  if (Kb < (1ull << 32)) {
    const uint32_t q = (uint32_t)((float)(uint32_t)Kb * invp);
    // q p by v_mul_u32_u24 as asm: written as __umul24 the compiler merged it
    // with the other path's product into one quarter-rate v_mul_lo_u32
    uint32_t qp;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(qp) : "v"(q), "v"(p));
    uint32_t x = (uint32_t)Kb - qp;  // in (-p, 2p) as a signed value; p < 2^24
    x = min(x, x + p);
    kbm = min(x, x - p);
  } else if (!BARRETT || Kb < (1ull << 38)) {
    // values below 8.2e12: the float quotient of Kb is within kQuotErr38 of
    // the true one (relative error < 2^-22, Kb / p < 2^38 / (TB + 1)), so
    // Kb - q p is exact in 32 bits (|.| < (kQuotErr38 + 1) p < 2^31, asserted
    // below); one more float quotient of that rest leaves it in (-p, 2p). 12
    // VALU where the 64-bit Barrett reduction takes ~24.
    const uint32_t q = (uint32_t)((float)Kb * invp);
    const int32_t r = (int32_t)((uint32_t)Kb - q * p);
    const int32_t q2 = (int32_t)((float)r * invp);
    uint32_t x = (uint32_t)(r - __mul24(q2, (int32_t)p));
    x = min(x, x + p);
    kbm = min(x, x - p);
  } else {
    kbm = mod_barrett(Kb, p, o.m);
  }
  const uint32_t nKbm = 0u - kbm;
  const uint32_t pmax = __builtin_amdgcn_readlane(p, 63);
  // some lane not live or with p^2 inside the segment: the set's primes
  // ascend (lanes past the table end hold 2^31 and up), so pmax decides, on
  // the scalar unit (a per-lane 64-bit p^2 and two compares: 1e12 +1.4%)
  const bool none = pmax > sqrt_vs;  // pmax^2 > Vs, sqrt_vs = isqrt(Vs)
  if (!none) {  // every lane live and past p^2: branch-free bodies chosen by the set's plan
    const uint32_t plan = (uint32_t)__builtin_amdgcn_readfirstlane(o.p) >> 20;  // lane 0: live
    const uint32_t n_run = plan >> 3;
    if ((plan & 3) == 2) unit_L_fast<2>(o, p, nKbm, ps, 0);
    else if ((plan & 3) == 1) unit_L_fast<1>(o, p, nKbm, ps, 0);
    else if (!(plan & 4)) unit_L_fast<0>(o, p, nKbm, ps, n_run);
    else unit_L_fast<0, true>(o, p, nKbm, ps, n_run);
    return;
  }
  const uint32_t pmin = __builtin_amdgcn_readfirstlane(p);
  const uint64_t p2 = (uint64_t)p * p;
  const bool live = p2 < Vend;
  const bool slow = p2 > Vs;
  const uint32_t D = slow && live ? (uint32_t)(p2 - Vs) : 0u;
  if (!live) return;
  // read here, not passed in: the compiler rematerialises a kernel-argument
  // value by a scalar load, and hoisted into the common path that load (with
  // the s_waitcnt lgkmcnt(0) before its register is reused) drained every
  // wave's outstanding marks once per set
  const uint64_t rho_pack = *(volatile const uint64_t*)rho_pack_p;
  // Primes above KP/2 mark branch-free: two marks, dropped past the segment.
#pragma unroll
  for (uint32_t q = 0; q < 8; ++q) {
    uint32_t kk = plane_start(o.a[q], nKbm, ps.ne[q], p);
    if (slow) {
      const uint32_t pl = (pl_rot >> (3 * q)) & 7u;
      const uint32_t rho = (uint32_t)(rho_pack >> (5 * pl)) & 31u;
      const uint32_t kmin = kmin_for(D, rho);
      if (kmin > kk) {
        const uint32_t d = kmin - kk;  // < 2^18
        uint32_t qd = (uint32_t)((float)d * invp);
        while (qd * p < d) ++qd;
        while (qd > 0 && (qd - 1) * p >= d) --qd;
        kk += qd * p;
      }
    }
    const uint32_t pb4 = ps.pb[q];
    if (pmin > KP / 2) {
      mark_k(pb4, kk, ps.one);
      mark_k(pb4, kk + p, ps.one);
    } else {
      for (; kk < KP; kk += p) mark_k(pb4, kk, ps.one);
    }
  }
}

constexpr uint32_t kBkBatchU = 16;                                // loads in flight per lane (bucket unit)
constexpr uint32_t kBkUnit = 64 * kBkBatchU * DSE_BK_UNIT_BATCHES;  // band-1 entries per bucket unit
constexpr uint32_t kBkGrid0 = DSE_BK_GRID;                         // band-0 columns (fill workgroups)
#ifndef DSE_BK0_LISTS
#define DSE_BK0_LISTS 16
#endif
constexpr uint32_t kBk0Lists = DSE_BK0_LISTS;                      // band-0 columns per bucket unit
static_assert(kBkGrid0 % kBk0Lists == 0 && 64 % kBk0Lists == 0, "band-0 bucket units");

struct WheelLdsLow {
  uint64_t mid_m[kMidCap];         // Barrett factors of the staged mid primes
  uint32_t mid_p[kMidCap];         // p | (30^{-1} mod p) << 16
  uint32_t mid_x[kMidCap];         // Vs mod p of this workgroup's segment (MidRes)
  uint32_t mid_inc[kMidCap];       // G W mod p
  uint32_t x_seg;                  // the launch segment mid_x holds (~0: none)
  uint32_t lut[kMaxRanges][256];   // per range: period byte -> 15 odd slots
  uint4 itab[kGDW];                // init tables U_G, 4 copies shifted by 0..3 dwords (kGDW / 4 blocks each)
  uint32_t thr[5];
  uint32_t ctr;                    // unit counter
  unsigned long long rcnt[kMaxRanges];  // per range: primes counted by this workgroup
};
static_assert(sizeof(WheelLdsLow) <= kImgOff, "LDS below the image");
struct WheelLds : WheelLdsLow {
  uint8_t pad[kImgOff - sizeof(WheelLdsLow)];
  uint32_t img[IMG_WORDS];         // the segment image, at LDS byte kImgOff, the top of the allocation
};
static_assert(sizeof(WheelLds) == kImgOff + IMG_BYTES, "the image ends the allocation");

// BK: the range has bucketed primes (wa.bk_*). Two instantiations, so the
// ranges without (N up to 1.1e12) run a unit loop without the bucket code
// (with it, the loop's SGPR spills doubled and 1e11 ran 1.9% slower).
template <bool BK>
__global__ __launch_bounds__(NT) void wheel_segments_kernel(const void* __restrict__ table, WheelArgs wa) {
  // One static LDS object at LDS address 0, so the image sits at kImgOff,
  // the value every mark's ds_or adds in its offset field.
  __shared__ WheelLds lds;
  uint64_t* const s_mid_m = lds.mid_m;
  uint32_t* const s_mid_p = lds.mid_p;
  uint32_t* const s_thr = lds.thr;

  const TableHeader* th = reinterpret_cast<const TableHeader*>(table);
  const uint32_t np = th->count;
  const uint32_t* __restrict__ P = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + 16);
  const uint64_t* __restrict__ M =
      reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(table) + table_m_offset(th->cap));
  const uint32_t* __restrict__ A =
      reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + table_a_offset(th->cap));
  // the L list's words p | plan << 20 for this geometry (table pl[0] / pl[1])
  const uint32_t* __restrict__ PL = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) +
                                                                    table_l_offset(th->cap)) +
                                    (kWheelLogKP == 17 ? 0u : th->cap);

#if defined(DSE_PAD_NOPS) && DSE_PAD_NOPS > 0
  // code-placement A/B only: shifts the kernel's instruction stream by 4 B each
  asm volatile(".rept " DSE_STR(DSE_PAD_NOPS) "\n\ts_nop 0\n\t.endr");
#endif
  const uint32_t tid = threadIdx.x, lane_id = tid & 63, wave = tid >> 6;

  if (tid == 0) {
    // first index with p > kQMax, > TA, > TB1, > TB (capped by the LDS stage),
    // > kWheelMaxPrime (bucketed or absent): the table holds every odd prime
    // from 3 up, so these are the host's prime counts (wa.nthr), capped by
    // the table's size
    s_thr[0] = min(wa.nthr[0], np);
    s_thr[1] = min(wa.nthr[1], np);
    s_thr[2] = min(wa.nthr[2], np);
    s_thr[3] = min(min(wa.nthr[3], np), s_thr[0] + kMidCap);
    s_thr[2] = min(s_thr[2], s_thr[3]);
    s_thr[4] = max(s_thr[3], min(wa.nthr[4], np));
    lds.ctr = 0;
    lds.x_seg = ~0u;
  }
  if (tid < kMaxRanges) lds.rcnt[tid] = 0;
  for (uint32_t x = tid; x < 256 * wa.nranges; x += NT) {
    const uint32_t v8 = x & 255;
    const uint64_t rho_pack = wa.r[x >> 8].rho_pack;
    uint32_t v = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
      const uint32_t rho = (uint32_t)(rho_pack >> (5 * i)) & 31u;
      if (!(v8 & (1u << i))) v |= 1u << ((rho - 1) >> 1);  // plane bit i clear: prime
    }
    // composite bits of the 8 planes -> prime odd slots of the period, filed
    // under v ^ 3 (v >> 5) (see expand_segment)
    lds.lut[x >> 8][v8 ^ (3u * (v8 >> 5))] = v;
  }
  for (uint32_t idx = tid; idx < 4 * kGDW; idx += NT) reinterpret_cast<uint32_t*>(lds.itab)[idx] = g_init_tables.w[idx];
  __syncthreads();
  const uint32_t i_mid0 = s_thr[0], i_midB = s_thr[1], i_midB2 = s_thr[2], i_mid1 = s_thr[3];
  for (uint32_t i = tid; i < i_mid1 - i_mid0; i += NT) {
    const uint32_t q = P[i_mid0 + i];
    s_mid_p[i] = q | ((uint32_t)inv30_of(q) << 16);  // p < 2^14, 30^{-1} mod p < p
    s_mid_m[i] = M[i_mid0 + i];
    lds.mid_inc[i] = (uint32_t)(((uint64_t)gridDim.x * kWheelSpan) % q);
  }
  // Work units: list 1 = nA single mid primes (A), nB1 units of two primes
  // (B1), nB2 units of 8 primes (B2); list 2 = nL large units (two sets of 64
  // primes each); handed out through one dynamic queue. Issue arbitration
  // favours older waves, so any static split finishes the youngest waves
  // last; the queue makes them take fewer units instead.
  const uint32_t nA = i_midB - i_mid0;
  const uint32_t n_mid = i_mid1 - i_mid0;
  const uint32_t n_b1 = i_midB2 - i_mid0;      // staged index where B2 starts
  const uint32_t nB1 = (i_midB2 - i_midB + 1) / 2;
  const uint32_t nB2 = (i_mid1 - i_midB2 + 7) / 8;
  const uint32_t i_big = s_thr[4];             // L units end here
  constexpr uint32_t kLU = 128;                // primes per L unit
  const uint32_t n1 = nA + nB1 + nB2;

  const uint32_t nseg = wa.nseg;
  const uint32_t grid = gridDim.x;
  const uint32_t T = blockIdx.x < nseg ? (nseg - 1 - blockIdx.x) / grid + 1 : 0u;  // rounds
  // launch segment g -> its range (uniform: a scan of <= kMaxRanges starts)
  auto range_of = [&](uint32_t g) -> uint32_t {
    uint32_t r = 0;
    for (uint32_t i = 1; i < wa.nranges; ++i) r = g >= wa.r[i].seg0 ? i : r;
    return r;
  };

  // ---- init: small-prime patterns (7..61) of segment s into the image. Lane
  // (plane L & 7, run q = 8 w + (L >> 3)) of wave w writes its plane's words
  // of a run of about kInitWords consecutive blocks inside the wave's
  // [kExpandBlocks w, +kExpandBlocks): the blocks this wave expands, so it
  // may init them right after expanding.
  auto init_segment = [&](uint32_t* __restrict__ img, uint32_t g_seg) {
    const WheelRange& rg = wa.r[range_of(g_seg)];
    const uint64_t s = g_seg - rg.seg0;  // the range's segment
    uint32_t lane = lane_id;
    asm volatile("" : "+v"(lane));
    const uint32_t pl = lane & 7, q = 8 * wave + (lane >> 3);
    const uint32_t rho = (uint32_t)(rg.rho_pack >> (5 * pl)) & 31u;
    constexpr uint32_t R = kInitWords;  // words per lane
    static_assert(R % 4 == 0, "staggered init runs");
    // a half-wave's four lanes of one plane (j = 0..3) cover a region of 4R
    // blocks with runs of R + 1, R + 1, R + 1 and R - 3 blocks starting at
    // (R + 1) j: at step r they write blocks j + r (mod 4) -- distinct banks
    // (runs of R from multiples of R put all four on one bank: 4-way, 1%
    // of the kernel, profiles/r04/ab_init_stagger_1e11.txt)
    const uint32_t j = q & 3;
    const uint32_t b0 = 4 * R * (q >> 2) + (R + 1) * j;
    const uint32_t k0 = 32 * b0;        // its first period
    constexpr uint32_t H = 16;          // words per pass (bounds the registers: 16 acc + 20 read)
    static_assert(R % H == 0 && H % 4 == 0, "init passes");
    uint32_t boff[kNG], bsh[kNG];       // per group: the lane's first aligned 16-byte block, bit shift
    // rho takes 8 values over the lanes: left visible, the compiler evaluates
    // the group offsets for all 8 on the scalar unit and selects per lane
    // (a 6.8x SALU blow-up, 33 ms kernels); opaque, it is one VALU chain.
    const uint32_t rho_o = opaque(rho), k0_o = opaque(k0);
#pragma unroll
    for (int g = 0; g < kNG; ++g) {
      const uint32_t Mg = gmod(g);
      const uint32_t wg = (uint32_t)(kWheelSpan % Mg);
      const uint32_t sg = (uint32_t)(s % Mg);
      const uint32_t x = ((uint32_t)rg.v0g[g] + sg * wg + rho_o) % Mg;  // (Vs + rho) mod M_G
      const uint32_t o = (k0_o + x * kGInv30[g]) % Mg;                  // bit offset of period k0
      const uint32_t d0 = o >> 5, kc = d0 & 3;
      boff[g] = (kc * kGDW + gbase(g) + d0 - kc) / 4;                    // 16-byte block index
#if DSE_FAKE_CF_INIT  // profiling knockout: a 16-lane read group on consecutive 16-byte blocks (wrong patterns)
      boff[g] = gbase(g) / 4 + (lane & 15u);
#endif
      bsh[g] = o & 31;
    }
    uint32_t* const wp = img + 8 * b0 + pl;
#pragma unroll
    for (uint32_t h = 0; h < R; h += H) {
      uint32_t acc[H];
#pragma unroll
      for (uint32_t r = 0; r < H; ++r) acc[r] = 0;
#pragma unroll
      for (int g = 0; g < kNG; ++g) {
        const uint4* bp = lds.itab + boff[g] + h / 4;
        uint32_t blk[H + 4];
#pragma unroll
        for (uint32_t b = 0; b < H / 4 + 1; ++b) {
          const uint4 v = bp[b];
          blk[4 * b] = v.x; blk[4 * b + 1] = v.y; blk[4 * b + 2] = v.z; blk[4 * b + 3] = v.w;
        }
#pragma unroll
        for (uint32_t r = 0; r < H; ++r) acc[r] |= __builtin_amdgcn_alignbit(blk[r + 1], blk[r], bsh[g]);
        asm volatile("" ::: "memory");  // keep the next group's reads after these (register pressure)
      }
#pragma unroll
      for (uint32_t r = 0; r < H; ++r) {
        if (h + r >= R - 3 && j == 3) continue;  // the short run
        wp[8 * (h + r)] = acc[r];
      }
    }
    if (j != 3) {  // word R of the long runs
      uint32_t acc = 0;
#pragma unroll
      for (int g = 0; g < kNG; ++g) {
        const uint4* bp = lds.itab + boff[g] + R / 4;
        const uint4 v = bp[0];
        acc |= __builtin_amdgcn_alignbit(v.y, v.x, bsh[g]);
      }
      wp[8 * R] = acc;
    }
  };

  // ---- expand segment s to odd-only bits, count, store: each lane reads one
  // block (all 8 planes of 32 periods: 32 contiguous bytes, two
  // ds_read_b128); wave w takes blocks [kExpandBlocks w, +kExpandBlocks), 64
  // per step. ds_read_b128 serves a wave in 4 lane groups of 16 ({0-3,12-15,
  // 20-27}, {4-11,16-19,28-31} and the same + 32, MI355X_MICROARCH.md section
  // LDS); lane m of group g takes block 16 g + m of the step, so a group's
  // read touches each of 32 banks twice (having lanes m >= 8 read their upper
  // 16 bytes first covered all 64 once, but cost 8 v_cndmask per block to
  // put the halves back: 1e11 +0.4%, profiles/r05/ab_expand_reads.txt).
  // Output words 15 R .. 15 R + 14 of block R: a wave stores 3,840
  // contiguous bytes per step.
  auto expand_segment = [&](const uint32_t* __restrict__ img, uint32_t g_seg) {
    const uint32_t ri = range_of(g_seg);
    const WheelRange& rg = wa.r[ri];
    const uint64_t s = g_seg - rg.seg0;  // the range's segment
    const uint64_t out_words = 2ull * ((rg.nbits + 63) / 64);  // 32-bit words of the caller's mask
    uint32_t* __restrict__ out = rg.out;
    const uint32_t* __restrict__ s_lut = lds.lut[ri];
    uint32_t my_count = 0;
    uint32_t lane = lane_id;
    asm volatile("" : "+v"(lane));
    const uint32_t l = lane & 31;
    const uint32_t gsub = (l >= 4 && l < 12) || (l >= 16 && l < 20) || l >= 28;
    const uint32_t m = l < 4 ? l : l < 12 ? l - 4 : l < 20 ? l - 8 : l < 28 ? l - 12 : l - 16;
    const uint32_t bl = 16 * (2 * (lane >> 5) + gsub) + m;  // block within the step
    const uint64_t seg_word0 = s * (uint64_t)kOutWordsPerSeg;
#pragma unroll 1
    for (uint32_t t = 0; t < kExpandBlocks / 64; ++t) {
      const uint32_t blk = kExpandBlocks * wave + 64 * t + bl;
      const uint4* rp = reinterpret_cast<const uint4*>(img + 8 * blk);
      const uint4 lo = rp[0], hi = rp[1];
      uint32_t W[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};  // composite bits of planes 0..7
      // composite candidates of the block's 256 (8 planes x 32 periods), from
      // the raw words (the transpose keeps it): 8 v_bcnt instead of 15 over
      // the output words; the range's first block (small primes put back by
      // rg.fix) and its end count the output instead
      uint32_t n_comp = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) n_comp += __popc(W[j]);
      // Transpose every byte column of the 8 x 32 bit matrix in place (rows =
      // planes): afterwards W[j] byte q bit i = plane i, period 8q + j.
      bit_block_swaps(W);
      // LUT index of every period byte v: v ^ 3 (v >> 5), a bijection that
      // puts the common bytes (all composite, one prime) in distinct banks
      // (indexed by v, 255 / 223 / 191 / 127 would share bank 31)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t h = (W[j] >> 5) & 0x07070707u;
        W[j] ^= h + (h << 1);  // 3h <= 21: no carry into the next byte
      }
      uint32_t o[15];
#pragma unroll
      for (int w = 0; w < 15; ++w) o[w] = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t e = s_lut[(W[j] >> (8 * q)) & 0xFFu];
          const int pos = 15 * (8 * q + j);
          o[pos >> 5] |= e << (pos & 31);
          if ((pos & 31) > 17) o[(pos >> 5) + 1] |= e >> (32 - (pos & 31));
        }
      }
      const uint64_t w0 = seg_word0 + 15ull * blk;  // caller's 32-bit word index
      if (s == 0 && blk == 0) {
        o[0] |= (uint32_t)rg.fix;
        o[1] |= (uint32_t)(rg.fix >> 32);
      }
      const uint64_t bit0 = 32ull * w0;
      if (bit0 + 480 <= rg.nbits) {  // whole block inside the range (a separate path: no phi copies of o[])
        uint32_t cnt = 0;
        if (s == 0 && blk == 0) {
#pragma unroll
          for (int w = 0; w < 15; ++w) cnt += __popc(o[w]);
        } else {
          cnt = 256u - n_comp;
        }
        my_count += cnt;
        if (out) {
#pragma unroll
          for (int w = 0; w < 15; ++w) out[w0 + w] = o[w];
        }
      } else {  // range end (last segment only): mask, count, store what is inside the caller's words
        const uint32_t rem = bit0 >= rg.nbits ? 0u : (uint32_t)(rg.nbits - bit0);  // < 480 valid bits
        uint32_t cnt = 0;
#pragma unroll
        for (int w = 0; w < 15; ++w) {
          const uint32_t b = 32u * w;
          o[w] = b >= rem ? 0u : (rem - b >= 32 ? o[w] : o[w] & ((1u << (rem - b)) - 1u));
          cnt += __popc(o[w]);
        }
        my_count += cnt;
        if (out) {
#pragma unroll
          for (int w = 0; w < 15; ++w)
            if (w0 + w < out_words) out[w0 + w] = o[w];
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) my_count += __shfl_xor(my_count, o);
    if (lane == 0 && my_count) atomicAdd(&lds.rcnt[ri], (unsigned long long)my_count);
  };

  // ---- mark segment s into image img -------------------------------------
  auto mark_segment = [&](uint32_t* __restrict__ img, uint32_t g_seg) {
    const WheelRange& rg = wa.r[range_of(g_seg)];
    const uint64_t s = g_seg - rg.seg0;  // the range's segment
    const uint64_t Vs = rg.V0 + s * kWheelSpan;  // segment base value
    const uint64_t Vend = Vs + kWheelSpan;
    // Lane-derived values are segment-invariant; left visible, the compiler
    // hoists dozens of them out of the round loop and spills them. Recompute.
    uint32_t lane = lane_id;
    asm volatile("" : "+v"(lane));
    const uint32_t img0 = lds_addr(img) - kImgOff;  // 0: mark addresses are image-relative
    const uint32_t one = opaque(1u);
    // Bucketed hits of the primes > 2^kBucketLoLog as units of the queue,
    // interleaved with the marking units, so their global-load latency
    // overlaps other waves' marking instead of stalling every wave at the
    // segment start: n0u band-0 units (kBk0Lists columns each), then band-1
    // units of kBkUnit entries, then one unit over the spill list if it is
    // not empty.
    uint32_t bk_b0 = 0, bk_b1 = 0, n0u = 0, n1u = 0, n3 = 0;
    if (BK) {
      n0u = wa.bk_k0 ? kBkGrid0 / kBk0Lists : 0u;
      bk_b0 = wa.bk_start[s];
      bk_b1 = wa.bk_start[s + 1];
      n1u = (bk_b1 - bk_b0 + kBkUnit - 1) / kBkUnit;
      n3 = n0u + n1u + (wa.bk_k0 && *wa.bk_nspill ? 1u : 0u);
    }
    // the range's rho_pack in the kernel-argument segment (after the table
    // pointer), for unit_L's rare slow path: not &rg.rho_pack, which would
    // make the compiler copy the whole argument block to scratch
    const uint64_t* rho_pack_p = reinterpret_cast<const uint64_t*>(
        (const char*)__builtin_amdgcn_kernarg_segment_ptr() + kWaOffset +
        range_of(g_seg) * sizeof(WheelRange) + offsetof(WheelRange, rho_pack));
    uint32_t sqrt_vs = (uint32_t)__builtin_sqrt((double)Vs);  // isqrt(Vs) < 2^32 (Vs < 2^64)
    while ((uint64_t)sqrt_vs * sqrt_vs > Vs) --sqrt_vs;
    while ((uint64_t)(sqrt_vs + 1) * (sqrt_vs + 1) <= Vs) ++sqrt_vs;
    sqrt_vs = __builtin_amdgcn_readfirstlane(sqrt_vs);
    uint32_t sqrt_ve = (uint32_t)__builtin_sqrt((double)(Vend - 1));  // p^2 < Vend <=> p <= isqrt(Vend - 1)
    while ((uint64_t)sqrt_ve * sqrt_ve > Vend - 1) --sqrt_ve;
    while ((uint64_t)(sqrt_ve + 1) * (sqrt_ve + 1) <= Vend - 1) ++sqrt_ve;
    sqrt_ve = __builtin_amdgcn_readfirstlane(sqrt_ve);
    const uint32_t rot = (i_mid1 + lane) & 7;  // = table index & 7 of this lane's large primes
    // absolute residue (q + rot) & 7 at step q: its plane and e bit
    const uint32_t pl_rot = ((rg.pl_pack >> (3 * rot)) | (rg.pl_pack << (24 - 3 * rot))) & 0xFFFFFFu;
    const uint32_t e_rot = ((rg.e_iota >> rot) | (rg.e_iota << (8 - rot))) & 0xFFu;
    PlaneSteps ps;
    ps.one = one;
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
      ps.pb[q] = img0 + 4 * ((pl_rot >> (3 * q)) & 7u) + (DSE_FAKE_CF_L ? ((lane_id >> 3) & 3u) << 5 : 0u);
      ps.ne[q] = 0u - ((e_rot >> q) & 1u);
    }
    const uint64_t Kb = rg.KB0 + s * (uint64_t)KP;
    const bool need_m = BK && Kb >= (1ull << 38);  // unit_L's Barrett path (unit_L<BK>)
    MidRes mr;
    mr.x = lds.mid_x;
    mr.inc = lds.mid_inc;
    mr.have = __builtin_amdgcn_readfirstlane(lds.x_seg) == g_seg;
    // One dynamic queue over both lists, interleaved (list 1 at even, list 2
    // at odd positions while both last). Claims run two units ahead: the LDS
    // atomic for unit j+2 is issued when unit j starts and read when it ends
    // (by then this wave's marks of unit j have drained), and a large unit's
    // operands are loaded while the unit before it runs.
    // large units of this segment: up to its piece's bound (WheelRange::lcap)
    const uint32_t i_live = max(i_mid1, min(i_big, rg.lcap[min((uint32_t)(s >> rg.lsh), kLPieces - 1)]));
    const uint32_t n2 = (i_live - i_mid1 + kLU - 1) / kLU;
    const uint32_t n_int = min(n1, n2), n_all = n1 + n2;
    // The claim is an asm ds_add_rtn: written as a C++ atomic, the AMDGPU
    // atomic optimizer aggregates it over the wave and waits for its return
    // on the spot (draining the previous unit's marks with it), which
    // defeats the two-ahead issue. Read through claimed().
    const uint32_t ctr_addr = lds_addr(&lds.ctr);
    auto claim = [&]() -> uint32_t {
      uint32_t j = 0;
      if (lane == 0) asm volatile("ds_add_rtn_u32 %0, %1, %2" : "=v"(j) : "v"(ctr_addr), "v"(1u) : "memory");
      return j;  // per-lane value; lane 0 holds the claim
    };
    auto claimed = [&](uint32_t j) -> uint32_t {
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(j)::"memory");
      return __builtin_amdgcn_readlane(j, 0);
    };
    auto is_l = [&](uint32_t u) -> bool { return u < 2 * n_int ? (u & 1) != 0 : n2 > n1; };
    auto idx_of = [&](uint32_t u) -> uint32_t { return u < 2 * n_int ? u >> 1 : u - n_int; };
    // queue position -> marking unit (or ~0u: bucket unit bk_of(q)); the n3
    // bucket units interleave 1:1 with the marking units from the start
    const uint32_t mb = min(n3, n_all), n_q = n_all + n3;
    auto unit_of = [&](uint32_t q) -> uint32_t {
      if (q < 2 * mb) return (q & 1) ? ~0u : q >> 1;
      return n3 > n_all ? ~0u : q - mb;
    };
    auto bk_of = [&](uint32_t q) -> uint32_t { return q < 2 * mb ? q >> 1 : q - mb; };
    // a claimed queue position, decoded once: kind << 30 | index (kind 0: a mid
    // unit of list 1, 1: a large unit, 2: a bucket unit), ~0u past the end
    constexpr uint32_t kIdx = (1u << 30) - 1;
    auto decode = [&](uint32_t q) -> uint32_t {
      if (q >= n_q) return ~0u;
      const uint32_t u = unit_of(q);
      if (u == ~0u) return 2u << 30 | bk_of(q);
      return (is_l(u) ? 1u << 30 : 0u) | idx_of(u);
    };
    // Operands are only ever loaded into nxt and copied to cur at the top of
    // an iteration, after they have landed: had the first unit's loads gone
    // straight into cur, the compiler's wait analysis, merging that entry
    // with the loop's back edge, waited inside every unit for the next unit's
    // loads just issued (a vmcnt(4) and a vmcnt(0) per large unit).
    LargeOps cur, nxt;
    LargeOps cur1, nxt1;  // the unit's second 64 primes
    uint32_t d_nxt = decode(claimed(claim()));
    if ((d_nxt >> 30) == 1) {
      load_L(nxt, PL, M, A, i_mid1 + kLU * (d_nxt & kIdx) + lane, i_big, need_m);
      load_L(nxt1, PL, M, A, i_mid1 + kLU * (d_nxt & kIdx) + 64 + lane, i_big, need_m);
    }
    uint32_t d_after = decode(claimed(claim()));
    // the first unit's operands landed before the loop (an asm that reads
    // them makes the compiler wait here), so on no path into the loop does a
    // set's register still wait for a load
    asm volatile("" ::"v"(nxt.p), "v"(nxt.a[0]), "v"(nxt.a[1]), "v"(nxt.a[2]), "v"(nxt.a[3]), "v"(nxt.a[4]),
                 "v"(nxt.a[5]), "v"(nxt.a[6]), "v"(nxt.a[7]), "v"(nxt1.p), "v"(nxt1.a[0]), "v"(nxt1.a[1]),
                 "v"(nxt1.a[2]), "v"(nxt1.a[3]), "v"(nxt1.a[4]), "v"(nxt1.a[5]), "v"(nxt1.a[6]), "v"(nxt1.a[7]));
    for (;;) {
      cur = nxt;
      cur1 = nxt1;
      undef_ops(nxt);  // dead until the next unit's loads: cur and nxt are never one register
      undef_ops(nxt1);
      const uint32_t d_cur = d_nxt;
      d_nxt = d_after;
      if (d_cur == ~0u) break;
      // issued and read in the same iteration: the asm output is written when
      // the LDS returns it, so the value must not be live across a loop phi
      // (a register copy there reads it early; a claim carried from one
      // iteration into the next gave wrong counts)
      const uint32_t c2 = claim();  // unit after next, read at the end of this one
      if ((d_nxt >> 30) == 1) {
        load_L(nxt, PL, M, A, i_mid1 + kLU * (d_nxt & kIdx) + lane, i_big, need_m);
        load_L(nxt1, PL, M, A, i_mid1 + kLU * (d_nxt & kIdx) + 64 + lane, i_big, need_m);
      }
      if (BK && (d_cur >> 30) == 2) {  // a bucket unit, kBkBatchU loads in flight per lane
        const uint32_t bu = d_cur & kIdx;
        if (bu < n0u) {  // band 0: columns kBk0Lists bu .. +kBk0Lists, 4 at a time, each read by the whole wave
          const uint64_t li0 = s * (uint64_t)kBkGrid0 + bu * kBk0Lists;
          const uint32_t nl = lane < kBk0Lists ? wa.bk_n0[li0 + lane] : 0u;
#pragma unroll 1
          for (uint32_t g = 0; g < kBk0Lists; g += 4) {
            uint32_t n[4], nmax = 0;
            const uint32_t* __restrict__ r[4];
#pragma unroll
            for (uint32_t l = 0; l < 4; ++l) {
              n[l] = min((uint32_t)__builtin_amdgcn_readlane((int)nl, (int)(g + l)), wa.bk_k0);
              r[l] = wa.bk_reg0 + ((uint64_t)(bu * kBk0Lists + g + l) * wa.nseg + s) * wa.bk_k0;
              nmax = max(nmax, n[l]);
            }
            for (uint32_t o = lane; o < nmax + lane; o += 256) {  // contiguous 256-entry pieces of 4 lists
              uint32_t e[16];
#pragma unroll
              for (uint32_t l = 0; l < 4; ++l)
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t)
                  e[4 * l + t] = o + 64 * t < n[l] ? __builtin_nontemporal_load(r[l] + o + 64 * t) : 0u;
#pragma unroll
              for (uint32_t l = 0; l < 4; ++l)
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t)
                  if (o + 64 * t < n[l]) mark_entry(img0, e[4 * l + t], one);
            }
          }
        } else if (bu < n0u + n1u) {  // band 1: kBkUnit entries of the segment's list
          const uint32_t beg = bk_b0 + (bu - n0u) * kBkUnit, end = min(bk_b1, beg + kBkUnit);
          for (uint32_t j = beg + lane; j < end; j += 64 * kBkBatchU) {
            uint32_t e[kBkBatchU];
#pragma unroll
            for (uint32_t t = 0; t < kBkBatchU; ++t)
              e[t] = j + 64 * t < end ? __builtin_nontemporal_load(wa.bk_entries + j + 64 * t) : 0u;
#pragma unroll
            for (uint32_t t = 0; t < kBkBatchU; ++t)
              if (j + 64 * t < end) mark_entry(img0, e[t], one);
          }
        } else {  // the spill list (band-0 regions that overflowed): this segment's hits
          const uint32_t ns = (uint32_t)min((uint64_t)*wa.bk_nspill, wa.bk_spill_cap);
          for (uint32_t j = lane; j < ns; j += 64) {
            const unsigned long long v = wa.bk_spill[j];
            if ((uint32_t)(v >> 32) == (uint32_t)s) mark_entry(img0, (uint32_t)v, one);
          }
        }
        d_after = decode(claimed(c2));
        continue;
      }
      const uint32_t k = d_cur & kIdx;
      if ((d_cur >> 30) == 0) {
        if (k < nA) {
          const uint32_t pi = __builtin_amdgcn_readfirstlane(s_mid_p[k]);
          const uint32_t p = pi & 0xFFFFu;
          const uint64_t m = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(s_mid_m[k] >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)s_mid_m[k]);
          if ((uint64_t)p * p < Vend) unit_A(img0, pi, m, mr, k, Vs, rg.rho_pack, lane, one);
        } else if (k < nA + nB1) {
          const uint32_t j0 = nA + (k - nA) * 2;
          const uint32_t pf = __builtin_amdgcn_readfirstlane(s_mid_p[j0]) & 0xFFFFu;
          if ((uint64_t)pf * pf < Vend)
            unit_B1(img0, s_mid_p, s_mid_m, mr, j0, min(2u, n_b1 - j0), Vs, rg.rho_pack, lane, one);
        } else {
          const uint32_t j0 = n_b1 + (k - nA - nB1) * 8;
          const uint32_t pf = __builtin_amdgcn_readfirstlane(s_mid_p[j0]) & 0xFFFFu;
          if ((uint64_t)pf * pf < Vend)
            unit_B2(img0, s_mid_p, s_mid_m, mr, j0, min(8u, n_mid - j0), Vs, Vend, rg.rho_pack, lane, one);
        }
      } else {
        // a set marks if its first prime's square is below the segment's end
        const uint32_t p0 = __builtin_amdgcn_readfirstlane(cur.p) & kLPrimeMask;
        if (p0 <= sqrt_ve) unit_L<BK>(cur, Vs, Vend, Kb, ps, pl_rot, rho_pack_p, sqrt_vs);
        const uint32_t p1 = __builtin_amdgcn_readfirstlane(cur1.p) & kLPrimeMask;
        if (p1 <= sqrt_ve) unit_L<BK>(cur1, Vs, Vend, Kb, ps, pl_rot, rho_pack_p, sqrt_vs);
      }
      d_after = decode(claimed(c2));
    }
  };

  if (T > 0) init_segment(lds.img, blockIdx.x);
  __syncthreads();
  for (uint32_t t = 0; t < T; ++t) {
    const uint32_t s = blockIdx.x + t * grid;
    mark_segment(lds.img, s);
    lds_drain();
    __syncthreads();
    expand_segment(lds.img, s);
    // init of this workgroup's next segment, on the rows this wave just
    // expanded: no barrier in between, and waves drift into init while
    // others still expand
    if (t + 1 < T) init_segment(lds.img, s + grid);
    if (tid == 0) {
      lds.ctr = 0;  // all claims of this segment returned before the barrier above
      // the mid units left their residues for segment s + grid: valid if it is
      // of the same range and every mid unit ran (p^2 < Vs for p <= TB)
      const uint32_t r0 = range_of(s), r1 = range_of(s + grid);
      const uint64_t Vs = wa.r[r0].V0 + (uint64_t)(s - wa.r[r0].seg0) * kWheelSpan;
      lds.x_seg = t + 1 < T && r1 == r0 && Vs >= (uint64_t)TB * TB ? s + grid : ~0u;
    }
    __syncthreads();
  }

  if (tid < wa.nranges && lds.rcnt[tid]) atomicAdd(wa.r[tid].count, lds.rcnt[tid]);
}

#if DSE_WHEEL_MAIN_TU
// floor((2^64-1)/p) for 2 <= p < 2^32 without a 64-bit division: a double
// quotient (relative error 2^-52, so off by < 2^11) corrected by the exact
// remainder, itself below 2^43 in magnitude and so exact in a double.
__device__ __forceinline__ uint64_t barrett_factor(uint32_t p) {
  const double dp = (double)p;
  uint64_t m = (uint64_t)(18446744073709551615.0 / dp);        // rounds 2^64-1 up to 2^64: may overshoot
  if (m > ~0ull / 2) m = ~0ull / 2;                              // p >= 2: the true m < 2^63
  int64_t r = (int64_t)(~0ull - m * (uint64_t)p);                // true remainder + (true m - m) * p
  m += (int64_t)__builtin_floor((double)r / dp);
  r = (int64_t)(~0ull - m * (uint64_t)p);
  while (r < 0) { --m; r += p; }
  while (r >= (int64_t)p) { ++m; r -= p; }
  return m;
}

// m[i] = floor((2^64-1)/p) and the rotated wheel-offset row of every table
// prime: a[8i + ((j - i) & 7)] = first k >= 0 with p | R30[j] + 30k (p >= 7).
__global__ void wheel_offsets_kernel(void* __restrict__ table) {
  const TableHeader* h = reinterpret_cast<const TableHeader*>(table);
  const uint32_t n = h->count == 0xFFFFFFFFu ? 0u : h->count;
  const uint32_t* P = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + 16);
  uint64_t* M = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(table) + table_m_offset(h->cap));
  uint32_t* A = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(table) + table_a_offset(h->cap));
  uint32_t* PL = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(table) + table_l_offset(h->cap));
  static_assert(kWheelLogKP == 17, "pl[0] is the full geometry's, pl[1] the half geometry's");
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t p = P[i];
    if (p > kWheelMaxPrime) break;  // bucketed primes (P ascends: all later ones too): the walks divide in double precision
    // the plans of the prime's set of 64 in the L list (unit_L), per geometry
    uint32_t plan0 = 0, plan1 = 0;
    if (i >= kL0) {
      const uint32_t s0 = i - (i - kL0) % 64;
      const uint32_t pmin = P[s0], pmax = P[min(s0 + 63, n - 1)];
      plan0 = l_plan(pmin, pmax, 1u << 17);
      plan1 = l_plan(pmin, pmax, 1u << 16);
    }
    PL[i] = p | plan0 << 20;
    PL[h->cap + i] = p | plan1 << 20;
    const uint64_t m = barrett_factor(p);
    M[i] = m;
    if (p < 7) {
#pragma unroll
      for (int j = 0; j < 8; ++j) A[8ull * i + j] = 0;
      continue;
    }
    const uint64_t inv = inv30_of(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t t = kR30[j] % p;
      const uint32_t u = t ? p - t : 0u;
      A[8ull * i + ((j - i) & 7)] = mod_barrett((uint64_t)u * inv, p, m);  // row rotated by i & 7
    }
  }
}

// ---------------------------------------------------------------------------
// Bucketed pass of the ranges whose sqrt(max value) exceeds kWheelMaxPrime
// (high-offset windows) for their primes above 2^kBucketLoLog (or the
// bucket_lo_log2 option): such a prime hits a 3.9 M-integer segment about
// 2^20 / p times (at most twice), so instead of
// visiting every (prime, segment) pair the kernels below walk each prime's
// multiples p*m, gcd(m, 30) = 1, across the whole range once and file every
// hit under its segment (bucket_entry). Band 0 (one level): each fill
// workgroup files its hits into per-(segment, workgroup) regions of a fixed
// capacity, overflow into a spill list. Band 1 (two levels): two identical
// walks, count (LDS per-segment counters -> per-workgroup column) and stage
// (regions from the scanned columns), then a sort by segment. The wheel
// kernel ORs its segment's band-0 regions, band-1 list and spilled hits.
// ---------------------------------------------------------------------------
constexpr uint32_t kBucketThreads = 256;
#ifndef DSE_BK_SEGS
#define DSE_BK_SEGS 8192
#endif
#ifndef DSE_BK_GRID1
#define DSE_BK_GRID1 4096
#endif
// Two bands of bucketed primes: band 0 (p <= split, kBucketGrid workgroups)
// is filled one level, band 1 (p > split, kBucketGrid1 workgroups) staged in
// two levels; the count kernel's columns are band 1's workgroups.
constexpr uint32_t kBucketGrid = DSE_BK_GRID;
constexpr uint32_t kBucketGrid1 = DSE_BK_GRID1;
constexpr uint32_t kBucketCols = kBucketGrid1;
static_assert(kBucketCols % 64 == 0, "column scan: whole lanes");
#ifndef DSE_BK_SPLIT_LOG
#define DSE_BK_SPLIT_LOG 28
#endif
constexpr uint32_t kBucketSplitLog = DSE_BK_SPLIT_LOG;  // production split: primes <= 2^28 one-level
// bucketed ranges bucket the primes above 2^kBucketLoLog (<= kWheelMaxPrime;
// profiles/r05/window_bucket_lo.txt)
constexpr uint32_t kBucketLoLog = 19;
static_assert((1ull << kBucketLoLog) <= kWheelMaxPrime && kBucketLoLog >= 17, "bucket threshold");
constexpr uint32_t kBucketMaxSegs = DSE_BK_SEGS; // segments per pass (LDS counters)
constexpr uint32_t kCoprime30 = (1u << 1) | (1u << 7) | (1u << 11) | (1u << 13) | (1u << 17) | (1u << 19) |
                                (1u << 23) | (1u << 29);
// gap from R30[w] to the next coprime residue: 6 4 2 4 2 4 6 2 (3 bits each)
constexpr uint32_t kGap30 = 6u | (4u << 3) | (2u << 6) | (4u << 9) | (2u << 12) | (4u << 15) | (6u << 18) | (2u << 21);

struct BucketArgs {
  uint64_t V0;         // v_start - 1 of the pass
  uint64_t span;       // integers covered by the pass: nseg * kWheelSpan
  uint64_t plane_lut;  // plane of relative residue rho (odd) in bits [3(rho >> 1), +3)
  uint32_t nseg;       // segments in the pass (<= kBucketMaxSegs)
  uint64_t vmax;       // largest value of the pass (primes with p^2 > vmax have no hits)
  uint64_t split;      // band 0: 2^kBucketLoLog < p <= split, band 1: p > split
};

// Band-0 output of a pass (bucket_fill_wg).
struct BandZero {
  uint32_t* reg0;                  // [kBucketGrid][nseg][k0] regions
  uint32_t* n0;                    // [nseg][kBucketGrid] region fills
  unsigned long long* spill;       // segment << 32 | entry
  uint32_t* nspill;                // spill list length
  uint32_t k0;                     // region capacity
  uint64_t spill_cap;              // spill list capacity (rigorous)
  uint32_t* flag;                  // scratch flag[0] (sticky overflow) ...
  unsigned long long* count;       // ... and bit 63 of the count, if the spill list overflows
};

// First index in [lo, hi) where the ascending table P has P[i] > bound (hi
// if none), by one wave: 64 pivots per step (a step's loads are independent,
// so a 50 M-prime table takes 4 dependent loads instead of 26).
__device__ uint32_t wave_upper_bound(const uint32_t* __restrict__ P, uint32_t lo, uint32_t hi, uint64_t bound,
                                     bool squared) {
  const uint32_t lane = threadIdx.x & 63;
  auto le = [&](uint32_t i) { const uint64_t p = P[i]; return (squared ? p * p : p) <= bound; };
  while (hi - lo > 64) {
    const uint32_t step = (hi - lo + 63) / 64, i = lo + lane * step;
    const uint32_t c = (uint32_t)__popcll(__ballot(i < hi && le(i)));  // pivots at or below the bound
    if (c == 0) return lo;
    const uint32_t nhi = min(hi, lo + c * step);  // the answer is in (pivot c-1, pivot c]
    lo += (c - 1) * step + 1;
    hi = nhi;
  }
  return lo + (uint32_t)__popcll(__ballot(lo + lane < hi && le(lo + lane)));
}

// range[0] = first table index with p > lo_p (the pass's bucket threshold),
// range[1] = first with p^2 > vmax, range[2] = first with p > split (clamped
// to [range[0], range[1]]). One wave.
__global__ __launch_bounds__(64) void bucket_range_kernel(const void* __restrict__ table, uint64_t lo_p, uint64_t vmax,
                                                          uint64_t split, uint32_t* __restrict__ range,
                                                          uint32_t* __restrict__ nspill) {
  const TableHeader* th = reinterpret_cast<const TableHeader*>(table);
  const uint32_t np = th->count == 0xFFFFFFFFu ? 0u : th->count;
  const uint32_t* P = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + 16);
  const uint32_t i_lo = wave_upper_bound(P, 0, np, lo_p, false);
  const uint32_t i_hi = max(i_lo, wave_upper_bound(P, i_lo, np, vmax, true));
  const uint32_t i_sp = wave_upper_bound(P, i_lo, i_hi, split, false);
  if (threadIdx.x == 0) {
    range[0] = i_lo;
    range[1] = i_hi;
    range[2] = i_sp;
    *nspill = 0;  // the band-0 spill list of this pass
  }
}

// First coprime-to-30 multiple of p at or above max(V0 + 1, p^2): its offset
// o from V0 and 3 * (index of the multiplier mod 30 in R30).
__device__ __forceinline__ uint64_t bucket_first(uint32_t p, const BucketArgs& ba, uint32_t& w3) {
  const uint64_t p2 = (uint64_t)p * p;
  const uint64_t vlo = max(ba.V0 + 1, p2);
  // floor(vlo / p) from a double quotient: vlo < 2^62 rounds by < 2^9 and
  // p > 2^17, so the estimate is within 1 of the truth; corrected exactly
  uint64_t q = (uint64_t)((double)vlo / (double)p);
  int64_t rs = (int64_t)(vlo - q * p);
  while (rs < 0) { rs += p; --q; }
  while (rs >= (int64_t)p) { rs -= p; ++q; }
  const uint64_t r = (uint64_t)rs;
  const uint64_t m0 = q + (r != 0);
  const uint32_t r30 = (uint32_t)(m0 % 30);
  const uint32_t d = __builtin_ctz(kCoprime30 >> r30);
  w3 = 3 * __popc(kCoprime30 & ((1u << (r30 + d)) - 1));
  return (uint64_t)p * (m0 + d) - ba.V0;
}

// The hit at offset o (< span): its segment s and entry = the LDS word index
// of (period k, plane) in the wheel kernel's image << 5 | k & 31, i.e. the
// address and bit the wheel kernel ORs, decoded here where the walk has VALU
// to spare (the fill kernels are bound by their stores), not in the wheel
// kernel (mark_entry). Word index = 8 * block + plane < 2^15, so an entry is
// < 2^20.
__device__ __forceinline__ uint32_t bucket_entry(uint64_t o, const BucketArgs& ba, uint32_t& s) {
  s = ((uint32_t)(o >> kWheelLogKP)) / 30u;  // o < 2^34
  const uint32_t u = (uint32_t)(o - (uint64_t)s * kWheelSpan);
  const uint32_t k = u / 30u, rho = u - 30u * k;
  const uint32_t pl = (uint32_t)(ba.plane_lut >> (3 * (rho >> 1))) & 7u;
  const uint32_t word = ((k >> 5) << 3) | pl;  // block k >> 5, plane pl
  return (word << 5) | (k & 31u);
}

// Grid-strided walk (workgroup b of its band) over this thread's bucketed
// primes [i_lo, i_hi): each prime is loaded one prime ahead, so the load's
// latency hides behind the previous prime's walk (loaded on demand, a
// thread's ~200 primes were a chain of dependent global loads: ~0.7 ms per
// walk at the 1e18 window).
template <typename Walk>
__device__ __forceinline__ void for_bucket_primes(const uint32_t* __restrict__ P, uint32_t i_lo, uint32_t i_hi,
                                                  uint32_t b, uint32_t stride, Walk walk) {
  uint32_t i = i_lo + b * kBucketThreads + threadIdx.x;
  if (i >= i_hi) return;
  uint32_t pn = P[i];
  for (;;) {
    const uint32_t p = pn;
    i += stride;
    const bool more = i < i_hi;
    if (more) pn = P[i];
    walk(p);
    if (!more) break;
  }
}

// Walk the coprime-to-30 multiples of p inside [V0 + 1, V0 + span), from p^2 on.
template <typename Emit>
__device__ __forceinline__ void bucket_walk(uint32_t p, const BucketArgs& ba, Emit emit) {
  uint32_t w3;
  uint64_t o = bucket_first(p, ba, w3);
  while (o < ba.span) {
    uint32_t s;
    const uint32_t e = bucket_entry(o, ba, s);
    emit(s, e);
    o += (uint64_t)p * ((kGap30 >> w3) & 7u);
    w3 = w3 == 21 ? 0u : w3 + 3;
  }
}

__global__ __launch_bounds__(kBucketThreads) void bucket_count_kernel(const void* __restrict__ table, BucketArgs ba,
                                                                    const uint32_t* __restrict__ range,
                                                                    uint32_t* __restrict__ cols) {
  extern __shared__ uint32_t cnt[];  // [nseg]
  const uint32_t* P = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + 16);
  for (uint32_t j = threadIdx.x; j < ba.nseg; j += kBucketThreads) cnt[j] = 0;
  __syncthreads();
  // band-1 workgroup x: column x
  for_bucket_primes(P, range[2], range[1], blockIdx.x, kBucketGrid1 * kBucketThreads, [&](uint32_t p) {
    bucket_walk(p, ba, [&](uint32_t sg, uint32_t) { atomicAdd(&cnt[sg], 1u); });
  });
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < ba.nseg; j += kBucketThreads) cols[(uint64_t)j * kBucketCols + blockIdx.x] = cnt[j];
}

// per segment (one wave each): exclusive scan of its row over the virtual
// workgroups, in place; total -> tot[s]
__global__ __launch_bounds__(256) void bucket_colscan_kernel(uint32_t* __restrict__ cols, uint32_t nseg,
                                                             uint32_t* __restrict__ tot) {
  constexpr uint32_t kPer = kBucketCols / 64;
  const uint32_t sg = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (sg >= nseg) return;
  uint32_t* c = cols + (uint64_t)sg * kBucketCols + lane * kPer;
  uint32_t v[kPer], sum = 0;
#pragma unroll
  for (uint32_t t = 0; t < kPer; ++t) sum += (v[t] = c[t]);
  uint32_t x = sum;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) tot[sg] = x;
  x -= sum;
#pragma unroll
  for (uint32_t t = 0; t < kPer; ++t) {
    c[t] = x;
    x += v[t];
  }
}

// exclusive scan of the segment totals -> start[0..nseg]. A total above the
// entry capacity (a rigorous bound, so never expected) sets *flag: the fill,
// stage and sort kernels of the pass then skip (the fill only zeroing its
// band-0 region fills), every segment's list is left empty (start[] all 0,
// n0[] all 0) and the pass's count gets bit 63 set, so neither an
// out-of-bounds store nor a silently wrong count can result; the host entry
// points report it as DSE_EINTERNAL (dse_device_status).
__global__ __launch_bounds__(1024) void bucket_startscan_kernel(const uint32_t* __restrict__ tot, uint32_t nseg,
                                                                uint32_t* __restrict__ start, uint64_t cap,
                                                                uint32_t* __restrict__ flag,
                                                                unsigned long long* __restrict__ count) {
  __shared__ uint32_t s_scan[1024];
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (nseg + 1023) / 1024;
  const uint32_t b0 = tid * per, b1 = min(nseg, b0 + per);
  uint32_t sum = 0;
  for (uint32_t b = b0; b < b1; ++b) sum += tot[b];
  s_scan[tid] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    const uint32_t x = tid >= o ? s_scan[tid - o] : 0;
    __syncthreads();
    s_scan[tid] += x;
    __syncthreads();
  }
  const bool over = s_scan[1023] > cap;  // s_scan[1023]: every thread sees the same total
  uint32_t run = s_scan[tid] - sum;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t t = tot[b];
    start[b] = over ? 0u : run;
    run += t;
  }
  if (tid == 1023) {
    start[nseg] = over ? 0u : s_scan[1023];
    if (over) {
      flag[1] = 1u;  // this pass (read by the kernels below)
      flag[0] = 1u;  // sticky, cleared by dse_device_status
      atomicOr(count, 1ull << 63);
    } else {
      flag[1] = 0u;
    }
  }
}

#ifndef DSE_BK_CHUNK
#define DSE_BK_CHUNK 16  // band-0 fill walks chunks of this many segments (first group of kFillRG rounds) ...
#endif
#ifndef DSE_BK_CHUNK_GROW
#define DSE_BK_CHUNK_GROW 1  // ... doubled for each later group, up to 8x (profiles/r06/window_fill_chunks.txt)
#endif
#ifndef DSE_BK_FILL_RG
#define DSE_BK_FILL_RG 16
#endif
constexpr uint32_t kFillRG = DSE_BK_FILL_RG;  // stride rounds of primes walked together

// Band 0, one-level fill: every hit is one dword store at its slot. Workgroup
// b owns region (s, b) of every segment s: k0 slots at reg0 + (b nseg + s) k0
// (a workgroup's regions are contiguous, so a slot is a 32-bit offset from
// one scalar base), slot = an LDS cursor per segment. No count pass: k0
// bounds the region's expected fill by many standard deviations (bucket_k0),
// and a hit past it goes to the spill list (a global atomic; the list's
// capacity is a rigorous bound on the band's hits), so nothing is dropped
// whatever k0 is. At the end the region fills go to n0[s kBucketGrid + b]
// (capped at k0).
//
// The walk is issue-bound (profiles/r06/window_fill_knockouts.txt: without
// its atomics and stores it still takes 2/3 of the fill's time), so a hit
// costs as few VALU as the walk allows: a prime's state is its period index
// k = o / 30 from V0 (32 bits: a pass spans < 2^30 periods) and its wheel
// step w, kept as w4 = 4 w; everything that depends on the step comes from
// 4-bit fields at bit 4 w (v_bfe reads only the low 5 bits of the offset, so
// w4 just counts up): the gap, the carry of the residue, and the plane. With
// p = 30 pq + pm and residue rho_w of step w, the next hit is
// k + pq gap_w + (rho_w + pm gap_w) / 30; bucket_fill_start builds the carry
// and plane fields once per prime (eight residues from the first hit's).
constexpr uint64_t kFillMaxSplit = 30ull << 24;  // band-0 primes p < 30 * 2^24: p / 30 < 2^24 (v_mul_u32_u24)
static_assert((1ull << kBucketSplitLog) <= kFillMaxSplit, "production split");
constexpr uint32_t kGap30x4 = 6u | (4u << 4) | (2u << 8) | (4u << 12) | (2u << 16) | (4u << 20) | (6u << 24) | (2u << 28);

struct FillWalk {
  uint32_t k;       // period index of the next hit from V0 (~0u: none left in the pass)
  uint32_t w4;      // 4 * wheel step (mod 32 as used)
  uint32_t pq;      // p / 30
  uint32_t carry;   // 4-bit fields: (rho_w + pm gap_w) / 30
  uint32_t plane;   // 4-bit fields: plane of rho_w
};

__device__ __forceinline__ FillWalk bucket_fill_start(uint32_t p, const BucketArgs& ba) {
  uint32_t w3;
  const uint64_t o = bucket_first(p, ba, w3);
  FillWalk f{~0u, 0u, p / 30u, 0u, 0u};
  if (o >= ba.span) return f;
  const uint32_t kq = (uint32_t)(o / 30u);  // o < span + 6 p < 2^36: kq < 2^31
  uint32_t rho = (uint32_t)(o - 30ull * kq);
  const uint32_t w0 = w3 / 3u, pm = p - 30u * f.pq;
  f.k = kq;
  f.w4 = 4u * w0;
  for (uint32_t j = 0; j < 8; ++j) {
    const uint32_t w = (w0 + j) & 7u, gap = (kGap30x4 >> (4u * w)) & 15u;
    const uint32_t t = rho + pm * gap;  // < 30 + 29 * 6
    const uint32_t c = t / 30u;
    f.carry |= c << (4u * w);
    f.plane |= ((uint32_t)(ba.plane_lut >> (3u * (rho >> 1))) & 7u) << (4u * w);
    rho = t - 30u * c;
  }
  return f;
}

// (band-0 workgroup b; cur: nseg words of LDS)
__device__ __forceinline__ void bucket_fill_wg(uint32_t* cur, uint32_t b, const void* __restrict__ table,
                                               const BucketArgs& ba, const uint32_t* __restrict__ range,
                                               const BandZero& bz) {
  const uint32_t* P = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + 16);
  const uint32_t i_lo = range[0], i_hi = range[2];
  for (uint32_t j = threadIdx.x; j < ba.nseg; j += kBucketThreads) cur[j] = 0;
  __syncthreads();
  char* const reg_b = reinterpret_cast<char*>(bz.reg0 + (uint64_t)b * ba.nseg * bz.k0);  // this workgroup's regions
  const uint32_t k0 = bz.k0;
  // slot pos of region (sg, b), or the spill list past its capacity
  auto put = [&](uint32_t sg, uint32_t pos, uint32_t e) {
    if (pos < k0) {
      *reinterpret_cast<uint32_t*>(reg_b + 4u * (__umul24(sg, k0) + pos)) = e;  // < 2^32: per-workgroup regions
    } else {
      const uint32_t j = atomicAdd(bz.nspill, 1u);
      if (j < bz.spill_cap) {
        bz.spill[j] = (unsigned long long)sg << 32 | e;
      } else {  // only with a test-shrunk capacity (bucket_cap_divisor): fail loudly
        bz.flag[0] = 1u;
        atomicOr(bz.count, 1ull << 63);
      }
    }
  };
  auto emit = [&](uint32_t sg, uint32_t e) {
#if defined(DSE_BK_FILL_KO) && DSE_BK_FILL_KO == 3  // profiling knockout: the walk alone
    asm volatile("" ::"v"(e), "v"(sg));
    return;
#endif
    const uint32_t pos = atomicAdd(&cur[sg], 1u);
#if defined(DSE_BK_FILL_KO) && DSE_BK_FILL_KO == 1  // profiling knockout: no global store
    asm volatile("" ::"v"(e), "v"(pos));
    return;
#elif defined(DSE_BK_FILL_KO) && DSE_BK_FILL_KO == 2  // profiling knockout: one coalesced line per store
    bz.reg0[(uint64_t)b * kBucketThreads + threadIdx.x] = e + pos;
    return;
#endif
    put(sg, pos, e);
  };
  // Segment-ordered walk: a thread walks its primes of kFillRG stride rounds
  // together, chunk by chunk of DSE_BK_CHUNK segments, so region (s, b) gets
  // its hits within one chunk's time (while its lines are still in the L2)
  // instead of over the whole walk. Snake order: odd rounds of the stride
  // take their block in reverse thread order, so the thread with one round's
  // smallest prime (the most hits, ~1/p) gets the next round's largest (in
  // plain order the threads holding a band's smallest primes walk up to
  // ~1.7x the mean).
  constexpr uint32_t stride = kBucketGrid * kBucketThreads;
  constexpr uint32_t kKPMask = (1u << kWheelLogKP) - 1;
  const uint32_t j = b * kBucketThreads + threadIdx.x;
  const uint32_t jr = stride - 1 - j;
  const uint32_t kspan = ba.nseg << kWheelLogKP;  // periods of the pass (< 2^30)
  for (uint64_t r0 = 0; i_lo + r0 * stride < i_hi; r0 += kFillRG) {
    FillWalk f[kFillRG];
#pragma unroll
    for (uint32_t r = 0; r < kFillRG; ++r) {
      const uint64_t i = i_lo + (r0 + r) * stride + (((r0 + r) & 1) ? jr : j);
      f[r] = FillWalk{~0u, 0u, 0u, 0u, 0u};
      if (i < i_hi) f[r] = bucket_fill_start(P[i], ba);
    }
    // later groups walk larger primes (fewer hits per chunk: lanes idle in
    // the divergent walk) at larger chunks
    const uint32_t cseg = DSE_BK_CHUNK << min(3u, (uint32_t)(r0 / kFillRG) * DSE_BK_CHUNK_GROW);
    for (uint32_t end = cseg;; end += cseg) {
      const uint32_t klim = min(end << kWheelLogKP, kspan);
      bool left = false;
#pragma unroll
      for (uint32_t r = 0; r < kFillRG; ++r) {
        while (f[r].k < klim) {
          const uint32_t k = f[r].k, w4 = f[r].w4;
          const uint32_t pl = __builtin_amdgcn_ubfe(f[r].plane, w4, 4);
          const uint32_t gap = __builtin_amdgcn_ubfe(kGap30x4, w4, 4);
          const uint32_t c = __builtin_amdgcn_ubfe(f[r].carry, w4, 4);
          // entry (bucket_entry): LDS word (block << 3 | plane) << 5 | bit
          emit(k >> kWheelLogKP, ((k & kKPMask & ~31u) << 3) | (pl << 5) | (k & 31u));
          f[r].k = k + __umul24(f[r].pq, gap) + c;  // pq < 2^24
          f[r].w4 = w4 + 4u;
        }
        left |= f[r].k < kspan;
      }
      if (!left) break;
    }
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < ba.nseg; j += kBucketThreads) bz.n0[(uint64_t)j * kBucketGrid + b] = min(cur[j], bz.k0);
}

// Band 1, two-level fill: every global store is a run of consecutive dwords.
//
// Level 1 (bucket_stage_kernel) files each hit under its super-bucket of
// kSupSegs consecutive segments, key = (segment mod kSupSegs) << 20 | entry.
// Each wave stages kStageCap keys per super-bucket in LDS (a slot per lane
// from an LDS atomic) and writes a full stage as one 256 B run into its
// workgroup's region of that super-bucket; the region of (band-1 workgroup g,
// super-bucket S) starts at
//   start[S kSupSegs] + sum over S's segments s of cols[s][g]
// (cols = per-segment exclusive scans over the virtual workgroups), so the
// temporary array holds each super-bucket where its band-1 entries will end
// up. A lane whose stage is full keeps its hit and retries after the flush.
// Lanes move on to their next prime independently, its (p, m) loaded one
// prime ahead (a wave-synchronous walk that waited on that load at every
// prime change was latency-bound).
//
// Level 2 (bucket_sort_kernel): job (S, group of kSortGroup band-1
// workgroups) reads its contiguous slice of super-bucket S, whose per-segment
// counts are known (cols again), and counting-sorts tiles of kSortTile keys by
// segment in LDS, the next tile's keys loaded while the current one sorts;
// each segment's run of a tile is stored contiguously at its cursor, which
// starts at start[s] + cols[s][first workgroup of the group].
constexpr uint32_t kSupLog = 7;
constexpr uint32_t kSupSegs = 1u << kSupLog;       // segments per super-bucket
constexpr uint32_t kStageCap = 64;                 // keys per (wave, super-bucket) stage: one 256 B run
constexpr uint32_t kKeyShift = 20;                 // entry = LDS word index << 5 | bit < 2^20
static_assert(IMG_WORDS * 32 <= (1u << kKeyShift) && kKeyShift + kSupLog <= 32, "bucket key layout");
#ifndef DSE_BK_SORT_GROUP
#define DSE_BK_SORT_GROUP 64
#endif
constexpr uint32_t kSortGroup = DSE_BK_SORT_GROUP;  // band-1 workgroups per level-2 job
#ifndef DSE_BK_SORT_TILE
#define DSE_BK_SORT_TILE 8192
#endif
constexpr uint32_t kSortTile = DSE_BK_SORT_TILE;   // keys per LDS counting sort
#ifndef DSE_BK_SORT_THREADS
#define DSE_BK_SORT_THREADS 1024
#endif
constexpr uint32_t kSortThreads = DSE_BK_SORT_THREADS;
static_assert(kSortTile % kSortThreads == 0 && kSortThreads >= kSupSegs, "sort tile");
static_assert(kBucketGrid1 % kSortGroup == 0, "sort groups");

__host__ __device__ constexpr uint32_t stage_lds_words(uint32_t nsup) {
  return nsup + (kBucketThreads / 64) * nsup * (kStageCap + 1);
}

// (band-1 workgroup b; sm: stage_lds_words(nsup) words of LDS)
__device__ __forceinline__ void bucket_stage_wg(uint32_t* sm, uint32_t b, const void* __restrict__ table,
                                                const BucketArgs& ba, const uint32_t* __restrict__ range,
                                                const uint32_t* __restrict__ cols, const uint32_t* __restrict__ start,
                                                uint32_t* __restrict__ tmp, uint32_t nsup) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t i_hi = range[1];
  constexpr uint32_t stride = kBucketGrid1 * kBucketThreads;
  uint32_t i = range[2] + b * kBucketThreads + tid;  // index of the prefetched prime
  if (__syncthreads_or(i < i_hi) == 0) return;
  uint32_t* cur = sm;                                          // [nsup] region cursors of this workgroup
  uint32_t* scnt = sm + nsup + wave * nsup * (kStageCap + 1);  // [nsup] this wave's stage fills
  uint32_t* stage = scnt + nsup;                               // [nsup][kStageCap]
  for (uint32_t S = tid; S < nsup; S += kBucketThreads) cur[S] = start[S << kSupLog];
  for (uint32_t S = lane; S < nsup; S += 64) scnt[S] = 0;
  __syncthreads();
  for (uint32_t s = tid; s < ba.nseg; s += kBucketThreads)
    atomicAdd(&cur[s >> kSupLog], cols[(uint64_t)s * kBucketCols + b]);
  __syncthreads();

  const uint32_t* P = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(table) + 16);
  uint32_t pn = i < i_hi ? P[i] : 0u;
  uint32_t p = 0, w3 = 0;
  uint64_t o = ba.span;
  // next prime of this lane with a hit in the pass (o >= span: none left)
  auto next_prime = [&]() {
    while (i < i_hi) {
      p = pn;
      i += stride;
      if (i < i_hi) pn = P[i];
      o = bucket_first(p, ba, w3);
      if (o < ba.span) return;
    }
    o = ba.span;
  };
  next_prime();
  while (__ballot(o < ba.span)) {
    uint32_t S = 0, pos = kStageCap;
    if (o < ba.span) {
      uint32_t s;
      const uint32_t e = bucket_entry(o, ba, s);
      S = s >> kSupLog;
      pos = atomicAdd(&scnt[S], 1u);
      if (pos < kStageCap) stage[S * kStageCap + pos] = ((s & (kSupSegs - 1)) << kKeyShift) | e;
    }
    // stages that just filled: exactly one lane took their last slot and reserves the run
    const bool filled = pos == kStageCap - 1;
    uint32_t g = 0;
    if (filled) g = atomicAdd(&cur[S], kStageCap);
    uint64_t full = __ballot(filled);
    __builtin_amdgcn_wave_barrier();
    while (full) {
      const uint32_t l = (uint32_t)__builtin_ctzll(full);
      full &= full - 1;
      const uint32_t Sf = (uint32_t)__builtin_amdgcn_readlane((int)S, (int)l);
      const uint32_t gf = (uint32_t)__builtin_amdgcn_readlane((int)g, (int)l);
      tmp[gf + lane] = stage[Sf * kStageCap + lane];
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) scnt[Sf] = 0;  // lanes that overshot the full stage retry next step
      __builtin_amdgcn_wave_barrier();
    }
    if (pos < kStageCap) {  // placed: advance to the next hit (or prime)
      o += (uint64_t)p * ((kGap30 >> w3) & 7u);
      w3 = w3 == 21 ? 0u : w3 + 3;
      if (o >= ba.span) next_prime();
    }
  }
  // partial stages
  for (uint32_t S = 0; S < nsup; ++S) {
    const uint32_t n = scnt[S];
    if (n == 0) continue;
    uint32_t g = 0;
    if (lane == 0) g = atomicAdd(&cur[S], n);
    g = (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
    if (lane < n) tmp[g + lane] = stage[S * kStageCap + lane];
  }
}

// Band-0 fill and band-1 stage in one launch: workgroups [0, nfill) fill,
// the rest stage, so the request-bound scattered stores of the one and the
// latency-bound staging of the other share the CUs (and neither pays a tail).
__global__ __launch_bounds__(kBucketThreads) void bucket_fill_stage_kernel(
    const void* __restrict__ table, BucketArgs ba, const uint32_t* __restrict__ range,
    const uint32_t* __restrict__ cols, const uint32_t* __restrict__ start, BandZero bz,
    uint32_t* __restrict__ tmp, uint32_t nsup, uint32_t nfill, const uint32_t* __restrict__ flag) {
  extern __shared__ uint32_t sm[];
  const uint32_t x = blockIdx.x;
  if (flag[1]) {  // capacity overflow (bucket_startscan_kernel): no hits, but every band-0 region empty
    if (x < nfill)
      for (uint32_t j = threadIdx.x; j < ba.nseg; j += kBucketThreads) bz.n0[(uint64_t)j * kBucketGrid + x] = 0;
    return;
  }
#if defined(DSE_BK_FILL_KO) && DSE_BK_FILL_KO == 4  // profiling knockout: band-0 fill only
  if (x >= nfill) return;
#elif defined(DSE_BK_FILL_KO) && DSE_BK_FILL_KO == 5  // profiling knockout: band-1 staging only
  if (x < nfill) return;
#endif
  if (x < nfill)
    bucket_fill_wg(sm, x, table, ba, range, bz);
  else
    bucket_stage_wg(sm, x - nfill, table, ba, range, cols, start, tmp, nsup);
}

__global__ __launch_bounds__(kSortThreads) void bucket_sort_kernel(BucketArgs ba, const uint32_t* __restrict__ cols,
                                                                   const uint32_t* __restrict__ start,
                                                                   const uint32_t* __restrict__ tmp,
                                                                   uint32_t* __restrict__ entries,
                                                                   const uint32_t* __restrict__ flag) {
  if (flag[1]) return;  // capacity overflow (bucket_startscan_kernel)
#if defined(DSE_BK_FILL_KO) && DSE_BK_FILL_KO == 4  // profiling knockout: nothing staged to sort
  return;
#endif
  constexpr uint32_t kPer = kSortTile / kSortThreads;
  constexpr uint32_t kPerLane = kSupSegs / 64;  // scan: segment counts per lane of wave 0
  __shared__ uint32_t sorted[kSortTile];
  __shared__ uint32_t hist[kSupSegs], off[kSupSegs], curs[kSupSegs];
  __shared__ uint32_t rb[2];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  constexpr uint32_t ngroups = kBucketGrid1 / kSortGroup;
  const uint32_t S = blockIdx.x / ngroups, g0 = (blockIdx.x % ngroups) * kSortGroup,
                 g1 = g0 + kSortGroup;
  const uint32_t s0 = S << kSupLog;
  if (tid < 2) rb[tid] = 0;
  if (tid < kSupSegs) hist[tid] = 0;
  __syncthreads();
  if (tid < kSupSegs) {
    const uint32_t s = s0 + tid;
    uint32_t c0 = 0, c1 = 0;
    if (s < ba.nseg) {
      c0 = cols[(uint64_t)s * kBucketCols + g0];
      c1 = g1 < kBucketCols ? cols[(uint64_t)s * kBucketCols + g1] : start[s + 1] - start[s];
      curs[tid] = start[s] + c0;
    }
    atomicAdd(&rb[0], c0);
    atomicAdd(&rb[1], c1);
  }
  __syncthreads();
  const uint32_t r0 = start[s0] + rb[0], r1 = start[s0] + rb[1];
  uint32_t nxt[kPer];
  auto load_tile = [&](uint32_t base) {
    const uint32_t n = min(kSortTile, r1 - base);
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
      const uint32_t j = q * kSortThreads + tid;
      nxt[q] = j < n ? __builtin_nontemporal_load(tmp + base + j) : 0u;
    }
  };
  if (r0 < r1) load_tile(r0);
  for (uint32_t base = r0; base < r1; base += kSortTile) {
    const uint32_t n = min(kSortTile, r1 - base);
    uint32_t key[kPer], rk[kPer];
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) key[q] = nxt[q];
    if (base + kSortTile < r1) load_tile(base + kSortTile);
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q)
      rk[q] = q * kSortThreads + tid < n ? atomicAdd(&hist[key[q] >> kKeyShift], 1u) : 0u;
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the segment counts (one wave, kPerLane each)
      uint32_t c[kPerLane], sum = 0;
#pragma unroll
      for (uint32_t t = 0; t < kPerLane; ++t) sum += (c[t] = hist[lane * kPerLane + t]);
      uint32_t x = sum;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
      }
      x -= sum;
#pragma unroll
      for (uint32_t t = 0; t < kPerLane; ++t) {
        off[lane * kPerLane + t] = x;
        x += c[t];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q)
      if (q * kSortThreads + tid < n) sorted[off[key[q] >> kKeyShift] + rk[q]] = key[q];
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kPer; ++q) {
      const uint32_t j = q * kSortThreads + tid;
      if (j < n) {
        const uint32_t v = sorted[j], k = v >> kKeyShift;
        entries[curs[k] + j - off[k]] = v & ((1u << kKeyShift) - 1);
      }
    }
    __syncthreads();
    if (tid < kSupSegs) {
      curs[tid] += hist[tid];
      hist[tid] = 0;
    }
    __syncthreads();
  }
}

#endif  // DSE_WHEEL_MAIN_TU
}  // namespace


#if DSE_WHEEL_MAIN_TU
hipError_t launch_wheel_offsets(void* table, int num_cus, hipStream_t stream, uint64_t n_hint) {
  // rows, factors and plans only for the primes <= kWheelMaxPrime (82,025 below 2^20): the kernel stops
  // at the first bucketed prime, so a window's 50.8 M-prime table needs no larger grid (the grid-stride
  // loop covers every index whatever the grid)
  n_hint = std::min<uint64_t>(n_hint, 1u << 17);
  const uint64_t grid = std::max<uint64_t>(4 * (uint64_t)num_cus, std::min<uint64_t>(n_hint / 1024 + 1, 1u << 16));
  hipLaunchKernelGGL(wheel_offsets_kernel, dim3((uint32_t)grid), dim3(256), 0, stream, table);
  return hipGetLastError();
}


hipError_t free_scratch(Scratch* s) {
  if (!s) return hipSuccess;
  hipError_t e = s->used ? hipEventSynchronize(s->done) : hipSuccess;  // the last pass may still read it
  const hipError_t f = s->ptr ? hipFree(s->ptr) : hipSuccess;
  const hipError_t g = s->done ? hipEventDestroy(s->done) : hipSuccess;
  if (s->flag) (void)hipFree(s->flag);
  s->flag = nullptr;
  s->ptr = nullptr;
  s->bytes = 0;
  s->done = nullptr;
  s->used = false;
  return e != hipSuccess ? e : f != hipSuccess ? f : g;
}
#endif  // DSE_WHEEL_MAIN_TU

namespace {


// One range's geometry (shared by the wheel kernel and the bucket walks):
// the planes of V0 mod 30, the small-prime fixes, the init offsets.
// *plane_lut: plane of relative residue rho in bits [3 (rho >> 1), +3).
[[maybe_unused]] WheelRange make_wheel_range(const RangeSpec& rs, uint64_t* plane_lut) {
  WheelRange w{};
  const uint64_t v_start = 3 + 2 * rs.g_start;
  w.V0 = v_start - 1;
  w.nbits = rs.nbits;
  w.KB0 = w.V0 / 30;
  w.out = rs.out;
  w.count = rs.count;
  const uint32_t v0m = (uint32_t)(w.V0 % 30);
  uint32_t n = 0;
  *plane_lut = 0;
  for (uint32_t rho = 1; rho < 30; rho += 2) {
    const uint32_t r = (v0m + rho) % 30;
    if (r % 3 == 0 || r % 5 == 0) continue;
    uint32_t iota = 0;
    while (kR30[iota] != r) ++iota;
    w.rho_pack |= (uint64_t)rho << (5 * n);
    w.pl_pack |= n << (3 * iota);
    if (v0m + rho >= 30) w.e_iota |= 1u << iota;
    *plane_lut |= (uint64_t)n << (3 * (rho >> 1));
    ++n;
  }
  // primes 3..79 inside the range: the wheel drops 3 and 5, the patterns mark 7..79 themselves
  constexpr uint32_t small[] = {3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61, 67, 71, 73, 79};
  static_assert(small[sizeof(small) / sizeof(small[0]) - 1] == kQMax && (kQMax - 3) / 2 < 64, "fix covers 3..kQMax");
  for (uint32_t v : small)
    if (v >= v_start && (v - v_start) / 2 < rs.nbits) w.fix |= 1ull << ((v - v_start) / 2);
  for (int g = 0; g < kNG; ++g) w.v0g[g] = (uint16_t)(w.V0 % gmod(g));
  return w;
}

[[maybe_unused]] uint64_t isqrt64(uint64_t x) {
  uint64_t r = (uint64_t)__builtin_sqrt((double)x);
  while (r * r > x) --r;
  while ((r + 1) * (r + 1) <= x) ++r;
  return r;
}

// A launch over the ranges rs[0..n) (1 <= n <= kMaxRanges, each < 2^31
// segments in all), their segments in order; thresholds: odd primes up to
// kQMax, TA, TB1, TB and wheel_max (<= kWheelMaxPrime: the primes above it are
// bucketed or absent).
[[maybe_unused]] WheelArgs make_wheel_args(const RangeSpec* rs, uint32_t n, uint64_t* plane_lut,
                                           uint64_t wheel_max = kWheelMaxPrime) {
  static const std::vector<uint32_t> odd_primes = [] {  // odd primes <= kWheelMaxPrime (sieved once)
    std::vector<uint8_t> comp(kWheelMaxPrime / 2 + 1, 0);  // comp[i]: 2i + 1 composite
    for (uint64_t i = 1; (2 * i + 1) * (2 * i + 1) <= kWheelMaxPrime; ++i)
      if (!comp[i])
        for (uint64_t j = ((2 * i + 1) * (2 * i + 1)) / 2; j <= kWheelMaxPrime / 2; j += 2 * i + 1) comp[j] = 1;
    std::vector<uint32_t> v;
    for (uint64_t i = 1; 2 * i + 1 <= kWheelMaxPrime; ++i)
      if (!comp[i]) v.push_back((uint32_t)(2 * i + 1));
    return v;
  }();
  const uint64_t lim[5] = {kQMax, TA, TB1, TB, std::min<uint64_t>(wheel_max, kWheelMaxPrime)};
  WheelArgs wa{};
  for (int t = 0; t < 5; ++t)
    wa.nthr[t] = (uint32_t)(std::upper_bound(odd_primes.begin(), odd_primes.end(), lim[t]) - odd_primes.begin());
  uint64_t seg = 0, lut = 0;
  for (uint32_t i = 0; i < n; ++i) {
    WheelRange& r = wa.r[i];
    r = make_wheel_range(rs[i], i ? &lut : plane_lut);
    r.seg0 = (uint32_t)seg;
    const uint64_t nseg_r = (rs[i].nbits + kWheelOutBits - 1) / kWheelOutBits;
    seg += nseg_r;
    // piece j = segments [j << lsh, (j + 1) << lsh): the odd primes with p^2
    // below the end of its last segment (the kernel's live test is p^2 < Vend)
    r.lsh = 0;
    while (nseg_r > 0 && ((nseg_r - 1) >> r.lsh) >= kLPieces) ++r.lsh;
    for (uint32_t j = 0; j < kLPieces; ++j) {
      const uint64_t last = nseg_r == 0 ? 0 : std::min<uint64_t>(((uint64_t)(j + 1) << r.lsh) - 1, nseg_r - 1);
      const uint64_t vend = r.V0 + (last + 1) * (uint64_t)kWheelSpan;
      r.lcap[j] = (uint32_t)(std::upper_bound(odd_primes.begin(), odd_primes.end(), isqrt64(vend - 1)) -
                             odd_primes.begin());
      if (r.lcap[j] == odd_primes.size()) r.lcap[j] = ~0u;  // past kWheelMaxPrime: no bound
    }
  }
  wa.nranges = n;
  wa.nseg = (uint32_t)seg;
  // (Non-temporal mask stores paid 5% at 1e12 only while segments claimed the
  // dead large units past their live primes; with lcap they do not:
  // profiles/r05/ab_nt_store_policy.txt, ab_nmin_and_nt_recheck.txt)
  return wa;
}


#if DSE_WHEEL_MAIN_TU
// Rigorous bound on the bucket entries of a pass spanning `span` integers with
// primes in (a, b]: each prime has <= 8 span / (30 p) + 8 coprime multiples;
// sum 1/p <= ln(ln b / ln a) + 1/ln^2 a and pi(b) <= 1.25506 b / ln b.
uint64_t bucket_cap(uint64_t span, double a, double b) {
  if (b <= a) return 64;
  const double la = __builtin_log(a), lb = __builtin_log(b);
  const double s = __builtin_log(lb / la) + 1.0 / (la * la);
  return (uint64_t)(8.0 * (double)span / 30.0 * s + 8.0 * 1.25506 * b / lb) + 1024;
}

// Band-0 region capacity k0 (bucket_fill_wg). A region collects the hits in one
// segment of one fill workgroup's primes: 256 per stride round r, all >= the
// round's first prime p(r), so its mean is at most lambda = (8 W / 30) sum_r
// 256 / p(r) (p(r) from the table index i_lo + r S: p_n >= n (ln n + ln ln n
// - 1), Dusart), and its variance at most lambda plus ~4 per prime below the
// segment span W: such a prime (2^19 < p < W, all in round 0) hits each of
// the 8 planes floor or ceil of KP / p times, a deviation of variance <= 1/4
// per plane, 2 per prime (4 taken). k0 = lambda + 10 sigma + 64:
// a region past it is a >10-sigma event, and even then its hits are spilled,
// not lost.
uint32_t bucket_k0(uint32_t i_lo, double a, double b) {
  if (b <= a) return 0;
  const double S = (double)kBucketGrid * kBucketThreads;
  const double n_band = 1.25506 * b / __builtin_log(b) - (double)i_lo;  // >= the band's primes
  const double mu = 8.0 * (double)kWheelSpan / 30.0;
  double lam = 0;
  for (double r = 0; r * S < n_band; r += 1) {
    const double n = (double)i_lo + r * S + 2;  // 1-based index of the round's first prime (2 is p_1)
    const double pl = std::max(a, n * (__builtin_log(n) + __builtin_log(__builtin_log(n)) - 1.0));
    lam += mu * kBucketThreads / pl;
  }
  const double var = lam + 4.0 * kBucketThreads;
  const uint64_t k0 = (uint64_t)(lam + 10.0 * __builtin_sqrt(var) + 64.0);
  return (uint32_t)((k0 + 15) & ~15ull);
}

constexpr uint64_t kBucketMaxEntries = 1ull << 31;  // 8 GB of band-1 entries per pass
constexpr uint64_t kBucketMaxRegionBytes = 24ull << 30;  // band-0 regions per pass

// Grow the context's scratch to `bytes` for a pass on `stream`, ordered after
// the previous pass whatever stream that ran on: a grow waits for it on the
// host (the old buffer is freed), otherwise `stream` waits for its event.
hipError_t ensure_scratch(Scratch* sc, uint64_t bytes, hipStream_t stream, char** out) {
  hipError_t e;
  if (!sc->done && (e = hipEventCreateWithFlags(&sc->done, hipEventDisableTiming)) != hipSuccess) return e;
  if (!sc->flag) {
    if ((e = hipMalloc(&sc->flag, 2 * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = hipMemsetAsync(sc->flag, 0, 2 * sizeof(uint32_t), stream)) != hipSuccess) return e;
  }
  if (sc->bytes < bytes) {
    if (sc->used && (e = hipEventSynchronize(sc->done)) != hipSuccess) return e;
    if (sc->ptr && (e = hipFree(sc->ptr)) != hipSuccess) return e;
    sc->ptr = nullptr;
    sc->bytes = 0;
    sc->used = false;
    if ((e = hipMalloc(&sc->ptr, bytes)) != hipSuccess) return e;
    sc->bytes = bytes;
  } else if (sc->used && (e = hipStreamWaitEvent(stream, sc->done, 0)) != hipSuccess) {
    return e;
  }
  *out = static_cast<char*>(sc->ptr);
  return hipSuccess;
}

// After the last kernel of a pass that reads the scratch.
hipError_t release_scratch(Scratch* sc, hipStream_t stream) {
  const hipError_t e = hipEventRecord(sc->done, stream);
  if (e == hipSuccess) sc->used = true;
  return e;
}

#endif  // DSE_WHEEL_MAIN_TU

hipError_t launch_wheel(const void* table, const WheelArgs& wa, int num_cus, hipStream_t stream) {
  if (wa.nseg == 0) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>(wa.nseg, (uint32_t)num_cus);
#if DSE_WHEEL_MAIN_TU
  // ranges without bucketed primes: the no-bucket instantiation, compiled in
  // dse_wheel_plain.hip with the default machine scheduler (its loop spills
  // fewer SGPRs there; the bucket instantiation is faster with iterative-ILP)
  if (!wa.bk_start) return launch_wheel_plain(table, &wa, num_cus, stream);
  hipLaunchKernelGGL(wheel_segments_kernel<true>, dim3(grid), dim3(NT), 0, stream, table, wa);
#else
  hipLaunchKernelGGL(wheel_segments_kernel<false>, dim3(grid), dim3(NT), 0, stream, table, wa);
#endif
  return hipGetLastError();
}

// Launches over rs[0..n), kMaxRanges ranges at a time.
[[maybe_unused]] hipError_t launch_wheel_batches(const void* table, const RangeSpec* rs, size_t n, int num_cus,
                                                 hipStream_t stream) {
  for (size_t i = 0; i < n; i += kMaxRanges) {
    uint64_t plane_lut;
    const hipError_t e = launch_wheel(
        table, make_wheel_args(rs + i, (uint32_t)std::min<size_t>(kMaxRanges, n - i), &plane_lut), num_cus, stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

#if DSE_WHEEL_PLAIN_TU
// The full-geometry wheel kernel for ranges without bucketed primes (N up to
// 1.1e12), on its own translation unit for its compile flags (Makefile).
// wa: the caller's WheelArgs (the same definition, this source).
hipError_t launch_wheel_plain(const void* table, const void* wa, int num_cus, hipStream_t stream) {
  return launch_wheel(table, *static_cast<const WheelArgs*>(wa), num_cus, stream);
}
#elif DSE_WHEEL_HALF_TU
// The half-size geometry (this translation unit: 2^16 periods per segment):
// the tail of a launch whose last round of full segments would leave most
// CUs idle (launch_sieve_ranges). Primes <= kWheelMaxPrime only.
hipError_t launch_wheel_ranges_half(const void* table, const RangeSpec* rs, size_t n, int num_cus,
                                    hipStream_t stream) {
  return launch_wheel_batches(table, rs, n, num_cus, stream);
}
#else
// Time of a half-size segment (dse_wheel_half.hip) relative to a full one,
// and of a launch relative to a round of full segments
// (profiles/r03/geometry_ab.txt).
constexpr double kHalfSegCost = DSE_HALF_SEG_COST, kLaunchCost = DSE_LAUNCH_COST;

namespace {

// The ranges without bucketed primes, pooled: one persistent launch (per
// kMaxRanges ranges) over all their segments. Segments go to the num_cus
// workgroups in rounds; a last, partial round of full segments leaves CUs
// idle for a whole segment time, so the segments past the last full round
// go to the half-size geometry instead when that finishes sooner: (their
// half segments / num_cus rounds) x kHalfSegCost plus the second launch.
hipError_t launch_pooled(const void* table, const RangeSpec* rs, size_t n, int num_cus, hipStream_t stream,
                         const SieveOpts* opts) {
  if (n == 0) return hipSuccess;
  const uint32_t geo = opts ? opts->wheel_geometry : 0;  // 0 auto, 1 full only, 2 half only
  constexpr uint64_t kHalfBits = kWheelOutBits / 2;
  const uint64_t G = (uint64_t)num_cus;
  uint64_t S = 0;
  for (size_t i = 0; i < n; ++i) S += (rs[i].nbits + kWheelOutBits - 1) / kWheelOutBits;
  uint64_t F = geo == 2 ? 0 : geo == 1 ? S : (S / G) * G;  // segments of the full geometry
  // split the list after its first F full segments
  std::vector<RangeSpec> full, half;
  uint64_t left = F;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t ns = (rs[i].nbits + kWheelOutBits - 1) / kWheelOutBits;
    const uint64_t take = std::min(ns, left);
    left -= take;
    const uint64_t fb = std::min(rs[i].nbits, take * kWheelOutBits);
    if (fb) full.push_back({rs[i].g_start, fb, rs[i].out, rs[i].count});
    if (fb < rs[i].nbits)
      half.push_back({rs[i].g_start + fb, rs[i].nbits - fb, rs[i].out ? rs[i].out + fb / 32 : nullptr,
                      rs[i].count});
  }
  if (geo == 0 && !half.empty()) {
    uint64_t nhalf = 0;
    for (const auto& h : half) nhalf += (h.nbits + kHalfBits - 1) / kHalfBits;
    if (kHalfSegCost * (double)((nhalf + G - 1) / G) + (F ? kLaunchCost : 0.0) >= 1.0) {
      half.clear();  // the whole list in the full geometry
      full.assign(rs, rs + n);
    }
  }
  hipError_t e = launch_wheel_batches(table, full.data(), full.size(), num_cus, stream);
  if (e != hipSuccess) return e;
  return half.empty() ? hipSuccess : launch_wheel_ranges_half(table, half.data(), half.size(), num_cus, stream);
}

// A range whose primes reach above kWheelMaxPrime: bucketed passes.
hipError_t launch_bucketed(const void* table, uint64_t g_start, uint64_t nbits, uint32_t* out,
                           unsigned long long* count, int num_cus, hipStream_t stream, Scratch* scratch,
                           const SieveOpts* opts) {
  const uint64_t vmax = 3 + 2 * (g_start + nbits - 1);
  const uint64_t root = isqrt64(vmax);
  uint64_t plane_lut;
  if (!scratch) return hipErrorInvalidValue;
  // primes above kWheelMaxPrime: passes of <= kBucketMaxSegs segments, each
  // with its own bucket build, then the wheel kernel over the pass
  const uint64_t total_seg = (nbits + kWheelOutBits - 1) / kWheelOutBits;
  uint64_t max_segs = kBucketMaxSegs;
  if (opts && opts->bucket_pass_segs >= 1 && opts->bucket_pass_segs < max_segs) max_segs = opts->bucket_pass_segs;
  // band 0 stops below 30 * 2^24 whatever the option (its walk's 24-bit step product, bucket_fill_wg)
  const uint64_t split =
      std::min<uint64_t>(1ull << (opts && opts->bucket_split_log2 ? opts->bucket_split_log2 : kBucketSplitLog), kFillMaxSplit);
  // primes above lo_p are bucketed: below kWheelMaxPrime for a range that is
  // bucketed anyway (a prime that hits a segment about once is cheaper as a
  // bucket entry than as 8 plane slots of an L unit; window: 2^19 -2%)
  const uint64_t lo_p = 1ull << (opts && opts->bucket_lo_log2 ? opts->bucket_lo_log2 : kBucketLoLog);
  const uint32_t cap_div = opts && opts->bucket_cap_div > 1 ? opts->bucket_cap_div : 1;  // test-only: overflow
  const uint32_t k0_div = opts && opts->bucket_k0_div > 1 ? opts->bucket_k0_div : 1;     // test-only: spills
  const double a0 = (double)lo_p, b0 = std::min((double)split, (double)root);  // band 0: (a0, b0]
  for (uint64_t s0 = 0; s0 < total_seg;) {
    uint64_t ns = std::min<uint64_t>(max_segs, total_seg - s0);
    RangeSpec piece{g_start + s0 * kWheelOutBits, kWheelOutBits, nullptr, count};
    WheelArgs wa = make_wheel_args(&piece, 1, &plane_lut, lo_p);  // (wa.nthr)
    const uint32_t k0_full = bucket_k0(wa.nthr[4], a0, b0);
    while (ns > 1 && (bucket_cap(ns * kWheelSpan, (double)split, (double)root) > kBucketMaxEntries ||
                      4ull * ns * kBucketGrid * k0_full > kBucketMaxRegionBytes))
      ns /= 2;
    const uint64_t g0 = g_start + s0 * kWheelOutBits;
    const uint64_t nb = std::min<uint64_t>(nbits - s0 * kWheelOutBits, ns * kWheelOutBits);
    const uint64_t vmax_p = 3 + 2 * (g0 + nb - 1);
    piece = {g0, nb, out ? out + s0 * (kWheelOutBits / 32) : nullptr, count};
    wa = make_wheel_args(&piece, 1, &plane_lut, lo_p);
    if (wa.nseg != ns) return hipErrorInvalidValue;  // the band-0 region layout's nseg (wheel side: wa.nseg)
    BucketArgs ba{};
    ba.V0 = wa.r[0].V0;
    ba.span = ns * kWheelSpan;
    ba.plane_lut = plane_lut;
    ba.nseg = (uint32_t)ns;
    ba.vmax = vmax_p;
    ba.split = split;
    const uint64_t root_p = isqrt64(vmax_p);
    const bool band0 = split > lo_p, band1 = split < root_p;
    // band 1: rigorous entry capacity (its keys, then its sorted entries);
    // band 0: regions of k0 slots per (segment, fill workgroup), the spill
    // list's capacity a rigorous bound on the band's hits
    const uint64_t cap = (band1 ? bucket_cap(ba.span, (double)split, (double)root_p) : 64) / cap_div;
    const uint32_t k0 = band0 ? std::max<uint32_t>(1, k0_full / k0_div / cap_div) : 0;
    const uint64_t spill_cap = band0 ? bucket_cap(ba.span, a0, std::min((double)split, (double)root_p)) / cap_div : 0;
    // scratch: [range 3, nspill][cols grid1*ns][tot ns][start ns+1][entries cap][band-1 keys cap]
    //          [band-0 regions ns*grid*k0][band-0 fills ns*grid][spill list (8 B) spill_cap]
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t o_cols = 256, o_tot = o_cols + 4ull * kBucketCols * ns, o_start = o_tot + 4 * ns + 256,
                   o_ent = al(o_start + 4 * (ns + 1)), o_tmp = al(o_ent + 4 * cap),
                   o_reg = al(band1 ? o_tmp + 4 * cap : o_tmp), o_n0 = al(o_reg + 4ull * ns * kBucketGrid * k0),
                   o_spill = al(o_n0 + (band0 ? 4ull * ns * kBucketGrid : 0)), bytes = o_spill + 8 * spill_cap;
    char* sc = nullptr;
    hipError_t e = ensure_scratch(scratch, bytes, stream, &sc);
    if (e != hipSuccess) return e;
    // from here on kernels may read the scratch: every exit records `done`
    // (a later grow frees the buffer only after it)
    auto fail_pass = [&](hipError_t err) {
      (void)release_scratch(scratch, stream);
      return err;
    };
    if (opts && opts->scratch_poison && (e = hipMemsetAsync(sc, 0xFF, bytes, stream)) != hipSuccess)
      return fail_pass(e);  // test-only: stale scratch contents
    uint32_t* range = reinterpret_cast<uint32_t*>(sc);
    uint32_t* cols = reinterpret_cast<uint32_t*>(sc + o_cols);
    uint32_t* tot = reinterpret_cast<uint32_t*>(sc + o_tot);
    uint32_t* start = reinterpret_cast<uint32_t*>(sc + o_start);
    uint32_t* ent = reinterpret_cast<uint32_t*>(sc + o_ent);
    uint32_t* tmp = reinterpret_cast<uint32_t*>(sc + o_tmp);
    BandZero bz{};
    bz.reg0 = reinterpret_cast<uint32_t*>(sc + o_reg);
    bz.n0 = reinterpret_cast<uint32_t*>(sc + o_n0);
    bz.spill = reinterpret_cast<unsigned long long*>(sc + o_spill);
    bz.nspill = range + 3;
    bz.k0 = k0;
    bz.spill_cap = spill_cap;
    bz.flag = scratch->flag;
    bz.count = count;
    hipLaunchKernelGGL(bucket_range_kernel, dim3(1), dim3(64), 0, stream, table, lo_p, vmax_p, ba.split, range,
                       bz.nspill);
    hipLaunchKernelGGL(bucket_count_kernel, dim3(kBucketGrid1), dim3(kBucketThreads), 4 * (uint32_t)ns, stream, table,
                       ba, range, cols);
    hipLaunchKernelGGL(bucket_colscan_kernel, dim3((uint32_t)((ns + 3) / 4)), dim3(256), 0, stream, cols,
                       (uint32_t)ns, tot);
    hipLaunchKernelGGL(bucket_startscan_kernel, dim3(1), dim3(1024), 0, stream, tot, (uint32_t)ns, start, cap,
                       scratch->flag, count);
    const uint32_t nsup = (uint32_t)((ns + kSupSegs - 1) >> kSupLog);
    const uint32_t nfill = band0 ? kBucketGrid : 0;
    const uint32_t lds_bytes = std::max(band0 ? 4 * (uint32_t)ns : 0u, band1 ? 4 * stage_lds_words(nsup) : 0u);
    if (lds_bytes > 65536 &&
        (e = hipFuncSetAttribute(reinterpret_cast<const void*>(&bucket_fill_stage_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes)) != hipSuccess)
      return fail_pass(e);
    hipLaunchKernelGGL(bucket_fill_stage_kernel, dim3(nfill + (band1 ? kBucketGrid1 : 0)), dim3(kBucketThreads),
                       lds_bytes, stream, table, ba, range, cols, start, bz, tmp, nsup, nfill, scratch->flag);
    if (band1) {
      hipLaunchKernelGGL(bucket_sort_kernel, dim3(nsup * (kBucketGrid1 / kSortGroup)), dim3(kSortThreads), 0,
                         stream, ba, cols, start, tmp, ent, scratch->flag);
    }
    if ((e = hipGetLastError()) != hipSuccess) return fail_pass(e);
    wa.bk_entries = ent;
    wa.bk_start = start;
    wa.bk_reg0 = bz.reg0;
    wa.bk_n0 = bz.n0;
    wa.bk_spill = bz.spill;
    wa.bk_nspill = bz.nspill;
    wa.bk_spill_cap = spill_cap;
    wa.bk_k0 = k0;
    if ((e = launch_wheel(table, wa, num_cus, stream)) != hipSuccess) return fail_pass(e);
    if ((e = release_scratch(scratch, stream)) != hipSuccess) return e;
    s0 += ns;
  }
  return hipSuccess;
}

}  // namespace

hipError_t launch_sieve_ranges(const void* table, const RangeSpec* rs, size_t n, int num_cus, hipStream_t stream,
                               Scratch* scratch, const SieveOpts* opts) {
  // ranges of up to 2^30 segments (the launch's 32-bit segment indices)
  constexpr uint64_t kMaxBits = (1ull << 30) * kWheelOutBits;
  std::vector<RangeSpec> pooled;
  for (size_t i = 0; i < n; ++i) {
    for (uint64_t b = 0; b < rs[i].nbits; b += kMaxBits) {
      const RangeSpec piece{rs[i].g_start + b, std::min(kMaxBits, rs[i].nbits - b),
                            rs[i].out ? rs[i].out + b / 32 : nullptr, rs[i].count};
      if (isqrt64(3 + 2 * (piece.g_start + piece.nbits - 1)) <= kWheelMaxPrime) {
        pooled.push_back(piece);
      } else {
        const hipError_t e = launch_bucketed(table, piece.g_start, piece.nbits, piece.out, piece.count, num_cus,
                                             stream, scratch, opts);
        if (e != hipSuccess) return e;
      }
    }
  }
  return launch_pooled(table, pooled.data(), pooled.size(), num_cus, stream, opts);
}

hipError_t launch_sieve_range(const void* table, uint64_t g_start, uint64_t nbits, uint32_t* out,
                              unsigned long long* count, int num_cus, hipStream_t stream, Scratch* scratch,
                              const SieveOpts* opts) {
  const RangeSpec rs{g_start, nbits, out, count};
  return launch_sieve_ranges(table, &rs, 1, num_cus, stream, scratch, opts);
}
#endif  // DSE_WHEEL_HALF_TU

}  // namespace dse

// Internal interface between the gfx950 kernels (dse_base.hip, dse_wheel.hip) and the
// C-ABI host layer (dse_host.cpp). Not installed; include/dse.h is the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dse {

// Base-prime table: one flat device buffer so ranks can broadcast it as bytes.
//   [0,16)            header {count, cap, limit}
//   [16, 16+4cap)     uint32 p[cap]      odd primes <= limit, ascending
//   [align8(...), +8cap) uint64 m[cap]  Barrett factors floor((2^64-1)/p) of the primes <= kWheelMaxPrime
//                                        (the bucketed primes' walks divide in double precision)
//   [align32(..), +32cap) uint32 a[8cap] wheel offsets, row i rotated by i mod 8:
//                                        a[8i+j] = first k >= 0 with p | R30[(j+i)&7] + 30k
//                                        (p >= 7; 0 for p = 3, 5)
//   [align32(..)+32cap, +8cap) uint32 pl[2][cap] the wheel kernel's large-prime words: p | plan << 20,
//                                        plan = the marking plan of the prime's set of 64 (unit_L;
//                                        pl[0] for 2^17-period segments, pl[1] for 2^16)
struct TableHeader {
  uint32_t count;
  uint32_t cap;
  uint64_t limit;
};

__host__ __device__ inline uint64_t table_m_offset(uint32_t cap) {
  return (16ull + 4ull * cap + 7ull) & ~7ull;
}
__host__ __device__ inline uint64_t table_a_offset(uint32_t cap) {
  return (table_m_offset(cap) + 8ull * cap + 31ull) & ~31ull;
}
__host__ __device__ inline uint64_t table_l_offset(uint32_t cap) { return table_a_offset(cap) + 32ull * cap; }
__host__ __device__ inline uint64_t table_bytes_for_cap(uint32_t cap) {
  return table_l_offset(cap) + 8ull * cap;
}

// The 8 residues mod 30 coprime to 30 (wheel planes, absolute numbering).
constexpr uint32_t kR30[8] = {1, 7, 11, 13, 17, 19, 23, 29};

// Mod-30 wheel segment geometry (dse_wheel.hip): a segment is 2^17 periods of
// 30 integers, 8 planes (one per coprime residue) x 8 columns of 2^14 periods
// (one 128 KiB LDS image). dse_wheel_half.hip compiles the same kernel with
// 2^16 periods per segment (range tails).
#ifndef DSE_WHEEL_LOG_KP
#define DSE_WHEEL_LOG_KP 17
#endif
constexpr int kWheelLogKP = DSE_WHEEL_LOG_KP;
constexpr uint64_t kWheelSpan = 30ull << kWheelLogKP;   // integers per segment
constexpr uint64_t kWheelOutBits = kWheelSpan / 2;      // odd candidates per segment
// Ranges with base primes above this go through the bucketed pass
// (dse_wheel.hip), which then buckets every prime above 2^kBucketLoLog.
#ifndef DSE_WHEEL_MAX_LOG
// Builds support 19 and 20 only: the L list's table words carry the prime in
// 20 bits (dse_wheel.hip kLPrimeMask), and the bucket threshold 2^19 must not
// exceed it. (r05 window A/B: 2^22 7.25 ms, 2^21 6.11, 2^20 5.62, 2^19 5.49)
#define DSE_WHEEL_MAX_LOG 20
#endif
constexpr uint64_t kWheelMaxPrime = 1ull << DSE_WHEEL_MAX_LOG;

// Largest limit the single-workgroup base-prime kernel handles (LDS bitmap).
constexpr uint64_t kBaseLimitMax = 2ull * 150u * 1024u * 8u + 1ull;  // 150 KiB of odd bits

// Big tables: odd primes < 2^31 (so p + SEG fits 32 bits in the kernel).
constexpr uint64_t kBigBaseLimitMax = (1ull << 31) - 1;

// Device scratch of one context (bucketed pass of high-offset ranges). Grows
// on demand, freed by free_scratch (dse_destroy). `done` is recorded on the
// stream of every pass after its last kernel that reads the buffer (any
// stream, the null stream included): the next pass's stream waits on it
// (hipStreamWaitEvent, no host block) and a grow or a free synchronises on it.
struct Scratch {
  void* ptr = nullptr;
  uint64_t bytes = 0;
  hipEvent_t done = nullptr;  // created on first use
  bool used = false;          // `done` has been recorded since the last grow
  uint32_t* flag = nullptr;   // device {sticky overflow, this pass's overflow} (bucket capacity)
};
hipError_t free_scratch(Scratch* s);

// Test-only knobs, set through dse_debug_set_option (include/dse.h); the
// defaults are the production configuration. No environment variable is read.
struct SieveOpts {
  uint32_t bucket_pass_segs = 0;  // > 0: cap the segments per bucket pass (multi-pass coverage)
  uint32_t bucket_split_log2 = 0; // > 0: bucketed primes <= 2^k filled one level, above two levels (0: production)
  uint32_t bucket_cap_div = 0;    // > 1: divide the (rigorous) bucket entry capacities, to test the overflow flag
  uint32_t bucket_k0_div = 0;     // > 1: divide the band-0 region capacity, to test the spill list
  uint32_t wheel_geometry = 0;    // ranges without buckets: 0 auto (half-size tail), 1 full only, 2 half only
  uint32_t scratch_poison = 0;    // 1: fill the bucket scratch with 0xFF bytes before every pass (stale contents)
  uint32_t bucket_lo_log2 = 0;    // k in 17..kWheelMaxLog: bucketed ranges bucket the primes above 2^k (0: production)
  uint64_t table_bcast_max = 0;   // > 0: broadcast cap of share_table in bytes (0: DSE_TABLE_BROADCAST_MAX_BYTES)
};

hipError_t launch_base_primes(uint64_t limit, void* table, uint32_t cap, hipStream_t stream);
// out[j] = sum_i in[i * n + j], i < nsrc (dse_debug_init_logical's count all-reduce)
hipError_t launch_sum_rows(const unsigned long long* in, uint32_t nsrc, uint32_t n, unsigned long long* out,
                           hipStream_t stream);
// Any limit <= kBigBaseLimitMax: the multi-workgroup kernel up to kBaseLimitMax,
// above it a sieve of [3, limit] by the wheel kernel + ordered compaction.
hipError_t launch_base_primes_big(uint64_t limit, void* table, uint32_t cap, int num_cus, hipStream_t stream);

// One odd-index range [g_start, g_start + nbits) of a launch: out (may be
// null) gets its mask as 32-bit words, *count (device) is incremented by its
// primes.
struct RangeSpec {
  uint64_t g_start;
  uint64_t nbits;
  uint32_t* out;
  unsigned long long* count;
};

// Sieve the ranges rs[0..n) on one stream: the ranges without bucketed primes
// share persistent launches of the wheel kernel (several chunks of one
// device: one launch, no idle partial rounds between them); ranges whose
// sqrt(max value) exceeds kWheelMaxPrime run their bucketed passes one by one
// (they need `scratch`). `opts` may be null. Empty ranges are skipped.
hipError_t launch_sieve_ranges(const void* table, const RangeSpec* rs, size_t n, int num_cus, hipStream_t stream,
                               Scratch* scratch, const SieveOpts* opts);
// Sieve odd indices [g_start, g_start+nbits) with the mod-30 wheel kernel: out
// (may be null) gets the mask as 32-bit words (2*ceil(nbits/64) of them, upper
// half of the last uint64 zeroed); *count (device) is incremented. Ranges whose
// sqrt(max value) exceeds kWheelMaxPrime need `scratch` (bucketed pass);
// `opts` may be null.
hipError_t launch_sieve_range(const void* table, uint64_t g_start, uint64_t nbits, uint32_t* out,
                              unsigned long long* count, int num_cus, hipStream_t stream, Scratch* scratch,
                              const SieveOpts* opts);
// The same sieve with the half-size segment geometry (2^16 periods,
// dse_wheel_half.hip): launch_sieve_ranges gives it the segments past the last
// full round of a launch when that finishes sooner. No bucketed primes.
hipError_t launch_wheel_ranges_half(const void* table, const RangeSpec* rs, size_t n, int num_cus,
                                    hipStream_t stream);
// The full-geometry wheel kernel without bucketed primes (dse_wheel_plain.hip,
// its own compile flags); wa points at the caller's WheelArgs (dse_wheel.hip).
hipError_t launch_wheel_plain(const void* table, const void* wa, int num_cus, hipStream_t stream);
// Fill the Barrett factors m[] and wheel offsets a[] of a table whose p[] is final.
// n_hint: table capacity when known (sizes the grid: about 4 primes per thread)
hipError_t launch_wheel_offsets(void* table, int num_cus, hipStream_t stream, uint64_t n_hint = 0);

}  // namespace dse

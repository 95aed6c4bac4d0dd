// Internal interface between the gfx950 kernels (dse_kernels.hip) and the
// C-ABI host layer (dse_host.cpp). Not installed; include/dse.h is the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dse {

// Base-prime table: one flat device buffer so ranks can broadcast it as bytes.
//   [0,16)            header {count, cap, limit}
//   [16, 16+4cap)     uint32 p[cap]      odd primes <= limit, ascending
//   [align8(...), +8cap) uint64 m[cap]  Barrett factors floor((2^64-1)/p)
struct TableHeader {
  uint32_t count;
  uint32_t cap;
  uint64_t limit;
};

__host__ __device__ inline uint64_t table_m_offset(uint32_t cap) {
  return (16ull + 4ull * cap + 7ull) & ~7ull;
}
__host__ __device__ inline uint64_t table_bytes_for_cap(uint32_t cap) {
  return table_m_offset(cap) + 8ull * cap;
}

// Segment geometry of the marking kernel (see DESIGN.md "Kernels").
constexpr int kLogSeg = 20;               // 2^20 odd candidates per LDS segment (128 KiB)
constexpr int kThreads = 1024;            // 16 waves per workgroup, one workgroup per CU
constexpr int kSmallMax = 61;             // primes <= 61: register patterns at write-back

// Largest limit the single-workgroup base-prime kernel handles (LDS bitmap).
constexpr uint64_t kBaseLimitMax = 2ull * 150u * 1024u * 8u + 1ull;  // 150 KiB of odd bits

// Big tables: odd primes < 2^31 (so p + SEG fits 32 bits in the kernel).
constexpr uint64_t kBigBaseLimitMax = (1ull << 31) - 1;

hipError_t launch_base_primes(uint64_t limit, void* table, uint32_t cap, hipStream_t stream);
// Any limit <= kBigBaseLimitMax: the one-workgroup kernel up to kBaseLimitMax,
// above it a sieve of [3, limit] by the segment kernel + ordered compaction.
hipError_t launch_base_primes_big(uint64_t limit, void* table, uint32_t cap, int num_cus, hipStream_t stream);

// Sieve odd indices [g_start, g_start+nbits): out (may be null) gets the mask as
// 32-bit words (2*ceil(nbits/64) of them, upper half of the last uint64 zeroed);
// *count (device) is incremented.
hipError_t launch_sieve_range(const void* table, uint64_t g_start, uint64_t nbits, uint32_t* out,
                              unsigned long long* count, int num_cus, hipStream_t stream);

}  // namespace dse

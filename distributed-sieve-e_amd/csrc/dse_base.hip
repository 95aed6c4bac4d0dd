// dse_base.hip -- base-prime tables on the device (gfx950).
//
// The reference finds every sieving prime with a serial survivor scan
// (find-first-prime / find-next-non-zero, sieve.clj:73-80,110-116) and relays
// each one to the other machines (sieve.clj:139). Here the odd primes up to
// sqrt(max value) are computed once, on the device, into a flat table
// (dse_internal.h) that ranks can RCCL-broadcast as bytes:
//   - limit <= kBaseLimitMax: base_mask_kernel (many workgroups, LDS slices)
//     + an ordered count / scan / write compaction;
//   - larger limits (high-offset windows, up to 2^31): the wheel kernel sieves
//     [3, limit] from a first-level table, then the same compaction;
//   - then wheel_offsets_kernel (dse_wheel.hip) fills the Barrett factors and
//     the mod-30 wheel-offset rows.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "dse_internal.h"

namespace dse {
namespace {

// ---------------------------------------------------------------------------
// Big base-prime tables (limit above kBaseLimitMax, e.g. 1e9 for the 1e18
// window): sieve [3, limit] with the segment kernel itself, then compact the
// prime bits into an ordered table. Scratch lives in the table's m[] region,
// which is only written at the very end.
// ---------------------------------------------------------------------------
constexpr uint32_t kCompactWordsPerThread = 2;
constexpr uint32_t kCompactThreads = 256;
constexpr uint32_t kCompactBlockWords = kCompactWordsPerThread * kCompactThreads;  // 512 words
constexpr uint32_t kCompactStage = 8192;  // LDS slots for a block's primes (32 KiB)

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
  __shared__ uint32_t s_stage[kCompactStage];
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
  // the block's primes are staged in LDS in order, then stored as one
  // contiguous run (each thread's primes are consecutive slots, so direct
  // stores would put a wave's lanes ~a dozen slots apart: one line each);
  // slots past kCompactStage (never at the densest block, 6,542 primes) go
  // straight to global memory
  const uint32_t base = block_offs[blockIdx.x], total = s_scan[kCompactThreads - 1];
  uint32_t pos = s_scan[tid] - c;
#pragma unroll
  for (uint32_t k = 0; k < kCompactWordsPerThread; ++k) {
    uint64_t x = v[k];
    while (x) {
      const uint32_t b = __ffsll((long long)x) - 1;
      x &= x - 1;
      const uint32_t q = (uint32_t)(3 + 2 * ((w0 + k) * 64 + b));
      if (pos < kCompactStage)
        s_stage[pos] = q;
      else if (base + pos < cap)
        P[base + pos] = q;
      ++pos;
    }
  }
  __syncthreads();
  const uint32_t n = min(total, kCompactStage);
  for (uint32_t j = tid; j < n; j += kCompactThreads)
    if (base + j < cap) P[base + j] = s_stage[j];
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

// out[j] = sum over i < nsrc of in[i * n + j] (the logical-device stand-in for
// the count all-reduce, dse_debug_init_logical)
__global__ __launch_bounds__(256) void sum_rows_kernel(const unsigned long long* __restrict__ in, uint32_t nsrc,
                                                       uint32_t n, unsigned long long* __restrict__ out) {
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) {
    unsigned long long t = 0;
    for (uint32_t i = 0; i < nsrc; ++i) t += in[(uint64_t)i * n + j];
    out[j] = t;
  }
}

}  // namespace

hipError_t launch_sum_rows(const unsigned long long* in, uint32_t nsrc, uint32_t n, unsigned long long* out,
                           hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(sum_rows_kernel, dim3(std::min<uint32_t>((n + 255) / 256, 1024u)), dim3(256), 0, stream, in,
                     nsrc, n, out);
  return hipGetLastError();
}

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
  // sqrt(limit) < 2^16 <= kWheelMaxPrime: no bucketed pass, no scratch
  e = launch_sieve_range(t0, 0, nb, reinterpret_cast<uint32_t*>(mask), cnt, num_cus, stream, nullptr, nullptr);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(compact_count_kernel, dim3(nblocks), dim3(kCompactThreads), 0, stream, mask, words, sums);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, stream, sums, nblocks, table, cap, limit);
  uint32_t* P = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(table) + 16);
  hipLaunchKernelGGL(compact_write_kernel, dim3(nblocks), dim3(kCompactThreads), 0, stream, mask, words, sums, P,
                     cap);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return launch_wheel_offsets(table, num_cus, stream, cap);  // m[] and a[]
}

}  // namespace dse

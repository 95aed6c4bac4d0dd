// lds_oor_bench.hip -- what does a ds_or_b32 outside the workgroup's LDS
// allocation do on gfx950, and what does it cost? (profiling aid, not product
// code)
//
// 1. Semantics: a 1024-thread workgroup with 160 KiB of LDS fills it with a
//    pattern, then every lane ORs all-ones into addresses at and past the end
//    of the allocation (163,840 .. 2^31, some through the instruction's
//    offset field), and reads one back; the pattern must be intact and the
//    read must return 0. Prints the mismatches (expected: 0) and the reads.
// 2. Cost: the wheel kernel's mark stream (3 VALU + ds_or_b32 per mark, random
//    banks, 16 waves per CU) with the 128 KiB image at LDS byte 32,768 (the
//    base in the ds offset field), where a fraction of the lanes mark past
//    the image (k >= 2^17: address >= 163,840, i.e. outside the allocation)
//    instead of being masked off by exec. CU-cycles per ds_or wave-instruction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint32_t kWords = 40960;  // 160 KiB

__global__ __launch_bounds__(1024) void semantics(uint32_t* bad, uint32_t* rd) {
  __shared__ uint32_t lds[kWords];
  for (uint32_t i = threadIdx.x; i < kWords; i += 1024) lds[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t ones = 0xFFFFFFFFu;
  uint32_t a0 = 163840u + 4 * lane, a1 = 163840u + 4096u + 4 * threadIdx.x, a2 = (1u << 20) + 4 * lane,
           a3 = (1u << 24) + 4 * lane, a4 = 0x7FFFFF00u + 4 * (lane & 31), a5 = 131072u + 4 * lane;
  asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5));
  asm volatile(
      "ds_or_b32 %0, %6\n\t"
      "ds_or_b32 %1, %6\n\t"
      "ds_or_b32 %2, %6\n\t"
      "ds_or_b32 %3, %6\n\t"
      "ds_or_b32 %4, %6\n\t"
      "ds_or_b32 %5, %6 offset:32768\n\t"
      "s_waitcnt lgkmcnt(0)"
      :
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(ones)
      : "memory");
  uint32_t r;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a2) : "memory");
  __syncthreads();
  uint32_t nbad = 0;
  for (uint32_t i = threadIdx.x; i < kWords; i += 1024) nbad += lds[i] != i * 2654435761u;
  atomicAdd(bad, nbad);
  if (r) atomicAdd(rd, 1u);
}

constexpr uint32_t kImgOff = 32768;  // image at LDS bytes [32768, 163840)

// OOR_MASK: lanes whose bit is set mark at k | 2^17 (past the image: outside
// the allocation); EXEC_HALF: lanes 32..63 masked off by exec instead (the
// kernel's predicated marks).
template <uint64_t OOR_MASK, bool EXEC_HALF>
__global__ __launch_bounds__(1024) void stream(uint32_t* out, unsigned long long* cyc, uint32_t iters) {
  __shared__ uint32_t lds[kWords];
  for (uint32_t i = threadIdx.x; i < kWords; i += 1024) lds[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  // address (k & 0x1FFE0) | pb: in the image, or past it for the OOR lanes
  const uint32_t pb = 4 * (lane & 7) | (((OOR_MASK >> lane) & 1) ? (1u << 17) : 0u);
  const uint32_t p = 1537 + 2 * ((threadIdx.x * 2654435761u) % 4000u);
  uint32_t k = (threadIdx.x * 977u) & 0x1FFFFu;
  uint32_t one = 1;
  asm volatile("" : "+v"(one));
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (!EXEC_HALF || lane < 32) {
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        uint32_t a, b;
        asm volatile(
            "v_and_or_b32 %0, %2, %3, %4\n\t"
            "v_lshlrev_b32 %1, %2, %6\n\t"
            "v_add_u32 %2, %2, %5\n\t"
            "ds_or_b32 %0, %1 offset:32768"
            : "=&v"(a), "=&v"(b), "+v"(k)
            : "s"(0x1FFE0u), "v"(pb), "v"(p), "v"(one)
            : "memory");
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  out[blockIdx.x * 1024 + threadIdx.x] = lds[kImgOff / 4 + threadIdx.x * 32];
  if (lane == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <uint64_t M, bool H>
void run(const char* name, uint32_t* d, unsigned long long* dc) {
  const uint32_t iters = 1024, cus = 256;
  hipLaunchKernelGGL((stream<M, H>), dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  hipLaunchKernelGGL((stream<M, H>), dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  (void)hipDeviceSynchronize();
  static unsigned long long h[256 * 16];
  (void)hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
  double sum = 0;
  for (uint32_t i = 0; i < cus * 16; ++i) sum += (double)h[i];
  const double per_wave_instr = sum / (cus * 16) / (16.0 * iters);
  printf("%-40s %.2f CU-cycles per ds_or_b32 wave-instruction\n", name, per_wave_instr / 16);
}

int main() {
  uint32_t* d;
  unsigned long long* dc;
  (void)hipMalloc(&d, 256 * 1024 * 4);
  (void)hipMalloc(&dc, 256 * 16 * 8);
  (void)hipMemset(d, 0, 8);
  hipLaunchKernelGGL(semantics, dim3(256), dim3(1024), 0, 0, d, d + 1);
  uint32_t h[2] = {~0u, ~0u};
  hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
  printf("semantics: %s; LDS words changed by out-of-range ds_or: %u; non-zero out-of-range reads: %u\n",
         hipGetErrorString(e), h[0], h[1]);
  run<0ull, false>("all lanes in range", d, dc);
  run<0ull, true>("lanes 32-63 off by exec", d, dc);
  run<0xFFFFFFFF00000000ull, false>("lanes 32-63 out of range", d, dc);
  run<0xAAAAAAAAAAAAAAAAull, false>("odd lanes out of range", d, dc);
  run<0xFFFFFFFFFFFFFFFFull, false>("all lanes out of range", d, dc);
  (void)hipFree(d);
  (void)hipFree(dc);
  return 0;
}

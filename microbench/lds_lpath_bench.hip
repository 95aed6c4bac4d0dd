// lds_lpath_bench.hip -- the wheel kernel's large-prime (L) mark pattern on
// gfx950 LDS (profiling aid): lane L at step q marks plane (q + L) & 7 at a
// random (row, column) of a 128 KiB image laid out as word (row, 8*plane+col)
// = row*64 + 8*plane + col. Variants: ds_or_b32 (the kernel today), ds_or_b64
// on the 8-byte pair of columns (2k, 2k+1) with the bit in its half, and
// ds_or_b32 with ~40% of the lanes exec-masked off. In-kernel s_memtime,
// cycles per wave-instruction per CU (16 waves per CU).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(1024) void k(uint32_t* out, unsigned long long* cyc, uint32_t iters) {
  __shared__ uint32_t img[32768];
  for (uint32_t i = threadIdx.x; i < 32768; i += 1024) img[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t x = (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u) ^ 0x9e3779b9u;
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)img;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
      x = x * 1664525u + 1013904223u;
      const uint32_t plane = (q + lane) & 7, col = (x >> 10) & 7, row = (x >> 13) & 511, b = x & 31;
      if (MODE == 0) {
        const uint32_t a = base + row * 256 + (8 * plane + col) * 4;
        asm volatile("ds_or_b32 %0, %1" ::"v"(a), "v"(1u << b) : "memory");
      } else if (MODE == 1) {
        const uint32_t a = base + row * 256 + (8 * plane + (col & 6)) * 4;
        const uint64_t d = 1ull << (((col & 1) << 5) | b);
        asm volatile("ds_or_b64 %0, %1" ::"v"(a), "v"(d) : "memory");
      } else {
        const uint32_t a = base + row * 256 + (8 * plane + col) * 4;
        if ((x >> 24) < 154) asm volatile("ds_or_b32 %0, %1" ::"v"(a), "v"(1u << b) : "memory");
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  out[blockIdx.x * 1024 + threadIdx.x] = img[threadIdx.x * 32];
  if (lane == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE>
void run(const char* name, uint32_t* d, unsigned long long* dc) {
  const uint32_t iters = 512, cus = 256;
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  (void)hipDeviceSynchronize();
  unsigned long long h[256 * 16];
  (void)hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
  unsigned long long mx = 0;
  for (uint32_t i = 0; i < cus * 16; ++i) mx = h[i] > mx ? h[i] : mx;
  printf("%-22s %.2f cycles per wave-instruction per CU\n", name, (double)mx / (16.0 * iters * 8));
}

int main() {
  uint32_t* d;
  unsigned long long* dc;
  (void)hipMalloc(&d, 256 * 1024 * 4);
  (void)hipMalloc(&dc, 256 * 16 * 8);
  run<0>("or_b32 L pattern", d, dc);
  run<1>("or_b64 column pairs", d, dc);
  run<2>("or_b32 60% exec", d, dc);
  (void)hipFree(d);
  (void)hipFree(dc);
  return 0;
}

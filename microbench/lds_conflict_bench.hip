// lds_conflict_bench.hip -- cost of one ds_or_b32 wave-instruction on gfx950
// as a function of the bank pattern (profiling aid for the wheel kernel's L
// marks). Addresses are precomputed in registers (16 per lane, one per
// instruction), so the loop is ds_or_b32 only; 16 waves per CU; in-kernel
// s_memtime, mean over waves -> CU-cycles per wave-instruction.
//   way-k : every bank of a half-wave takes k lanes at k distinct rows
//   L     : the kernel's L pattern: 4 lanes per plane, column c random,
//           bank 8 (c & 3) + plane
//   random: 32 lanes to 32 random banks
//   half  : conflict-free, lanes 32..63 exec-masked off
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ uint32_t hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(1024) void k(uint32_t* out, unsigned long long* cyc, uint32_t iters) {
  __shared__ uint32_t img[32768];
  for (uint32_t i = threadIdx.x; i < 32768; i += 1024) img[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, h = lane & 31;
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)img;
  uint32_t a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t r = hash(threadIdx.x * 16 + j + blockIdx.x * 65536);
    const uint32_t row = r & 511;
    uint32_t bank;
    if (MODE >= 1 && MODE <= 4) bank = h / MODE;             // MODE lanes per bank (k-way)
    else if (MODE == 5) bank = 8 * ((r >> 9) & 3) + ((h + j) & 7);  // L pattern
    else if (MODE == 6) bank = (r >> 9) & 31;                 // random
    else bank = h;                                            // conflict-free (0) / half (7)
    a[j] = base + row * 256 + 4 * ((bank + 32 * (lane >> 5)) & 63);
  }
  const uint32_t bit = 1u << (lane & 31);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
    if (MODE == 7 && lane >= 32) continue;
#pragma unroll
    for (int j = 0; j < 16; ++j) asm volatile("ds_or_b32 %0, %1" ::"v"(a[j]), "v"(bit) : "memory");
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
  double sum = 0;
  for (uint32_t i = 0; i < cus * 16; ++i) sum += (double)h[i];
  printf("%-16s %.2f CU-cycles per ds_or_b32 wave-instruction\n", name, sum / (cus * 16) / (16.0 * iters * 16) * 16);
}

int main() {
  uint32_t* d;
  unsigned long long* dc;
  (void)hipMalloc(&d, 256 * 1024 * 4);
  (void)hipMalloc(&dc, 256 * 16 * 8);
  run<0>("conflict-free", d, dc);
  run<2>("2-way", d, dc);
  run<3>("3-way", d, dc);
  run<4>("4-way", d, dc);
  run<5>("L pattern", d, dc);
  run<6>("random", d, dc);
  run<7>("half lanes", d, dc);
  (void)hipFree(d);
  (void)hipFree(dc);
  return 0;
}

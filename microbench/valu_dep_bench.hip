// valu_dep_bench.hip -- dependent-issue cost of VALU chains on gfx950
// (profiling aid): 16 waves per CU, C independent chains per lane
// interleaved (C = 1, 2, 4, 8), plus a conflict-free mark-like sequence
// (add, lshl, and_or, lshl, ds_or) with 1 or 2 interleaved streams. Prints
// cycles per wave-instruction per wave (mean over waves, s_memtime).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int C, int MODE>
__global__ __launch_bounds__(1024) void k(uint32_t* out, unsigned long long* cyc, uint32_t iters) {
  __shared__ uint32_t img[32768];
  for (uint32_t i = threadIdx.x; i < 32768; i += 1024) img[i] = 0;
  uint32_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = threadIdx.x * 7 + j * 131;
  const uint32_t s = (threadIdx.x & 31) | 1;
  const uint32_t cb = 4 * (threadIdx.x & 63);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16 / C; ++r) {
#pragma unroll
      for (int j = 0; j < C; ++j) {
        if (MODE == 0) {
          asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[j]) : "v"(s));
        } else if (MODE == 1) {
          asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(v[j]) : "v"(s));
        } else {
          uint32_t a, b;
          asm volatile(
              "v_lshlrev_b32 %0, 3, %2\n\t"
              "v_and_or_b32 %0, %0, %4, %3\n\t"
              "v_lshlrev_b32 %1, %2, 1\n\t"
              "ds_or_b32 %0, %1\n\t"
              "v_add_u32 %2, %2, %5"
              : "=&v"(a), "=&v"(b), "+v"(v[j])
              : "v"(cb), "s"(0x1ff00u), "v"(s)
              : "memory");
        }
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= v[j];
  out[blockIdx.x * 1024 + threadIdx.x] = r + img[threadIdx.x];
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int C, int MODE>
void run(const char* name, uint32_t* d, unsigned long long* dc, int cus) {
  const uint32_t iters = 1024;
  hipLaunchKernelGGL((k<C, MODE>), dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  hipLaunchKernelGGL((k<C, MODE>), dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  (void)hipDeviceSynchronize();
  unsigned long long h[256 * 16];
  (void)hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
  double sum = 0;
  for (int i = 0; i < cus * 16; ++i) sum += (double)h[i];
  const double per_wave_instr = 16.0 * iters * (MODE == 2 ? 5 : 1);
  const double cyc = sum / (cus * 16) / per_wave_instr;
  printf("%-28s chains=%d  %.2f cycles per instr per wave  -> %.3f instr/CU-cycle\n", name, C, cyc, 16.0 / cyc);
}

int main() {
  int cus = 256;
  uint32_t* d;
  unsigned long long* dc;
  (void)hipMalloc(&d, (size_t)cus * 1024 * 4);
  (void)hipMalloc(&dc, (size_t)cus * 16 * 8);
  run<1, 0>("v_add dep", d, dc, cus);
  run<2, 0>("v_add dep", d, dc, cus);
  run<4, 0>("v_add dep", d, dc, cus);
  run<8, 0>("v_add dep", d, dc, cus);
  run<1, 1>("v_and_or dep", d, dc, cus);
  run<2, 1>("v_and_or dep", d, dc, cus);
  run<4, 1>("v_and_or dep", d, dc, cus);
  run<8, 1>("v_and_or dep", d, dc, cus);
  run<1, 2>("mark seq (4 VALU + ds_or)", d, dc, cus);
  run<2, 2>("mark seq (4 VALU + ds_or)", d, dc, cus);
  run<4, 2>("mark seq (4 VALU + ds_or)", d, dc, cus);
  (void)hipFree(d);
  (void)hipFree(dc);
  return 0;
}

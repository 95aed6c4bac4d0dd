// valu_rate_bench.hip -- issue rate of a few VALU forms on gfx950 (profiling
// aid for the wheel kernel's VALU budget). 16 waves per CU, 16 independent
// chains per lane, inline asm so the compiler cannot fold the chains; the rate
// is wave-instructions per CU per shader cycle, timed in-kernel with s_memtime
// (cycle counter, independent of the clock the chip holds).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int MODE>
__global__ __launch_bounds__(1024) void k(uint32_t* out, unsigned long long* cyc, uint32_t iters) {
  uint32_t v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = threadIdx.x * 7 + j;
  uint64_t a64[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a64[j] = threadIdx.x * 0x1234567ull + j;
  const uint32_t s = threadIdx.x & 31;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < iters; ++i) {
    if (MODE == 0) {
#define OP(j) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[j]) : "v"(s));
      REP16(OP)
#undef OP
    } else if (MODE == 1) {
#define OP(j) asm volatile("v_lshl_or_b32 %0, %0, %1, %1" : "+v"(v[j]) : "v"(s));
      REP16(OP)
#undef OP
    } else if (MODE == 2) {
#define OP(j) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(v[j]) : "v"(s));
      REP16(OP)
#undef OP
    } else if (MODE == 3) {
#define OP(j) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(a64[(j) & 7]) : "v"(s));
      REP16(OP)
#undef OP
    } else if (MODE == 4) {
#define OP(j) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(v[j]));
      REP16(OP)
#undef OP
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) r ^= v[j];
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= (uint32_t)a64[j];
  out[blockIdx.x * 1024 + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE>
void run(const char* name, uint32_t* d, unsigned long long* dc, int cus) {
  const uint32_t iters = 2048;
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  (void)hipDeviceSynchronize();
  unsigned long long h[256 * 16];
  (void)hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
  unsigned long long mx = 0, sum = 0;
  for (int i = 0; i < cus * 16; ++i) { mx = h[i] > mx ? h[i] : mx; sum += h[i]; }
  const double ops = 16.0 * iters * 16;  // wave-instructions per CU
  printf("%-12s %.3f wave-instr/CU-cycle (max wave cycles %llu, mean %.0f)\n", name, ops / (double)mx, mx,
         (double)sum / (cus * 16));
}

int main() {
  int cus = 256;
  uint32_t* d;
  unsigned long long* dc;
  (void)hipMalloc(&d, (size_t)cus * 1024 * 4);
  (void)hipMalloc(&dc, (size_t)cus * 16 * 8);
  run<0>("v_add_u32", d, dc, cus);
  run<1>("v_lshl_or", d, dc, cus);
  run<2>("v_and_or", d, dc, cus);
  run<3>("v_lshl_b64", d, dc, cus);
  run<4>("v_fma_f32", d, dc, cus);
  (void)hipFree(d);
  (void)hipFree(dc);
  return 0;
}

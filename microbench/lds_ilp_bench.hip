// lds_ilp_bench.hip -- does instruction-level parallelism inside a wave speed
// up the wheel kernel's mark runs on gfx950? (profiling aid, not product code)
//
// Every lane walks C independent mark chains k += p through a 128 KiB
// word-interleaved image (address (k & ~31) | plane base, bit 1 << k: the
// kernel's mark_k_step), 16 waves per CU, one 1024-thread workgroup per CU as
// in the kernel. C = 1 is the kernel's mark_run; C = 2 / 4 interleave the
// chains inside one asm block so a ds_or never waits on the VALU that just
// wrote its operands. Prints CU-cycles (s_memtime, mean over waves / 16) per
// ds_or_b32 wave-instruction for each C, and with exec halved (tails).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int C>
__device__ __forceinline__ void steps(uint32_t (&k)[4], uint32_t pb, uint32_t p, uint32_t one) {
  uint32_t a0, b0, a1, b1, a2, b2, a3, b3;
  if (C == 1) {
    asm volatile(
        "v_and_or_b32 %0, %2, %3, %4\n\t"
        "v_lshlrev_b32 %1, %2, %6\n\t"
        "v_add_u32 %2, %2, %5\n\t"
        "ds_or_b32 %0, %1"
        : "=&v"(a0), "=&v"(b0), "+v"(k[0])
        : "s"(~31u), "v"(pb), "v"(p), "v"(one)
        : "memory");
  } else if (C == 2) {
    asm volatile(
        "v_and_or_b32 %0, %4, %6, %7\n\t"
        "v_lshlrev_b32 %1, %4, %9\n\t"
        "v_add_u32 %4, %4, %8\n\t"
        "v_and_or_b32 %2, %5, %6, %7\n\t"
        "v_lshlrev_b32 %3, %5, %9\n\t"
        "v_add_u32 %5, %5, %8\n\t"
        "ds_or_b32 %0, %1\n\t"
        "ds_or_b32 %2, %3"
        : "=&v"(a0), "=&v"(b0), "=&v"(a1), "=&v"(b1), "+v"(k[0]), "+v"(k[1])
        : "s"(~31u), "v"(pb), "v"(p), "v"(one)
        : "memory");
  } else {
    asm volatile(
        "v_and_or_b32 %0, %8, %12, %13\n\t"
        "v_lshlrev_b32 %1, %8, %15\n\t"
        "v_add_u32 %8, %8, %14\n\t"
        "v_and_or_b32 %2, %9, %12, %13\n\t"
        "v_lshlrev_b32 %3, %9, %15\n\t"
        "v_add_u32 %9, %9, %14\n\t"
        "ds_or_b32 %0, %1\n\t"
        "v_and_or_b32 %4, %10, %12, %13\n\t"
        "v_lshlrev_b32 %5, %10, %15\n\t"
        "v_add_u32 %10, %10, %14\n\t"
        "ds_or_b32 %2, %3\n\t"
        "v_and_or_b32 %6, %11, %12, %13\n\t"
        "v_lshlrev_b32 %7, %11, %15\n\t"
        "v_add_u32 %11, %11, %14\n\t"
        "ds_or_b32 %4, %5\n\t"
        "ds_or_b32 %6, %7"
        : "=&v"(a0), "=&v"(b0), "=&v"(a1), "=&v"(b1), "=&v"(a2), "=&v"(b2), "=&v"(a3), "=&v"(b3), "+v"(k[0]),
          "+v"(k[1]), "+v"(k[2]), "+v"(k[3])
        : "s"(~31u), "v"(pb), "v"(p), "v"(one)
        : "memory");
  }
}

// E extra VALU per mark (independent of the chain), a drain (s_waitcnt
// lgkmcnt(0), as a unit claim does) every D iterations of 16 marks (0: none)
template <int C, bool HALF, int E = 0, int D = 0>
__global__ __launch_bounds__(1024) void kern(uint32_t* out, unsigned long long* cyc, uint32_t iters) {
  __shared__ uint32_t img[32768];
  for (uint32_t i = threadIdx.x; i < 32768; i += 1024) img[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t pb = 4 * (lane & 7);
  const uint32_t p = 1537 + 2 * ((threadIdx.x * 2654435761u) % 4000u);
  uint32_t k[4];
  for (int c = 0; c < 4; ++c) k[c] = (threadIdx.x * 977u + c * 40503u) & 0x1FFFFu;
  uint32_t one = 1;
  asm volatile("" : "+v"(one));
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (!HALF || lane < 32) {
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 16 / C; ++r) {
        steps<C>(k, pb, p, one);
#pragma unroll
        for (int e = 0; e < E * C; ++e) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(one) : "v"(e) );
      }
      if (D && it % D == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int c = 0; c < 4; ++c) k[c] &= 0x1FFFFu;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  out[blockIdx.x * 1024 + threadIdx.x] = img[threadIdx.x * 32];
  if (lane == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int C, bool HALF, int E = 0, int D = 0>
void run(const char* name, uint32_t* d, unsigned long long* dc) {
  const uint32_t iters = 1024, cus = 256;
  hipLaunchKernelGGL((kern<C, HALF, E, D>), dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  hipLaunchKernelGGL((kern<C, HALF, E, D>), dim3(cus), dim3(1024), 0, 0, d, dc, iters);
  (void)hipDeviceSynchronize();
  static unsigned long long h[256 * 16];
  (void)hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
  double sum = 0;
  for (uint32_t i = 0; i < cus * 16; ++i) sum += (double)h[i];
  const double per_wave_instr = sum / (cus * 16) / (16.0 * iters);
  printf("%-28s %.2f CU-cycles per ds_or_b32 wave-instruction (%.1f per wave)\n", name, per_wave_instr / 16,
         per_wave_instr);
}

int main() {
  uint32_t* d;
  unsigned long long* dc;
  (void)hipMalloc(&d, 256 * 1024 * 4);
  (void)hipMalloc(&dc, 256 * 16 * 8);
  run<1, false>("1 chain (mark_k_step)", d, dc);
  run<2, false>("2 chains interleaved", d, dc);
  run<4, false>("4 chains interleaved", d, dc);
  run<1, true>("1 chain, half the lanes", d, dc);
  run<2, true>("2 chains, half the lanes", d, dc);
  run<1, false, 2>("1 chain, +2 VALU per mark", d, dc);
  run<1, false, 4>("1 chain, +4 VALU per mark", d, dc);
  run<1, false, 0, 1>("1 chain, drain every 16", d, dc);
  run<1, false, 0, 4>("1 chain, drain every 64", d, dc);
  run<1, false, 2, 4>("+2 VALU, drain every 64", d, dc);
  (void)hipFree(d);
  (void)hipFree(dc);
  return 0;
}

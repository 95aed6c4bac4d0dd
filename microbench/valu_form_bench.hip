// valu_form_bench.hip -- issue rate of the VALU forms the wheel kernel's
// mark paths use, on gfx950 (profiling aid): 16 waves per CU, 8 independent
// chains per lane, mean over waves, in-kernel s_memtime ->
// wave-instructions per CU-cycle.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(1024) void k(uint32_t* out, unsigned long long* cyc, uint32_t iters, uint32_t sk) {
  uint32_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = threadIdx.x * 7 + j * 131;
  const uint32_t w = threadIdx.x | 1;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MODE == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[j]) : "v"(w));
        if (MODE == 1) asm volatile("v_lshlrev_b32 %0, %0, 1" : "+v"(v[j]));                 // VOP3, const src1
        if (MODE == 2) asm volatile("v_lshlrev_b32 %0, %0, %1" : "+v"(v[j]) : "v"(w));        // VOP2
        if (MODE == 3) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(v[j]) : "s"(sk), "v"(w));  // v, s, v
        if (MODE == 4) asm volatile("v_lshl_or_b32 %0, %0, 5, %1" : "+v"(v[j]) : "v"(w));     // v, c, v
        if (MODE == 5) asm volatile("v_bfe_u32 %0, %0, 14, 3" : "+v"(v[j]));                  // v, c, c
        if (MODE == 6) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(v[j]) : "s"(sk), "v"(w));  // s, v, v
        if (MODE == 7) asm volatile("v_cndmask_b32 %0, 0, %0, vcc" : "+v"(v[j]));             // VOP2 (vcc)
        if (MODE == 8) asm volatile("v_min_u32 %0, %0, %1" : "+v"(v[j]) : "v"(w));            // VOP2
        if (MODE == 9) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(v[j]) : "v"(w));       // v, v, v
        if (MODE == 10) asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(v[j]) : "v"(w));  // v, v, vcc
        if (MODE == 11) asm volatile("v_cndmask_b32_e64 %0, 0, %0, s[40:41]" : "+v"(v[j]));  // e64, sgpr pair
        if (MODE == 12) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(v[j]), "v"(w) : "vcc");  // VOPC
        if (MODE == 13) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[j]) : "v"(w));
        if (MODE == 14) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[j]) : "v"(w));
        if (MODE == 15) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[j]) : "v"(w), "s"(sk));
        if (MODE == 16) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(v[j]) : "v"(w));
        if (MODE == 17) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v[j]) : "v"(w));
        if (MODE == 18) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[j]) : "v"(w));
        if (MODE == 19) asm volatile("v_or_b32 %0, %0, %1" : "+v"(v[j]) : "v"(w));
        if (MODE == 20) asm volatile("v_mov_b32 %0, %1" : "=v"(v[j]) : "v"(v[(j + 1) & 7]));
        if (MODE == 21) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(v[j]));
        if (MODE == 22) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[j]) : "v"(w));
        if (MODE == 23) asm volatile("v_ashrrev_i32 %0, 31, %0" : "+v"(v[j]));
        // select pairs (counted as 2 instructions): cmp + cndmask through VCC, through an SGPR pair, arithmetic mask
        if (MODE == 24) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %1, %0, vcc" : "+v"(v[j]) : "v"(w) : "vcc");
        if (MODE == 25) {
          uint64_t m;
          asm volatile("v_cmp_gt_u32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %2, %0, %1" : "+v"(v[j]), "=s"(m) : "v"(w));
        }
        if (MODE == 26) {
          uint32_t t;
          asm volatile("v_sub_u32 %1, %0, %2\n\tv_ashrrev_i32 %1, 31, %1" : "+v"(v[j]), "=&v"(t) : "v"(w));
          v[j] &= t;
        }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= v[j];
  out[blockIdx.x * 1024 + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE>
void run(const char* name, uint32_t* d, unsigned long long* dc) {
  const uint32_t iters = 2048, cus = 256;
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, d, dc, iters, 0x1ff00u);
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, d, dc, iters, 0x1ff00u);
  (void)hipDeviceSynchronize();
  unsigned long long h[256 * 16];
  (void)hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
  double sum = 0;
  for (uint32_t i = 0; i < cus * 16; ++i) sum += (double)h[i];
  const double per_wave = 16.0 * iters * (MODE >= 24 ? (MODE == 26 ? 3 : 2) : 1);  // instructions per wave
  printf("%-34s %.3f wave-instr/CU-cycle\n", name, 16.0 * per_wave / (sum / (cus * 16)));
}

int main() {
  uint32_t* d;
  unsigned long long* dc;
  (void)hipMalloc(&d, 256 * 1024 * 4);
  (void)hipMalloc(&dc, 256 * 16 * 8);
  run<0>("v_add_u32 (VOP2 v,v)", d, dc);
  run<1>("v_lshlrev_b32 e64 (v, const 1)", d, dc);
  run<2>("v_lshlrev_b32 e32 (v, v)", d, dc);
  run<3>("v_and_or_b32 (v, s, v)", d, dc);
  run<4>("v_lshl_or_b32 (v, const, v)", d, dc);
  run<5>("v_bfe_u32 (v, const, const)", d, dc);
  run<6>("v_bfi_b32 (s, v, v)", d, dc);
  run<7>("v_cndmask_b32 e32 (0, v, vcc)", d, dc);
  run<8>("v_min_u32 (VOP2 v,v)", d, dc);
  run<9>("v_add3_u32 (v, v, v)", d, dc);
  run<10>("v_cndmask_b32 e32 (v, v, vcc)", d, dc);
  run<11>("v_cndmask_b32 e64 (0, v, s[])", d, dc);
  run<12>("v_cmp_gt_u32 e32 -> vcc", d, dc);
  run<13>("v_mul_u32_u24", d, dc);
  run<14>("v_mul_hi_u32", d, dc);
  run<15>("v_perm_b32", d, dc);
  run<16>("v_alignbit_b32", d, dc);
  run<17>("v_sub_u32", d, dc);
  run<18>("v_xor_b32", d, dc);
  run<19>("v_or_b32", d, dc);
  run<20>("v_mov_b32", d, dc);
  run<21>("v_cvt_f32_u32", d, dc);
  run<22>("v_mul_f32", d, dc);
  run<23>("v_ashrrev_i32 (const)", d, dc);
  run<24>("cmp_e32 + cndmask_e32 (vcc) pair", d, dc);
  run<25>("cmp_e64 + cndmask_e64 (s[]) pair", d, dc);
  run<26>("sub + ashr (+ and) mask", d, dc);
  (void)hipFree(d);
  (void)hipFree(dc);
  return 0;
}

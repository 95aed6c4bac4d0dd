// lds_hi_bench.hip -- LDS read throughput by address range on gfx950
// (profiling aid): one 1024-thread workgroup per CU with ~155 KiB of LDS;
// every lane reads ds_read_b128 / ds_read_b32 at lane-consecutive addresses
// inside a 4 KiB window placed at byte offset `base`. In-kernel s_memtime.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint32_t kWords = 155 * 1024 / 4;

template <int MODE>
__global__ __launch_bounds__(1024) void k(uint32_t* out, unsigned long long* cyc, uint32_t base, uint32_t iters) {
  __shared__ uint4 lds[kWords / 4];
  uint32_t* w = reinterpret_cast<uint32_t*>(lds);
  for (uint32_t i = threadIdx.x; i < kWords; i += 1024) w[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t o = (it * 64 + lane) & 255;  // 256 blocks of 16 B = a 4 KiB window
    if (MODE == 0) {
      const uint4 v = lds[base / 16 + o];
      acc += v.x ^ v.y ^ v.z ^ v.w;
    } else {
      acc += w[base / 4 + ((it * 64 + lane) & 1023)];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE>
void run(const char* name, uint32_t base, uint32_t* d, unsigned long long* dc) {
  const uint32_t iters = 4096, cus = 256;
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, d, dc, base, iters);
  hipLaunchKernelGGL(k<MODE>, dim3(cus), dim3(1024), 0, 0, d, dc, base, iters);
  (void)hipDeviceSynchronize();
  unsigned long long h[256 * 16];
  (void)hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
  unsigned long long mx = 0;
  for (uint32_t i = 0; i < cus * 16; ++i) mx = h[i] > mx ? h[i] : mx;
  printf("%-10s base=%6u KiB: %.2f cycles per wave-instruction per CU\n", name, base / 1024,
         (double)mx / (16.0 * iters));
}

int main() {
  uint32_t* d;
  unsigned long long* dc;
  (void)hipMalloc(&d, 256 * 1024 * 4);
  (void)hipMalloc(&dc, 256 * 16 * 8);
  for (uint32_t base : {0u, 64u * 1024, 120u * 1024, 128u * 1024, 136u * 1024, 148u * 1024}) {
    run<0>("read_b128", base, d, dc);
    run<1>("read_b32", base, d, dc);
  }
  (void)hipFree(d);
  (void)hipFree(dc);
  return 0;
}

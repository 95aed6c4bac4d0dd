// LDS marking-rate microbenchmark for gfx950 (MI355X).
// Measures lane-marks per clock per CU for the LDS write/atomic forms a sieve
// could use, under the address patterns the sieve produces:
//   mode 0: ds_or_b32, lane-distinct banks (transposed sub-segment layout)
//   mode 1: ds_or_b32, pseudo-random words (one prime per lane)
//   mode 2: ds_or_b32, stride-p bits across lanes (one prime per wave), p=param
//   mode 3: ds_or_b32, all lanes same word
//   mode 4: ds_write_b32, lane-distinct banks
//   mode 5: ds_write_b32, pseudo-random
//   mode 6: ds_write_b8 (byte map), lane-distinct banks
//   mode 7: ds_write_b8, pseudo-random
//   mode 8: ds_or_b32, per-lane own sub-segment, own stride p (real sieve walk)
// Build: hipcc --offload-arch=gfx950 -O3 lds_mark_bench.hip -o lds_mark_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int WORDS = 16384;   // 64 KiB of LDS per workgroup
constexpr int ITER = 4096;

template <int MODE>
__global__ __launch_bounds__(512) void bench(unsigned* out, unsigned param) {
  __shared__ unsigned lds[WORDS];
  const unsigned tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (unsigned i = tid; i < WORDS; i += blockDim.x) lds[i] = 0;
  __syncthreads();
  unsigned x = tid * 2654435761u + blockIdx.x * 40503u + 1u;
  unsigned off = (lane * 977u + wave * 131u) & 16383u;  // bit offset in a 16384-bit sub-segment
  const unsigned p = param | 1u;
#pragma unroll 8
  for (int i = 0; i < ITER; ++i) {
    if constexpr (MODE == 0) {
      unsigned w = ((i * 8 + wave) * 64 + lane) & (WORDS - 1);
      __hip_atomic_fetch_or(&lds[w], 1u << (i & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (MODE == 1) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      __hip_atomic_fetch_or(&lds[x & (WORDS - 1)], 1u << (x >> 27), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (MODE == 2) {
      unsigned b = (i * 7919u + wave * 104729u + lane * p) & (WORDS * 32 - 1);
      __hip_atomic_fetch_or(&lds[b >> 5], 1u << (b & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (MODE == 3) {
      __hip_atomic_fetch_or(&lds[(i * 8 + wave) & (WORDS - 1)], 1u << (lane & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (MODE == 4) {
      unsigned w = ((i * 8 + wave) * 64 + lane) & (WORDS - 1);
      lds[w] = i;
    } else if constexpr (MODE == 5) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      lds[x & (WORDS - 1)] = i;
    } else if constexpr (MODE == 6) {
      unsigned w = ((i * 8 + wave) * 64 + lane) & (WORDS - 1);
      reinterpret_cast<unsigned char*>(lds)[w * 4 + (i & 3)] = 1;
    } else if constexpr (MODE == 7) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      reinterpret_cast<unsigned char*>(lds)[x & (WORDS * 4 - 1)] = 1;
    } else if constexpr (MODE == 8) {
      // lane-owned column (64 columns interleaved word-wise), walk with stride p in bits
      unsigned row = off >> 5;  // 0..511 rows of 64 words = 32768 words -> use 256 rows here
      unsigned w = ((row & 255) * 64 + lane);
      __hip_atomic_fetch_or(&lds[w & (WORDS - 1)], 1u << (off & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      off += p; off = off >= 8192u ? off - 8192u : off;
    }
  }
  __syncthreads();
  unsigned acc = 0;
  for (unsigned i = tid; i < WORDS; i += blockDim.x) acc += lds[i];
  atomicAdd(out, acc);
}

template <int MODE>
double run(unsigned* d_out, unsigned param, int blocks, int threads) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  bench<MODE><<<blocks, threads>>>(d_out, param);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) bench<MODE><<<blocks, threads>>>(d_out, param);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  double ops = 5.0 * blocks * threads * (double)ITER;
  double per_cu_clk = ops / (ms * 1e-3) / 256.0 / 2.4e9;
  return per_cu_clk;
}

int main() {
  unsigned* d_out; CHECK(hipMalloc(&d_out, 4));
  const int blocks = 256 * 2 * 4, threads = 512;
  printf("mode0 or  lane-banks   : %.2f lane-marks/clk/CU\n", run<0>(d_out, 0, blocks, threads));
  printf("mode1 or  random       : %.2f\n", run<1>(d_out, 0, blocks, threads));
  unsigned ps[] = {65, 97, 129, 257, 1025, 3001, 12289, 65537};
  for (unsigned p : ps) printf("mode2 or  stride p=%-6u: %.2f\n", p, run<2>(d_out, p, blocks, threads));
  printf("mode3 or  same word    : %.2f\n", run<3>(d_out, 0, blocks, threads));
  printf("mode4 w32 lane-banks   : %.2f\n", run<4>(d_out, 0, blocks, threads));
  printf("mode5 w32 random       : %.2f\n", run<5>(d_out, 0, blocks, threads));
  printf("mode6 w8  lane-banks   : %.2f\n", run<6>(d_out, 0, blocks, threads));
  printf("mode7 w8  random       : %.2f\n", run<7>(d_out, 0, blocks, threads));
  unsigned ps8[] = {67, 331, 1031, 4099};
  for (unsigned p : ps8) printf("mode8 or  lane-walk p=%-5u: %.2f\n", p, run<8>(d_out, p, blocks, threads));
  return 0;
}

#!/usr/bin/env python3
"""Build a timing-instrumented copy of the wheel kernel sources (profiling only;
the shipping sources carry no timing code).

  python tools/instrument_timing.py ROOT

copies distributed-sieve-e_amd/csrc/* (and include/dse.h) under ROOT and inserts s_memtime
stamps into dse_wheel.hip: per wave, the cycles of mark / mark barrier /
expand / init / segment barrier and, with the LDS drained after every unit,
of the A, B1, B2, L and bucket units, summed into a per-TU __device__ array
and read by an extra C entry point dse_debug_timing(unsigned long long[16]).
Then `SRC_DIR=ROOT/distributed-sieve-e_amd/csrc bash tools/build_variant.sh timing` builds
variants/libdse_timing.so, and tools/wave_timing.py reads it. Draining per
unit serialises the marking a little, so the unit split is an attribution,
not the production timing.
"""
import os
import shutil
import sys

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-sieve-e_amd", "csrc")


def sub(s, old, new, count=1):
    if s.count(old) != count:
        sys.exit(f"instrument_timing: anchor found {s.count(old)} times, expected {count}: {old[:70]!r}")
    return s.replace(old, new)


def main(root):
    out = os.path.join(root, "distributed-sieve-e_amd", "csrc")  # the tree layout dse_host.cpp includes from
    os.makedirs(out, exist_ok=True)
    os.makedirs(os.path.join(root, "include"), exist_ok=True)
    shutil.copy(os.path.join(SRC, "..", "..", "include", "dse.h"), os.path.join(root, "include", "dse.h"))
    for f in os.listdir(SRC):
        if f.endswith((".hip", ".cpp", ".h")) or f == "Makefile":
            shutil.copy(os.path.join(SRC, f), os.path.join(out, f))
    p = os.path.join(out, "dse_wheel.hip")
    s = open(p).read()
    s = sub(s, "namespace dse {\nnamespace {\n",
            "namespace dse {\nnamespace {\n__device__ unsigned long long g_timing[16];\n"
            "__device__ unsigned long long g_timing_w[16 * 5];  // per wave id: the 5 phases\n")
    s = sub(s, "  const uint32_t tid = threadIdx.x, lane_id = tid & 63, wave = tid >> 6;\n",
            "  const uint32_t tid = threadIdx.x, lane_id = tid & 63, wave = tid >> 6;\n"
            "  uint64_t t_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, t_prev = 0;\n"
            "#define DSE_TSTAMP(i) do { const uint64_t t_now = __builtin_amdgcn_s_memtime();"
            " if ((i) >= 0) t_acc[i] += t_now - t_prev; t_prev = t_now; } while (0)\n")
    # unit attribution (LDS drained after each unit)
    s = sub(s, "      const uint32_t k = d_cur & kIdx;\n      if ((d_cur >> 30) == 0) {\n",
            "      const uint32_t k = d_cur & kIdx;\n"
            "      const uint64_t t_u0 = __builtin_amdgcn_s_memtime();\n"
            "      const uint32_t u_type = (d_cur >> 30) == 0 ? (k < nA ? 5u : k < nA + nB1 ? 6u : 7u) : 8u;\n"
            "      if ((d_cur >> 30) == 0) {\n")
    s = sub(s, "      }\n      d_after = decode(claimed(c2));\n    }\n  };",
            "      }\n      lds_drain();\n      t_acc[u_type] += __builtin_amdgcn_s_memtime() - t_u0;\n"
            "      d_after = decode(claimed(c2));\n    }\n  };")
    s = sub(s, "      if (BK && (d_cur >> 30) == 2) {  // a bucket unit, kBkBatchU loads in flight per lane\n",
            "      if (BK && (d_cur >> 30) == 2) {  // a bucket unit, kBkBatchU loads in flight per lane\n"
            "        const uint64_t t_b0 = __builtin_amdgcn_s_memtime();\n")
    s = sub(s, "        d_after = decode(claimed(c2));\n        continue;",
            "        lds_drain();\n        t_acc[9] += __builtin_amdgcn_s_memtime() - t_b0;\n"
            "        d_after = decode(claimed(c2));\n        continue;")
    # phases of the segment loop
    s = sub(s, "  if (T > 0) init_segment(lds.img, blockIdx.x);\n  __syncthreads();\n",
            "  if (T > 0) init_segment(lds.img, blockIdx.x);\n  __syncthreads();\n  DSE_TSTAMP(-1);\n")
    s = sub(s, "    mark_segment(lds.img, s);\n    lds_drain();\n    __syncthreads();\n    expand_segment(lds.img, s);\n",
            "    mark_segment(lds.img, s);\n    lds_drain();\n    DSE_TSTAMP(0);\n    __syncthreads();\n"
            "    DSE_TSTAMP(1);\n    expand_segment(lds.img, s);\n    DSE_TSTAMP(2);\n")
    s = sub(s, "    if (t + 1 < T) init_segment(lds.img, s + grid);\n    if (tid == 0) {\n",
            "    if (t + 1 < T) init_segment(lds.img, s + grid);\n    DSE_TSTAMP(3);\n    if (tid == 0) {\n")
    s = sub(s, "    __syncthreads();\n  }\n\n  if (tid < wa.nranges && lds.rcnt[tid])",
            "    __syncthreads();\n    DSE_TSTAMP(4);\n  }\n"
            "  if (lane_id == 0)\n    for (int i = 0; i < 10; ++i) atomicAdd(&g_timing[i], (unsigned long long)t_acc[i]);\n"
            "  if (lane_id == 0)\n    for (int i = 0; i < 5; ++i) atomicAdd(&g_timing_w[wave * 5 + i], (unsigned long long)t_acc[i]);\n\n"
            "  if (tid < wa.nranges && lds.rcnt[tid])")
    s = sub(s, "}  // namespace dse\n", """#if DSE_WHEEL_PLAIN_TU
int timing_take_plain(unsigned long long* acc) {
#elif DSE_WHEEL_HALF_TU
int timing_take_half(unsigned long long* acc) {
#else
int timing_take_plain(unsigned long long* acc);
int timing_take_half(unsigned long long* acc);
int timing_take_main(unsigned long long* acc) {
#endif
  unsigned long long t[16], tw[80];
  if (hipMemcpyFromSymbol(t, HIP_SYMBOL(g_timing), sizeof(t)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(tw, HIP_SYMBOL(g_timing_w), sizeof(tw)) != hipSuccess) return -1;
  for (int i = 0; i < 16; ++i) acc[i] += t[i];
  for (int i = 0; i < 80; ++i) acc[16 + i] += tw[i];
  const unsigned long long z[80] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_timing_w), z, sizeof(tw)) != hipSuccess) return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_timing), z, sizeof(t)) == hipSuccess ? 0 : -1;
}
#if DSE_WHEEL_MAIN_TU
// out[0..16): phase and unit sums over all waves; out[16 + 5 w + i]: phase i
// (mark, mark barrier, expand, init, segment barrier) of the waves with id w
extern "C" int dse_debug_timing(unsigned long long* out) {
  for (int i = 0; i < 96; ++i) out[i] = 0;
  return (timing_take_main(out) || timing_take_plain(out) || timing_take_half(out)) ? -1 : 0;
}
#endif
}  // namespace dse
""")
    open(p, "w").write(s)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/dse_timing_src")

// dse_host.cpp -- C-ABI host layer of libdse.so (include/dse.h).
//
// Replaces the reference's orchestration of the hot path:
//   spread-work (sieve.clj:15-34)            -> dse_spread_work (exact int64)
//   gen-table + sieve-e (sieve.clj:9-172)    -> dse_sieve_chunk / dse_sieve_all
//   per-prime [mi ps p] relay through the
//     lead (sieve.clj:139, core.clj:118-134) -> one RCCL broadcast of base primes
//   (no result gather in the reference)      -> RCCL all-reduce of counts
//   finish (sieve.clj:82-108)                -> dse_write_primes_file
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dse.h"
#include "dse_internal.h"

namespace {

thread_local std::string g_err;
thread_local int32_t g_code = DSE_OK;

int32_t fail(int32_t code, const std::string& msg) {
  g_err = msg;
  g_code = code;
  return code;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(DSE_EHIP, std::string(#expr " failed: ") + hipGetErrorString(e_));      \
  } while (0)

#define NCCL_TRY(expr)                                                                    \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess)                                                                \
      return fail(DSE_ENCCL, std::string(#expr " failed: ") + ncclGetErrorString(r_));    \
  } while (0)

uint64_t isqrt_u64(uint64_t x) {
  uint64_t r = (uint64_t)std::sqrt((long double)x);
  while (r > 0 && r * r > x) --r;
  while ((r + 1) * (r + 1) <= x) ++r;
  return r;
}

// Upper bound on the number of odd primes <= x (Rosser-Schoenfeld
// pi(x) < 1.25506 x / ln x for x > 1), padded.
uint32_t prime_cap(uint64_t x) {
  if (x < 100) return 64;
  double b = 1.25506 * (double)x / std::log((double)x);
  return (uint32_t)b + 64;
}

struct ChunkMask {
  int32_t my_num = 0;
  uint64_t* dev_ptr = nullptr;
  uint64_t words = 0;
};

struct DevState {
  int device = 0;
  int num_cus = 0;
  hipStream_t stream = nullptr;
  void* table = nullptr;
  uint64_t table_bytes = 0;
  unsigned long long* counts = nullptr;  // device scratch
  uint64_t counts_len = 0;
  uint64_t* scratch_mask = nullptr;      // for dse_sieve_chunk
  uint64_t scratch_words = 0;
  std::vector<ChunkMask> resident;       // masks kept by dse_sieve_all
  dse::Scratch scratch;                  // bucketed-pass scratch (high-offset ranges)
  hipEvent_t xev = nullptr;              // logical devices: this device's side of a collective
};

}  // namespace

struct dse_ctx {
  std::vector<DevState> devs;
  std::vector<ncclComm_t> comms;
  int64_t last_n = -1;
  int32_t last_P = 0;
  dse::SieveOpts opts;  // test-only knobs (dse_debug_set_option)
  // dse_debug_init_logical: every DevState on device 0, the collectives
  // replaced by copies (xfer_table / allreduce_counts); on device 0:
  bool logical = false;
  // dse_debug_set_option("rccl_single"): a one-device context with a 1-rank
  // RCCL communicator, so share_table / allreduce_counts issue the real
  // grouped ncclBroadcast / ncclAllReduce on a one-GPU box.
  bool rccl_single = false;
  int64_t rccl_calls = 0;                  // collectives RCCL accepted (dse_debug_get_stat)
  int64_t table_local_builds = 0;          // tables built per device instead of broadcast (share_table)
  unsigned long long* lg_stage = nullptr;  // gathered counts [devs][n]
  unsigned long long* lg_sum = nullptr;    // their sum [n]
  uint64_t lg_n = 0;                       // n of the two buffers
  hipEvent_t lg_done = nullptr;            // the sum on device 0's stream
};

namespace {

int32_t ensure_table(DevState& d, uint64_t limit) {
  const uint64_t need = dse_base_table_bytes(limit);
  if (d.table_bytes < need) {
    if (d.table) HIP_TRY(hipFree(d.table));
    d.table = nullptr;
    d.table_bytes = 0;
    HIP_TRY(hipMalloc(&d.table, need));
    d.table_bytes = need;
  }
  return DSE_OK;
}

int32_t ensure_counts(DevState& d, uint64_t n) {
  if (d.counts_len < n) {
    if (d.counts) HIP_TRY(hipFree(d.counts));
    d.counts = nullptr;
    d.counts_len = 0;
    HIP_TRY(hipMalloc(&d.counts, n * sizeof(unsigned long long)));
    d.counts_len = n;
  }
  return DSE_OK;
}

int32_t build_table(DevState& d, uint64_t limit) {
  if (limit > dse::kBigBaseLimitMax)
    return fail(DSE_ERANGE, "base-prime limit " + std::to_string(limit) + " above the supported " +
                                std::to_string(dse::kBigBaseLimitMax));
  int32_t rc = ensure_table(d, limit);
  if (rc) return rc;
  HIP_TRY(dse::launch_base_primes_big(limit, d.table, prime_cap(limit), d.num_cus, d.stream));
  return DSE_OK;
}

// Enqueue a copy of the sticky bucket-overflow flag on d.stream (before the
// caller's stream sync); check_flag after the sync reports and clears it.
// d.stream first waits for the last bucketed pass on the context's scratch,
// whatever stream it ran on (an async pass on a user stream may still be
// running: its overflow must neither be reported as this call's nor be
// cleared before it is written).
int32_t fetch_flag(DevState& d, uint32_t* h) {
  *h = 0;
  if (!d.scratch.flag) return DSE_OK;
  if (d.scratch.used) HIP_TRY(hipStreamWaitEvent(d.stream, d.scratch.done, 0));
  HIP_TRY(hipMemcpyAsync(h, d.scratch.flag, sizeof(uint32_t), hipMemcpyDeviceToHost, d.stream));
  return DSE_OK;
}

int32_t check_flag(DevState& d, uint32_t h) {
  if (!h) return DSE_OK;
  HIP_TRY(hipMemsetAsync(d.scratch.flag, 0, sizeof(uint32_t), d.stream));
  HIP_TRY(hipStreamSynchronize(d.stream));
  return fail(DSE_EINTERNAL, "bucketed pass exceeded its entry capacity on device " + std::to_string(d.device) +
                                 "; the count and mask of this call are not valid");
}

int32_t free_resident(DevState& d) {
  for (auto& c : d.resident)
    if (c.dev_ptr) HIP_TRY(hipFree(c.dev_ptr));
  d.resident.clear();
  return DSE_OK;
}

int32_t chunk_geometry(int64_t n, int32_t P, int64_t* cs) {
  if (P < 1) return fail(DSE_EINVAL, "num-comps must be >= 1");
  if (n < 0) return fail(DSE_EINVAL, "n must be >= 0");
  int64_t nums = n >= 1 ? (n - 1) / 2 : 0;
  *cs = nums / P;
  return DSE_OK;
}

int32_t init_dev(DevState& d, int device) {
  d.device = device;
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  d.num_cus = prop.multiProcessorCount;
  HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  return DSE_OK;
}

// Base primes once, on device 0, then an RCCL broadcast of the primes (the
// table's header + p[]) to the other devices, which derive their Barrett
// factors and wheel offsets locally: the reference's prime broadcast
// (sieve.clj:139, core.clj:94-95,126) done once. Every device's table buffer
// must already hold dse_base_table_bytes(limit) bytes.
// A table whose primes exceed the broadcast cap (dse_base_table_broadcast_bytes:
// the window's 203 MB) is built on every device instead, each on its own
// stream: 0.2 ms of local work against 0.7-2 ms of broadcast (DESIGN.md
// section 5). The test option table_broadcast_max_bytes moves the cap.
int32_t share_table(dse_ctx* ctx, uint64_t limit) {
  int32_t rc;
  const int nd = (int)ctx->devs.size();
  const uint64_t pbytes = dse_base_table_prime_bytes(limit);
  const uint64_t cap = ctx->opts.table_bcast_max ? ctx->opts.table_bcast_max : DSE_TABLE_BROADCAST_MAX_BYTES;
  if ((nd > 1 || ctx->rccl_single) && pbytes > cap) {
    for (int i = 0; i < nd; ++i) {
      HIP_TRY(hipSetDevice(ctx->devs[i].device));
      if ((rc = build_table(ctx->devs[i], limit))) return rc;
    }
    ctx->table_local_builds += nd;
    return DSE_OK;
  }
  HIP_TRY(hipSetDevice(ctx->devs[0].device));
  if ((rc = build_table(ctx->devs[0], limit))) return rc;
  if (nd == 1 && !ctx->rccl_single) return DSE_OK;
  if (ctx->logical) {  // the broadcast as copies from device 0's table, each on its device's stream
    DevState& r = ctx->devs[0];
    HIP_TRY(hipEventRecord(r.xev, r.stream));
    for (int i = 1; i < nd; ++i) {
      DevState& d = ctx->devs[i];
      HIP_TRY(hipStreamWaitEvent(d.stream, r.xev, 0));
      HIP_TRY(hipMemcpyAsync(d.table, r.table, pbytes, hipMemcpyDeviceToDevice, d.stream));
      HIP_TRY(dse::launch_wheel_offsets(d.table, d.num_cus, d.stream, prime_cap(limit)));
    }
    return DSE_OK;
  }
  NCCL_TRY(ncclGroupStart());
  for (int i = 0; i < nd; ++i) {
    DevState& d = ctx->devs[i];
    NCCL_TRY(ncclBroadcast(ctx->devs[0].table, d.table, pbytes, ncclUint8, 0, ctx->comms[i], d.stream));
  }
  NCCL_TRY(ncclGroupEnd());
  ctx->rccl_calls += nd;
  for (int i = 1; i < nd; ++i) {
    DevState& d = ctx->devs[i];
    HIP_TRY(hipSetDevice(d.device));
    HIP_TRY(dse::launch_wheel_offsets(d.table, d.num_cus, d.stream, prime_cap(limit)));
  }
  return DSE_OK;
}

// Sum `n` uint64 counts over the devices with an RCCL all-reduce (in place).
int32_t allreduce_counts(dse_ctx* ctx, uint64_t n) {
  if (ctx->devs.size() < 2 && !ctx->rccl_single) return DSE_OK;
  if (ctx->logical) {  // gather + sum on device 0's stream, then every device copies the sum back
    const uint32_t nd = (uint32_t)ctx->devs.size();
    DevState& r = ctx->devs[0];
    HIP_TRY(hipSetDevice(r.device));
    if (ctx->lg_n < n) {
      if (ctx->lg_stage) HIP_TRY(hipFree(ctx->lg_stage));
      if (ctx->lg_sum) HIP_TRY(hipFree(ctx->lg_sum));
      ctx->lg_stage = ctx->lg_sum = nullptr;
      ctx->lg_n = 0;
      HIP_TRY(hipMalloc(&ctx->lg_stage, nd * n * sizeof(unsigned long long)));
      HIP_TRY(hipMalloc(&ctx->lg_sum, n * sizeof(unsigned long long)));
      ctx->lg_n = n;
    }
    for (uint32_t i = 0; i < nd; ++i) {
      DevState& d = ctx->devs[i];
      if (i) {
        HIP_TRY(hipEventRecord(d.xev, d.stream));
        HIP_TRY(hipStreamWaitEvent(r.stream, d.xev, 0));
      }
      HIP_TRY(hipMemcpyAsync(ctx->lg_stage + i * n, d.counts, n * sizeof(unsigned long long),
                             hipMemcpyDeviceToDevice, r.stream));
    }
    HIP_TRY(dse::launch_sum_rows(ctx->lg_stage, nd, (uint32_t)n, ctx->lg_sum, r.stream));
    HIP_TRY(hipEventRecord(ctx->lg_done, r.stream));
    for (uint32_t i = 0; i < nd; ++i) {
      DevState& d = ctx->devs[i];
      if (i) HIP_TRY(hipStreamWaitEvent(d.stream, ctx->lg_done, 0));
      HIP_TRY(hipMemcpyAsync(d.counts, ctx->lg_sum, n * sizeof(unsigned long long), hipMemcpyDeviceToDevice,
                             d.stream));
    }
    return DSE_OK;
  }
  NCCL_TRY(ncclGroupStart());
  for (size_t i = 0; i < ctx->devs.size(); ++i) {
    DevState& d = ctx->devs[i];
    NCCL_TRY(ncclAllReduce(d.counts, d.counts, n, ncclUint64, ncclSum, ctx->comms[i], d.stream));
  }
  NCCL_TRY(ncclGroupEnd());
  ctx->rccl_calls += (int64_t)ctx->devs.size();
  return DSE_OK;
}

}  // namespace

extern "C" {

const char* dse_version(void) { return "dse 0.1 gfx950"; }

const char* dse_last_error(void) { return g_err.c_str(); }

int32_t dse_last_status(void) { return g_code; }

int32_t dse_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

dse_ctx* dse_init(int32_t num_gpus) {
  g_err.clear();
  g_code = DSE_OK;
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || avail < 1) {
    fail(DSE_EHIP, "no HIP device visible");
    return nullptr;
  }
  if (num_gpus <= 0) num_gpus = avail;
  if (num_gpus > avail) {
    fail(DSE_EINVAL, "asked for " + std::to_string(num_gpus) + " GPUs, " + std::to_string(avail) + " visible");
    return nullptr;
  }
  dse_ctx* ctx = new dse_ctx();
  ctx->devs.resize(num_gpus);
  for (int i = 0; i < num_gpus; ++i)
    if (init_dev(ctx->devs[i], i) != DSE_OK) {
      dse_destroy(ctx);
      return nullptr;
    }
  if (num_gpus > 1) {
    ctx->comms.resize(num_gpus);
    std::vector<int> ids(num_gpus);
    for (int i = 0; i < num_gpus; ++i) ids[i] = i;
    ncclResult_t r = ncclCommInitAll(ctx->comms.data(), num_gpus, ids.data());
    if (r != ncclSuccess) {
      fail(DSE_ENCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
      ctx->comms.clear();
      dse_destroy(ctx);
      return nullptr;
    }
  }
  return ctx;
}

dse_ctx* dse_init_device(int32_t device) {
  g_err.clear();
  g_code = DSE_OK;
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || device < 0 || device >= avail) {
    fail(DSE_EINVAL, "device " + std::to_string(device) + " not visible");
    return nullptr;
  }
  dse_ctx* ctx = new dse_ctx();
  ctx->devs.resize(1);
  if (init_dev(ctx->devs[0], device) != DSE_OK) {
    dse_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

void dse_destroy(dse_ctx* ctx) {
  if (!ctx) return;
  for (auto& c : ctx->comms) ncclCommDestroy(c);
  if (ctx->logical && !ctx->devs.empty()) {
    (void)hipSetDevice(ctx->devs[0].device);
    if (ctx->lg_stage) (void)hipFree(ctx->lg_stage);
    if (ctx->lg_sum) (void)hipFree(ctx->lg_sum);
    if (ctx->lg_done) (void)hipEventDestroy(ctx->lg_done);
  }
  for (auto& d : ctx->devs) {
    (void)hipSetDevice(d.device);
    free_resident(d);
    if (d.table) (void)hipFree(d.table);
    if (d.counts) (void)hipFree(d.counts);
    if (d.scratch_mask) (void)hipFree(d.scratch_mask);
    (void)dse::free_scratch(&d.scratch);
    if (d.xev) (void)hipEventDestroy(d.xev);
    if (d.stream) (void)hipStreamDestroy(d.stream);
  }
  delete ctx;
}

dse_ctx* dse_debug_init_logical(int32_t num_logical) {
  g_err.clear();
  g_code = DSE_OK;
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || avail < 1) {
    fail(DSE_EHIP, "no HIP device visible");
    return nullptr;
  }
  if (num_logical < 1 || num_logical > 64) {
    fail(DSE_EINVAL, "num_logical must be in 1..64");
    return nullptr;
  }
  dse_ctx* ctx = new dse_ctx();
  ctx->logical = true;
  ctx->devs.resize(num_logical);
  for (int i = 0; i < num_logical; ++i) {
    DevState& d = ctx->devs[i];
    if (init_dev(d, 0) != DSE_OK || hipEventCreateWithFlags(&d.xev, hipEventDisableTiming) != hipSuccess) {
      if (!g_code) fail(DSE_EHIP, "event creation failed");
      dse_destroy(ctx);
      return nullptr;
    }
  }
  if (hipEventCreateWithFlags(&ctx->lg_done, hipEventDisableTiming) != hipSuccess) {
    fail(DSE_EHIP, "event creation failed");
    dse_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

int32_t dse_ctx_num_devices(const dse_ctx* ctx) { return ctx ? (int32_t)ctx->devs.size() : 0; }

int32_t dse_spread_work(int64_t n, int32_t P, int64_t* lo_hi, int64_t* cs) {
  int64_t c;
  int32_t rc = chunk_geometry(n, P, &c);
  if (rc) return rc;
  if (cs) *cs = c;
  if (lo_hi)
    for (int32_t k = 1; k <= P; ++k) {
      lo_hi[2 * (k - 1)] = 3 + 2 * (int64_t)(k - 1) * c;
      lo_hi[2 * (k - 1) + 1] = 3 + 2 * (int64_t)k * c;
    }
  return DSE_OK;
}

int32_t dse_tail_range(int64_t n, int32_t P, uint64_t* g_start, uint64_t* nbits) {
  int64_t cs;
  int32_t rc = chunk_geometry(n, P, &cs);
  if (rc) return rc;
  int64_t nums = n >= 1 ? (n - 1) / 2 : 0;
  if (g_start) *g_start = (uint64_t)(P * cs);
  if (nbits) *nbits = (uint64_t)(nums - P * cs);
  return DSE_OK;
}

uint64_t dse_base_table_bytes(uint64_t limit) { return dse::table_bytes_for_cap(prime_cap(limit)); }

uint64_t dse_base_limit_max(void) { return dse::kBigBaseLimitMax; }

uint64_t dse_base_limit_for_range(uint64_t g_start, uint64_t nbits) {
  if (nbits == 0) return 0;
  const uint64_t vmax = 3 + 2 * (g_start + nbits - 1);
  return isqrt_u64(vmax);
}

int32_t dse_base_primes_dev_async(dse_ctx* ctx, uint64_t limit, void* table_dev, uint64_t table_bytes,
                                  void* stream) {
  if (!ctx || !table_dev) return fail(DSE_EINVAL, "null ctx or table");
  if (table_bytes < dse_base_table_bytes(limit)) return fail(DSE_EINVAL, "table buffer too small");
  if (limit > dse::kBigBaseLimitMax) return fail(DSE_ERANGE, "base-prime limit above the supported maximum");
  HIP_TRY(hipSetDevice(ctx->devs[0].device));
  HIP_TRY(dse::launch_base_primes_big(limit, table_dev, prime_cap(limit), ctx->devs[0].num_cus,
                                      (hipStream_t)stream));
  return DSE_OK;
}

uint64_t dse_base_table_prime_bytes(uint64_t limit) { return 16ull + 4ull * prime_cap(limit); }

uint64_t dse_base_table_broadcast_bytes(uint64_t limit) {
  const uint64_t pbytes = dse_base_table_prime_bytes(limit);
  return pbytes <= DSE_TABLE_BROADCAST_MAX_BYTES ? pbytes : 0;
}

int32_t dse_base_table_finish_dev_async(dse_ctx* ctx, uint64_t limit, void* table_dev, uint64_t table_bytes,
                                        void* stream) {
  if (!ctx || !table_dev) return fail(DSE_EINVAL, "null ctx or table");
  if (table_bytes < dse_base_table_bytes(limit)) return fail(DSE_EINVAL, "table buffer too small");
  if (limit > dse::kBigBaseLimitMax) return fail(DSE_ERANGE, "base-prime limit above the supported maximum");
  HIP_TRY(hipSetDevice(ctx->devs[0].device));
  HIP_TRY(dse::launch_wheel_offsets(table_dev, ctx->devs[0].num_cus, (hipStream_t)stream, prime_cap(limit)));
  return DSE_OK;
}

int32_t dse_sieve_range_dev_async(dse_ctx* ctx, const void* table_dev, uint64_t g_start, uint64_t nbits,
                                  uint64_t* mask_dev, uint64_t* count_dev, void* stream) {
  if (!ctx || !table_dev || !count_dev) return fail(DSE_EINVAL, "null ctx, table or count");
  if (g_start > (1ull << 62) || nbits > (1ull << 62) - g_start)
    return fail(DSE_ERANGE, "odd-index range beyond 2^62");
  HIP_TRY(hipSetDevice(ctx->devs[0].device));
  HIP_TRY(dse::launch_sieve_range(table_dev, g_start, nbits, reinterpret_cast<uint32_t*>(mask_dev),
                                  reinterpret_cast<unsigned long long*>(count_dev), ctx->devs[0].num_cus,
                                  (hipStream_t)stream, &ctx->devs[0].scratch, &ctx->opts));
  return DSE_OK;
}

namespace {
int32_t sieve_range_host(dse_ctx* ctx, DevState& d, uint64_t g0, uint64_t nbits, uint64_t* mask_or_null,
                         uint64_t* count) {
  int32_t rc;
  HIP_TRY(hipSetDevice(d.device));
  const uint64_t words = (nbits + 63) / 64;
  if ((rc = build_table(d, dse_base_limit_for_range(g0, nbits)))) return rc;
  if ((rc = ensure_counts(d, 1))) return rc;
  if (mask_or_null && d.scratch_words < words) {
    if (d.scratch_mask) HIP_TRY(hipFree(d.scratch_mask));
    d.scratch_mask = nullptr;
    d.scratch_words = 0;
    HIP_TRY(hipMalloc(&d.scratch_mask, words * 8));
    d.scratch_words = words;
  }
  HIP_TRY(hipMemsetAsync(d.counts, 0, sizeof(unsigned long long), d.stream));
  HIP_TRY(dse::launch_sieve_range(d.table, g0, nbits,
                                  mask_or_null ? reinterpret_cast<uint32_t*>(d.scratch_mask) : nullptr,
                                  d.counts, d.num_cus, d.stream, &d.scratch, &ctx->opts));
  unsigned long long c = 0;
  HIP_TRY(hipMemcpyAsync(&c, d.counts, sizeof(c), hipMemcpyDeviceToHost, d.stream));
  if (mask_or_null && words)
    HIP_TRY(hipMemcpyAsync(mask_or_null, d.scratch_mask, words * 8, hipMemcpyDeviceToHost, d.stream));
  uint32_t hf;
  if ((rc = fetch_flag(d, &hf))) return rc;
  HIP_TRY(hipStreamSynchronize(d.stream));
  if ((rc = check_flag(d, hf))) return rc;
  if (count) *count = c;
  return DSE_OK;
}
}  // namespace

int32_t dse_sieve_odd_range(dse_ctx* ctx, uint64_t g_start, uint64_t nbits, uint64_t* mask_or_null,
                            uint64_t* count) {
  if (!ctx) return fail(DSE_EINVAL, "null ctx");
  if (g_start > (1ull << 62) || nbits > (1ull << 62) - g_start)
    return fail(DSE_ERANGE, "odd-index range beyond 2^62");
  return sieve_range_host(ctx, ctx->devs[0], g_start, nbits, mask_or_null, count);
}

int32_t dse_sieve_chunk(dse_ctx* ctx, int64_t n, int32_t P, int32_t my_num, uint64_t* mask_or_null,
                        uint64_t* count) {
  if (!ctx) return fail(DSE_EINVAL, "null ctx");
  int64_t cs;
  int32_t rc = chunk_geometry(n, P, &cs);
  if (rc) return rc;
  if (my_num < 1 || my_num > P) return fail(DSE_EINVAL, "my_num outside 1..P");
  if (cs < 1) return fail(DSE_EINVAL, "empty chunk (find-first-prime would throw)");
  DevState& d = ctx->devs[(my_num - 1) % ctx->devs.size()];
  return sieve_range_host(ctx, d, (uint64_t)(my_num - 1) * (uint64_t)cs, (uint64_t)cs, mask_or_null, count);
}

int32_t dse_sieve_all(dse_ctx* ctx, int64_t n, int32_t P, uint64_t* per_chunk_counts, uint64_t* pi_ref,
                      uint64_t* pi_full) {
  if (!ctx) return fail(DSE_EINVAL, "null ctx");
  int64_t cs;
  int32_t rc = chunk_geometry(n, P, &cs);
  if (rc) return rc;
  if (cs < 1) return fail(DSE_EINVAL, "empty chunk (find-first-prime would throw)");
  uint64_t tail_g, tail_n;
  dse_tail_range(n, P, &tail_g, &tail_n);
  const int nd = (int)ctx->devs.size();
  const uint64_t words = ((uint64_t)cs + 63) / 64;
  // every chunk and the tail are covered by the primes <= sqrt(largest odd <= n)
  const uint64_t limit = dse_base_limit_for_range(0, (uint64_t)P * (uint64_t)cs + tail_n);
  const uint64_t nc = (uint64_t)P + 1;  // per-chunk counts + tail

  // resident masks: one device buffer per chunk, on its device
  for (int i = 0; i < nd; ++i) {
    DevState& d = ctx->devs[i];
    HIP_TRY(hipSetDevice(d.device));
    // the same (n, P) as the last call: the same chunk map and mask sizes
    const bool reuse = ctx->last_n == n && ctx->last_P == P && !d.resident.empty() && d.resident[0].words == words;
    if (!reuse) {
      if ((rc = free_resident(d))) return rc;
      for (int32_t k = i + 1; k <= P; k += nd) {
        ChunkMask cm;
        cm.my_num = k;
        cm.words = words;
        HIP_TRY(hipMalloc(&cm.dev_ptr, words * 8));
        d.resident.push_back(cm);
      }
    }
    if ((rc = ensure_table(d, limit))) return rc;
    if ((rc = ensure_counts(d, nc))) return rc;
    HIP_TRY(hipMemsetAsync(d.counts, 0, nc * sizeof(unsigned long long), d.stream));
  }
  ctx->last_n = n;
  ctx->last_P = P;

  if ((rc = share_table(ctx, limit))) return rc;

  // each device sieves its chunks; the last device also sieves the tail.
  // All of a device's ranges go to one launch_sieve_ranges call: its chunks
  // (and the tail) share persistent launches of the wheel kernel, so no
  // chunk's partial last round leaves the CUs idle and no host launch sits
  // between chunks.
  for (int i = 0; i < nd; ++i) {
    DevState& d = ctx->devs[i];
    HIP_TRY(hipSetDevice(d.device));
    std::vector<dse::RangeSpec> rs;
    for (auto& cm : d.resident)
      rs.push_back({(uint64_t)(cm.my_num - 1) * (uint64_t)cs, (uint64_t)cs, reinterpret_cast<uint32_t*>(cm.dev_ptr),
                    d.counts + (cm.my_num - 1)});
    if (i == nd - 1 && tail_n) rs.push_back({tail_g, tail_n, nullptr, d.counts + P});
    HIP_TRY(dse::launch_sieve_ranges(d.table, rs.data(), rs.size(), d.num_cus, d.stream, &d.scratch, &ctx->opts));
  }

  // counts: RCCL all-reduce (each slot is non-zero on exactly one device)
  if ((rc = allreduce_counts(ctx, nc))) return rc;
  std::vector<unsigned long long> h(nc);
  HIP_TRY(hipSetDevice(ctx->devs[0].device));
  HIP_TRY(hipMemcpyAsync(h.data(), ctx->devs[0].counts, nc * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                         ctx->devs[0].stream));
  std::vector<uint32_t> hf(nd);
  for (int i = 0; i < nd; ++i) {
    HIP_TRY(hipSetDevice(ctx->devs[i].device));
    if ((rc = fetch_flag(ctx->devs[i], &hf[i]))) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->devs[i].stream));
  }
  for (int i = 0; i < nd; ++i) {
    HIP_TRY(hipSetDevice(ctx->devs[i].device));
    if ((rc = check_flag(ctx->devs[i], hf[i]))) return rc;
  }
  uint64_t sum = 0;
  for (int32_t k = 0; k < P; ++k) {
    if (per_chunk_counts) per_chunk_counts[k] = h[k];
    sum += h[k];
  }
  if (pi_ref) *pi_ref = 1 + sum;
  if (pi_full) *pi_full = 1 + sum + h[P];
  return DSE_OK;
}

int32_t dse_copy_chunk_mask(dse_ctx* ctx, int32_t my_num, uint64_t* mask) {
  if (!ctx || !mask) return fail(DSE_EINVAL, "null ctx or mask");
  for (auto& d : ctx->devs)
    for (auto& cm : d.resident)
      if (cm.my_num == my_num) {
        HIP_TRY(hipSetDevice(d.device));
        HIP_TRY(hipMemcpyAsync(mask, cm.dev_ptr, cm.words * 8, hipMemcpyDeviceToHost, d.stream));
        HIP_TRY(hipStreamSynchronize(d.stream));
        return DSE_OK;
      }
  return fail(DSE_EINVAL, "chunk " + std::to_string(my_num) + " is not resident");
}

int32_t dse_sieve_window(dse_ctx* ctx, uint64_t lo, uint64_t hi, uint64_t* count) {
  if (!ctx || !count) return fail(DSE_EINVAL, "null ctx or count");
  *count = 0;
  uint64_t a = lo < 3 ? 3 : lo;
  if (!(a & 1)) ++a;
  if (hi < a) return DSE_OK;
  const uint64_t b = (hi & 1) ? hi : hi - 1;
  const uint64_t g0 = (a - 3) / 2, nb = (b - a) / 2 + 1;
  const uint64_t limit = dse_base_limit_for_range(g0, nb);
  if (limit > dse::kBigBaseLimitMax)
    return fail(DSE_ERANGE, "window needs base primes up to " + std::to_string(limit) +
                                "; the device base-prime build supports " + std::to_string(dse::kBigBaseLimitMax));
  const int nd = (int)ctx->devs.size();
  int32_t rc;
  for (int i = 0; i < nd; ++i) {
    DevState& d = ctx->devs[i];
    HIP_TRY(hipSetDevice(d.device));
    if ((rc = ensure_counts(d, 1))) return rc;
    if ((rc = ensure_table(d, limit))) return rc;
    HIP_TRY(hipMemsetAsync(d.counts, 0, sizeof(unsigned long long), d.stream));
  }
  // one table, built on device 0 and RCCL-broadcast (as dse_sieve_all)
  if ((rc = share_table(ctx, limit))) return rc;
  // contiguous slices of the window, one per device
  const uint64_t part = (nb + nd - 1) / nd;
  for (int i = 0; i < nd; ++i) {
    DevState& d = ctx->devs[i];
    HIP_TRY(hipSetDevice(d.device));
    const uint64_t s = std::min<uint64_t>(nb, part * i), e = std::min<uint64_t>(nb, part * (i + 1));
    if (e > s)
      HIP_TRY(dse::launch_sieve_range(d.table, g0 + s, e - s, nullptr, d.counts, d.num_cus, d.stream, &d.scratch,
                                      &ctx->opts));
  }
  if ((rc = allreduce_counts(ctx, 1))) return rc;
  unsigned long long c = 0;
  HIP_TRY(hipSetDevice(ctx->devs[0].device));
  HIP_TRY(hipMemcpyAsync(&c, ctx->devs[0].counts, sizeof(c), hipMemcpyDeviceToHost, ctx->devs[0].stream));
  std::vector<uint32_t> hf(nd);
  for (int i = 0; i < nd; ++i) {
    HIP_TRY(hipSetDevice(ctx->devs[i].device));
    if ((rc = fetch_flag(ctx->devs[i], &hf[i]))) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->devs[i].stream));
  }
  for (int i = 0; i < nd; ++i) {
    HIP_TRY(hipSetDevice(ctx->devs[i].device));
    if ((rc = check_flag(ctx->devs[i], hf[i]))) return rc;
  }
  *count = c;
  return DSE_OK;
}

int32_t dse_device_status(dse_ctx* ctx) {
  if (!ctx) return fail(DSE_EINVAL, "null ctx");
  int32_t rc;
  for (auto& d : ctx->devs) {
    if (!d.scratch.flag) continue;
    HIP_TRY(hipSetDevice(d.device));
    if (d.scratch.used) HIP_TRY(hipEventSynchronize(d.scratch.done));
    uint32_t hf;
    if ((rc = fetch_flag(d, &hf))) return rc;
    HIP_TRY(hipStreamSynchronize(d.stream));
    if ((rc = check_flag(d, hf))) return rc;
  }
  return DSE_OK;
}

int32_t dse_debug_set_option(dse_ctx* ctx, const char* name, int64_t value) {
  if (!ctx || !name) return fail(DSE_EINVAL, "null ctx or option name");
  const std::string n(name);
  if (n == "bucket_pass_segments") {
    if (value < 0 || value > 0xFFFFFFFFll) return fail(DSE_EINVAL, "bucket_pass_segments out of range");
    ctx->opts.bucket_pass_segs = (uint32_t)value;
    return DSE_OK;
  }
  if (n == "bucket_split_log2") {
    if (value < 0 || value > 63) return fail(DSE_EINVAL, "bucket_split_log2 out of range");
    ctx->opts.bucket_split_log2 = (uint32_t)value;
    return DSE_OK;
  }
  if (n == "wheel_geometry") {
    if (value < 0 || value > 2) return fail(DSE_EINVAL, "wheel_geometry must be 0, 1 or 2");
    ctx->opts.wheel_geometry = (uint32_t)value;
    return DSE_OK;
  }
  if (n == "bucket_k0_divisor") {
    if (value < 0 || value > 0xFFFFFFFFll) return fail(DSE_EINVAL, "bucket_k0_divisor out of range");
    ctx->opts.bucket_k0_div = (uint32_t)value;
    return DSE_OK;
  }
  if (n == "scratch_poison") {
    if (value < 0 || value > 1) return fail(DSE_EINVAL, "scratch_poison must be 0 or 1");
    ctx->opts.scratch_poison = (uint32_t)value;
    return DSE_OK;
  }
  if (n == "bucket_lo_log2") {
    // primes above 2^value are bucketed; those up to it go to the wheel kernel's
    // L units, which hold primes <= kWheelMaxPrime only: a larger value would
    // leave (kWheelMaxPrime, 2^value] in neither place
    if (value != 0 && (value < 17 || value > DSE_WHEEL_MAX_LOG))
      return fail(DSE_EINVAL, "bucket_lo_log2 must be 0 or 17.." + std::to_string(DSE_WHEEL_MAX_LOG));
    ctx->opts.bucket_lo_log2 = (uint32_t)value;
    return DSE_OK;
  }
  if (n == "rccl_single") {
    if (value < 0 || value > 1) return fail(DSE_EINVAL, "rccl_single must be 0 or 1");
    if (ctx->logical || ctx->devs.size() != 1)
      return fail(DSE_EINVAL, "rccl_single needs a one-device context (dse_init(1) or dse_init_device)");
    if (value == 1 && ctx->comms.empty()) {
      int dev = ctx->devs[0].device;
      HIP_TRY(hipSetDevice(dev));
      ncclComm_t c;
      NCCL_TRY(ncclCommInitAll(&c, 1, &dev));
      ctx->comms.push_back(c);
    } else if (value == 0 && !ctx->comms.empty()) {
      HIP_TRY(hipSetDevice(ctx->devs[0].device));
      HIP_TRY(hipStreamSynchronize(ctx->devs[0].stream));
      NCCL_TRY(ncclCommDestroy(ctx->comms[0]));
      ctx->comms.clear();
    }
    ctx->rccl_single = value == 1;
    return DSE_OK;
  }
  if (n == "table_broadcast_max_bytes") {
    if (value < 0) return fail(DSE_EINVAL, "table_broadcast_max_bytes must be >= 0");
    ctx->opts.table_bcast_max = (uint64_t)value;
    return DSE_OK;
  }
  if (n == "bucket_cap_divisor") {
    if (value < 0 || value > 0xFFFFFFFFll) return fail(DSE_EINVAL, "bucket_cap_divisor out of range");
    ctx->opts.bucket_cap_div = (uint32_t)value;
    return DSE_OK;
  }
  return fail(DSE_EINVAL, "unknown option " + n);
}

int32_t dse_debug_get_stat(dse_ctx* ctx, const char* name, int64_t* value) {
  if (!ctx || !name || !value) return fail(DSE_EINVAL, "null ctx, stat name or value");
  const std::string n(name);
  if (n == "rccl_calls") {
    *value = ctx->rccl_calls;
    return DSE_OK;
  }
  if (n == "table_local_builds") {
    *value = ctx->table_local_builds;
    return DSE_OK;
  }
  if (n == "rccl_comms") {
    *value = (int64_t)ctx->comms.size();
    return DSE_OK;
  }
  if (n == "rccl_ranks") {  // ranks of the context's communicators, as RCCL reports them
    int c = 0;
    if (!ctx->comms.empty()) NCCL_TRY(ncclCommCount(ctx->comms[0], &c));
    *value = c;
    return DSE_OK;
  }
  return fail(DSE_EINVAL, "unknown stat " + n);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// finish writer (sieve.clj:82-108)
// ---------------------------------------------------------------------------
namespace {

inline int fmt_u64(uint64_t v, char* out) {
  char t[24];
  int n = 0;
  do {
    t[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  for (int i = 0; i < n; ++i) out[i] = t[n - 1 - i];
  return n;
}

// java.lang.Double.toString of an integer-valued double 1 <= v < 2^53.
inline int fmt_java_double(uint64_t v, char* out) {
  if (v < 10000000ull) {
    int n = fmt_u64(v, out);
    out[n++] = '.';
    out[n++] = '0';
    return n;
  }
  char d[24];
  int len = fmt_u64(v, d);
  int sig = len;
  while (sig > 1 && d[sig - 1] == '0') --sig;
  int n = 0;
  out[n++] = d[0];
  out[n++] = '.';
  if (sig == 1) out[n++] = '0';
  for (int i = 1; i < sig; ++i) out[n++] = d[i];
  out[n++] = 'E';
  n += fmt_u64((uint64_t)(len - 1), out + n);
  return n;
}

}  // namespace

extern "C" int32_t dse_write_range_file(const char* path, int32_t my_num, uint64_t g_start, uint64_t nbits,
                                        const uint64_t* mask) {
  if (!path || !mask) return fail(DSE_EINVAL, "null path or mask");
  if (my_num < 1) return fail(DSE_EINVAL, "my_num must be >= 1");
  if (my_num == 1 && nbits < 4) return fail(DSE_EINVAL, "finish's 2/3/5/7 hack needs a chunk of >= 4 candidates");
  const uint64_t cs = nbits;
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(DSE_EIO, std::string("cannot open ") + path);
  std::vector<char> buf(1 << 20);
  size_t used = 0;
  int per_line = 0;
  const uint64_t base = g_start;
  auto emit = [&](uint64_t v) {
    if (used + 64 > buf.size()) {
      std::fwrite(buf.data(), 1, used, f);
      used = 0;
    }
    if (per_line) {
      buf[used++] = ',';
      buf[used++] = ' ';
    }
    used += (size_t)(my_num == 1 ? fmt_java_double(v, buf.data() + used) : fmt_u64(v, buf.data() + used));
    if (++per_line == 10) {
      buf[used++] = '\n';
      per_line = 0;
    }
  };
  const uint64_t words = (cs + 63) / 64;
  uint64_t j0 = 0;
  if (my_num == 1) {  // positions 0..3 become 2.0 3.0 5.0 7.0 (sieve.clj:93-96)
    emit(2);
    emit(3);
    emit(5);
    emit(7);
    j0 = 4;
  }
  for (uint64_t w = j0 / 64; w < words; ++w) {
    uint64_t v = mask[w];
    if (w == j0 / 64) v &= ~0ull << (j0 % 64);
    if (w == words - 1 && (cs & 63)) v &= (1ull << (cs & 63)) - 1;
    while (v) {
      const int b = __builtin_ctzll(v);
      v &= v - 1;
      emit(3 + 2 * (base + w * 64 + (uint64_t)b));
    }
  }
  if (per_line) buf[used++] = '\n';
  std::fwrite(buf.data(), 1, used, f);
  if (std::fclose(f) != 0) return fail(DSE_EIO, std::string("write failed: ") + path);
  return DSE_OK;
}

extern "C" int32_t dse_write_primes_file(const char* path, int32_t my_num, int64_t n, int32_t P,
                                         const uint64_t* mask) {
  int64_t cs;
  int32_t rc = chunk_geometry(n, P, &cs);
  if (rc) return rc;
  if (my_num < 1 || my_num > P) return fail(DSE_EINVAL, "my_num outside 1..P");
  if (cs < 4) return fail(DSE_EINVAL, "finish's 2/3/5/7 hack needs a chunk of >= 4 candidates");
  return dse_write_range_file(path, my_num, (uint64_t)(my_num - 1) * (uint64_t)cs, (uint64_t)cs, mask);
}

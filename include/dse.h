/*
 * dse.h -- C ABI of the MI355X-native chunked odd-only sieve (libdse.so).
 *
 * This is the drop-in boundary for the hot path of dpbriggs/Distributed-Sieve-e:
 * the reference's lead/follower entry points (core.clj:136-205) call
 * spread-work / gen-table / sieve-e / finish (sieve.clj:9-172); here those
 * calls become the functions below, which launch hand-written gfx950 HIP
 * kernels. Each declaration names the reference interface it replaces.
 *
 * Conventions
 *  - Every function returns DSE_OK (0) or a negative DSE_E* status; the
 *    message of the last failure on the calling thread is dse_last_error().
 *  - Host output buffers are caller-allocated (ctypes / JNA Memory / FFM
 *    MemorySegment). The library never retains caller pointers.
 *  - Device buffers are owned by the dse_ctx, except in the *_dev entry
 *    points, which take caller-owned device pointers (e.g. torch tensors).
 *  - Calls are blocking (like sieve-e on the caller's main thread,
 *    core.clj:163,196) unless the name ends in _async.
 *  - Chunk semantics are the reference's exactly: cs = floor(floor((n-1)/2)/P),
 *    chunk k (1-based) holds the odd values [3+2(k-1)cs, 3+2k*cs); the
 *    floor((n-1)/2) - P*cs highest odd candidates are dropped (sieve.clj:21-34).
 *  - Mask layout: little-endian uint64 words, bit j of chunk k = 1 iff the
 *    value 3+2((k-1)cs+j) is prime (= element j non-zero before finish);
 *    bits past cs in the last word are 0.
 */
#ifndef DSE_H
#define DSE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSE_OK 0
#define DSE_EINVAL -1   /* bad argument (P < 1, cs < 4 where finish needs it, ...) */
#define DSE_EHIP -2     /* HIP runtime error */
#define DSE_ENCCL -3    /* RCCL error */
#define DSE_ENOMEM -4   /* host or device allocation failed */
#define DSE_EIO -5      /* file I/O */
#define DSE_ERANGE -6   /* input outside the supported range */
#define DSE_EINTERNAL -7 /* device-side invariant broken (bucket capacity overflow); result not valid */

typedef struct dse_ctx dse_ctx;

/* Library version string, e.g. "dse 0.1 gfx950". */
const char *dse_version(void);

/* Message of the last failed call on this thread ("" if none). */
const char *dse_last_error(void);

/* DSE_E* status of the last failed call on this thread (DSE_OK if none); for
 * the entry points that return a pointer (dse_init, dse_init_device). */
int32_t dse_last_status(void);

/* Number of visible HIP devices (0 if none). */
int32_t dse_device_count(void);

/* One process driving num_gpus devices 0..num_gpus-1 (0 = all visible), with
 * one RCCL communicator over them when num_gpus > 1. Replaces the lead's
 * socket server + client wait (core.clj:76-116, 141-147). NULL on failure. */
dse_ctx *dse_init(int32_t num_gpus);

/* One context bound to a single device, for one-process-per-GPU ranks that
 * bring their own communicator (torch.distributed / RCCL). Replaces the
 * follower's connect (core.clj:13-31, 186). NULL on failure. */
dse_ctx *dse_init_device(int32_t device);

void dse_destroy(dse_ctx *ctx);

/* Number of devices the context drives. */
int32_t dse_ctx_num_devices(const dse_ctx *ctx);

/* sieve.clj:15-34 spread-work, in exact int64: lo_hi[2(k-1)], lo_hi[2(k-1)+1]
 * = bounds of chunk k (caller allocates 2*P entries; may be NULL); *cs = chunk
 * size in odd candidates. */
int32_t dse_spread_work(int64_t n, int32_t P, int64_t *lo_hi, int64_t *cs);

/* Odd indices [*g_start, *g_start + *nbits) that spread-work drops
 * (values 3+2P*cs .. n); *nbits <= P-1. */
int32_t dse_tail_range(int64_t n, int32_t P, uint64_t *g_start, uint64_t *nbits);

/* gen-table + sieve-e for ONE chunk (sieve.clj:9-13, 118-172; core.clj:152,
 * 163, 192, 196): sieve chunk my_num of the (n, P) run on the context's
 * device ((my_num-1) mod num_devices). mask_or_null: host buffer of
 * ceil(cs/64) uint64 words, or NULL for count only. *count = primes in the
 * chunk (odd values only; the "2" that finish injects is not counted). */
int32_t dse_sieve_chunk(dse_ctx *ctx, int64_t n, int32_t P, int32_t my_num,
                        uint64_t *mask_or_null, uint64_t *count);

/* gen-table + sieve-e for an arbitrary odd-index range (a chunk given by its
 * bounds [lo, hi): g_start = (lo-3)/2, nbits = (hi-lo)/2), on the context's
 * first device. mask_or_null: ceil(nbits/64) words; *count = primes. */
int32_t dse_sieve_odd_range(dse_ctx *ctx, uint64_t g_start, uint64_t nbits,
                            uint64_t *mask_or_null, uint64_t *count);

/* The whole lead/follower run (core.clj:136-205) on the context's devices:
 * base primes <= sqrt(max value) computed once on device 0 and broadcast with
 * RCCL (replaces the per-prime [mi ps p] relay, sieve.clj:139 /
 * core.clj:118-134), chunk k sieved on device (k-1) mod num_devices with its
 * mask left resident in that device's HBM, the dropped tail sieved on the last
 * device, counts combined with an RCCL all-reduce.
 * per_chunk_counts: P entries (may be NULL). *pi_ref = 1 + sum(counts) (what
 * the reference's files hold); *pi_full = pi_ref + primes in the tail = pi(n).
 * Either pi pointer may be NULL. */
int32_t dse_sieve_all(dse_ctx *ctx, int64_t n, int32_t P, uint64_t *per_chunk_counts,
                      uint64_t *pi_ref, uint64_t *pi_full);

/* Copy chunk my_num's mask kept resident by the last dse_sieve_all into a host
 * buffer of ceil(cs/64) words. DSE_EINVAL if that chunk is not resident. */
int32_t dse_copy_chunk_mask(dse_ctx *ctx, int32_t my_num, uint64_t *mask);

/* Sieve the odd values in [lo, hi] (any 64-bit window, lo,hi odd or even;
 * "segment-only" mode outside the reference's chunk semantics). Counts
 * primes in [max(lo,3), hi] among odd values. With several devices: the base
 * primes are built on device 0 and RCCL-broadcast (as in dse_sieve_all), each
 * device sieves one contiguous slice, the counts are RCCL all-reduced. */
int32_t dse_sieve_window(dse_ctx *ctx, uint64_t lo, uint64_t hi, uint64_t *count);

/* sieve.clj:82-108 finish: write chunk my_num's primes to path, byte-exact
 * with the reference's file: chunk 1 values printed as Java Doubles ("2.0",
 * "1.0000019E7") with the 2/3/5/7 hack, others as Longs; 10 per line,
 * ", "-separated, LF-terminated lines. mask: ceil(cs/64) words. Needs cs >= 4. */
int32_t dse_write_primes_file(const char *path, int32_t my_num, int64_t n, int32_t P,
                              const uint64_t *mask);

/* finish for a chunk given by its odd-index range: same format as
 * dse_write_primes_file; my_num == 1 selects the Double printing + hack. */
int32_t dse_write_range_file(const char *path, int32_t my_num, uint64_t g_start, uint64_t nbits,
                             const uint64_t *mask);

/* ---- Device-resident entry points (one-process-per-GPU ranks) ---------- */

/* Bytes of a base-prime table able to hold every odd prime <= limit. */
uint64_t dse_base_table_bytes(uint64_t limit);

/* Largest base-prime limit the device kernel supports. */
uint64_t dse_base_limit_max(void);

/* isqrt of the largest value in odd-index range [g_start, g_start+nbits):
 * the base-prime limit that range needs. */
uint64_t dse_base_limit_for_range(uint64_t g_start, uint64_t nbits);

/* Build the table of odd primes <= limit into caller-owned device memory
 * table_dev (dse_base_table_bytes(limit) bytes) on stream (hipStream_t, NULL
 * = default). Asynchronous. The table is plain bytes: ranks may broadcast it
 * with any collective (RCCL) before sieving. */
int32_t dse_base_primes_dev_async(dse_ctx *ctx, uint64_t limit, void *table_dev,
                                  uint64_t table_bytes, void *stream);

/* Bytes at the start of a base-prime table that hold the primes themselves
 * (header + p[]). Ranks broadcast only these (the reference's prime
 * broadcast, sieve.clj:139 / core.clj:126) and complete the rest locally with
 * dse_base_table_finish_dev_async. */
uint64_t dse_base_table_prime_bytes(uint64_t limit);

/* How ranks should share the base table for `limit`: the bytes to broadcast
 * from rank 0 (dse_base_table_prime_bytes(limit)), or 0 when every rank should
 * build its own table with dse_base_primes_dev_async instead. The primes are
 * broadcast (as the reference broadcasts them, sieve.clj:139) while they fit
 * in DSE_TABLE_BROADCAST_MAX_BYTES; a larger table (the 1e18 window's 50.8 M
 * primes, 203 MB) is rebuilt on every device, which takes less time than
 * moving it. dse_sieve_all / dse_sieve_window follow
 * the same rule. */
#define DSE_TABLE_BROADCAST_MAX_BYTES (8ull << 20)
uint64_t dse_base_table_broadcast_bytes(uint64_t limit);

/* Complete a table of odd primes <= limit whose first
 * dse_base_table_prime_bytes(limit) bytes are in place (e.g. received by
 * broadcast): Barrett factors and mod-30 wheel offsets, on this context's
 * device. Asynchronous on stream. */
int32_t dse_base_table_finish_dev_async(dse_ctx *ctx, uint64_t limit, void *table_dev,
                                        uint64_t table_bytes, void *stream);

/* Sieve odd indices [g_start, g_start+nbits) with a base table on the device:
 * mask_dev (ceil(nbits/64) uint64 words, or NULL) receives the prime bits,
 * *count_dev (device uint64) is INCREMENTED by the prime count (zero it
 * first). Asynchronous on stream. A device-side failure (DSE_EINTERNAL: a
 * bucket pass over its entry capacity, a rigorous bound, so never expected)
 * sets bit 63 of *count_dev and is reported by dse_device_status. */
int32_t dse_sieve_range_dev_async(dse_ctx *ctx, const void *table_dev, uint64_t g_start,
                                  uint64_t nbits, uint64_t *mask_dev, uint64_t *count_dev,
                                  void *stream);

/* Wait for the context's last bucketed pass, then read and clear its
 * device-side error flag: DSE_OK, or DSE_EINTERNAL if any pass since the last
 * check overflowed. The blocking entry points check it themselves. */
int32_t dse_device_status(dse_ctx *ctx);

/* ---- Test-only ---------------------------------------------------------- */

/* Set a test-only option of this context (the production library reads no
 * environment variable; defaults are the production configuration):
 *   "bucket_pass_segments" = k > 0: bucketed passes of at most k segments
 *   (covers the multi-pass path on small windows); 0 = default.
 *   "bucket_split_log2" = k in 0..63: bucketed primes <= 2^k take the
 *   one-level fill, larger ones the two-level staged fill; 0 = the default
 *   split (2^28).
 *   "wheel_geometry" = 0 (default): a range's last partial round of full
 *   segments is sieved as half-size segments when that is faster; 1: full
 *   segments only; 2: half-size segments only (covers that kernel in tests).
 *   "bucket_cap_divisor" = d >= 0: divide each pass's bucket entry capacities
 *   by d (> 1), forcing the overflow path (DSE_EINTERNAL); 0 or 1 = default.
 *   "bucket_k0_divisor" = d >= 0: divide the band-0 region capacity by d
 *   (> 1), so hits go through the spill list (results unchanged); 0 or 1 =
 *   default.
 *   "scratch_poison" = 1: fill the bucket scratch with 0xFF bytes before
 *   every bucketed pass (stale contents: results unchanged, and an overflowed
 *   pass still reads only what it wrote); 0 = default.
 *   "bucket_lo_log2" = k in 17..20 (at most the build's wheel limit, 2^20 in
 *   production): a range that needs the bucketed pass (sqrt of its largest
 *   value above 2^20) buckets every prime above 2^k instead of the production
 *   threshold; 0 = default.
 *   "table_broadcast_max_bytes" = b > 0: dse_sieve_all / dse_sieve_window
 *   broadcast the table's primes while they take at most b bytes and build
 *   the table on every device above that; 0 = default
 *   (DSE_TABLE_BROADCAST_MAX_BYTES).
 *   "rccl_single" = 1: give a one-device context (dse_init(1) or
 *   dse_init_device) a 1-rank RCCL communicator (ncclCommInitAll), so
 *   dse_sieve_all / dse_sieve_window issue the same grouped ncclBroadcast of
 *   the primes and ncclAllReduce of the counts as an 8-GPU context instead of
 *   skipping them (the RCCL path exercised on a one-GPU box); 0 = default (no
 *   communicator, no collective for one device).
 * DSE_EINVAL for an unknown name or a value out of range. */
int32_t dse_debug_set_option(dse_ctx *ctx, const char *name, int64_t value);

/* Read a test-only statistic of this context into *value:
 *   "rccl_calls": RCCL collectives (one per device and call) accepted so far;
 *   "rccl_comms": communicators the context holds;
 *   "rccl_ranks": ranks of its communicator as ncclCommCount reports (0: none);
 *   "table_local_builds": base tables built on a device of their own instead
 *   of broadcast (one per device and call).
 * DSE_EINVAL for an unknown name. */
int32_t dse_debug_get_stat(dse_ctx *ctx, const char *name, int64_t *value);

/* A context of num_logical devices that all run on device 0 (each its own
 * stream, table, counts, masks and scratch; a device's chunks are pooled into
 * one persistent launch, as on a real device), so the multi-device
 * code of dse_sieve_all / dse_sieve_window -- chunk map, table completion on
 * the non-root devices, tail on the last device, flag checks -- runs on a
 * one-GPU box. Only the two RCCL collectives are replaced: the broadcast of
 * the primes by a device-to-device copy from device 0's table, the count
 * all-reduce by a gather + sum on device 0 and a copy back, each ordered
 * with events exactly where the RCCL calls would run. Test-only; NULL on
 * failure (dse_last_status). */
dse_ctx *dse_debug_init_logical(int32_t num_logical);

#ifdef __cplusplus
}
#endif

#endif /* DSE_H */

/*
 * dse_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A CPU restatement of the reference's chunked odd-only sieve
 * (/root/reference/src/mail_sieve_e/sieve.clj and the prime relay in
 * /root/reference/src/mail_sieve_e/core.clj). It is the checker the parity
 * tests, __graft_entry__.smoke() and bench.py's cpu_baseline leg compare the
 * HIP path against. Nothing in the product (libdse.so, mail_sieve_e) links or
 * calls this file.
 *
 * Parity status: the reference ships no fixtures and cannot run here (Clojure
 * on the JVM; no java/lein in the image), so this restatement is pinned by
 * independent known answers instead: published pi(10^k), sympy.isprime sweeps,
 * the README's chunk size (README.txt:16) and the SURVEY.md section 4 table.
 * See DESIGN.md "Oracle".
 *
 * Two checkers live here:
 *   ref_*   a faithful, single-threaded restatement of sieve.clj: the same
 *           spread-work bounds, the same survivor scan with its end-of-chunk
 *           sentinel, the same per-prime lead/follower marking walk (including
 *           the early-indices skip), processed in the race-free order.
 *   fast_*  an OpenMP odd-only segmented sieve used only to produce golden
 *           hashes at sizes the faithful restatement cannot reach; it is itself
 *           cross-checked against ref_* in tests/test_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define REF_OK 0
#define REF_EINVAL -1
#define REF_ENOMEM -2
#define REF_EIO -3
#define REF_EINTERNAL -4

/* sieve.clj:15-34 spread-work. nums = floor((n-1)/2) (:21), chunk-size =
 * floor(nums/num-comps) (:23); chunk k (1-based) = [3+2(k-1)cs, 3+2k*cs)
 * (:25-32). The remainder nums - P*cs is dropped. Exact in int64 (the
 * reference uses Double, identical below 2^53). */
int ref_spread_work(int64_t n, int32_t P, int64_t *lo_hi, int64_t *cs_out) {
  if (P < 1 || n < 0) return REF_EINVAL;
  int64_t nums = (n - 1) / 2;
  if (n < 1) nums = 0; /* Math/floor of a negative ratio would be <0; no chunks */
  int64_t cs = nums / P;
  if (cs_out) *cs_out = cs;
  if (lo_hi)
    for (int32_t k = 1; k <= P; ++k) {
      lo_hi[2 * (k - 1)] = 3 + 2 * (int64_t)(k - 1) * cs;
      lo_hi[2 * (k - 1) + 1] = 3 + 2 * (int64_t)k * cs;
    }
  return REF_OK;
}

/* sieve.clj:47-71 mark-composites: zero the odd multiples of p (from 3p) that
 * fall inside chunk my_num. mi = reporting machine, ps = prime position in the
 * reporter's chunk, coll = chunk my_num (1 = non-zero, 0 = zeroed). */
static void ref_mark_composites(int64_t mi, int64_t cs, int64_t ps, int64_t p, int64_t my_num,
                                uint8_t *coll) {
  /* :56 early-indices = (my-num - 1) * floor((cs - ps)/p), a Double */
  double early = (double)(my_num - 1) * floor((double)(cs - ps) / (double)p);
  /* :57 (drop (dec early) (indices ...)): drops ceil(early-1) elements when positive */
  double ndrop = early - 1.0;
  int64_t first_i = 1 + (ndrop > 0 ? (int64_t)ceil(ndrop) : 0);
  /* :36-45 indices: k = ps + cs*(mi-1), elements k + i*p for i >= 1 */
  int64_t k = ps + cs * (mi - 1);
  int64_t lower = (my_num - 1) * cs; /* :58 */
  int64_t upper = my_num * cs - 1;   /* :59 */
  for (int64_t head = k + first_i * p; head <= upper; head += p) /* :60-63 */
    if (head >= lower) coll[head % cs] = 0;                      /* :64-67 */
}

/* sieve.clj:73-80 find-next-non-zero. (get coll cs) is nil and (not= 0 nil)
 * is true, so the scan returns cs at the end of the chunk; it returns nil (-1
 * here) only when start >= cs. */
static int64_t ref_find_next_non_zero(const uint8_t *coll, int64_t start, int64_t cs) {
  for (int64_t stop = start + 1; stop <= cs; ++stop)
    if (stop == cs || coll[stop] != 0) return stop;
  return -1;
}

/* sieve.clj:110-116 find-first-prime */
static int64_t ref_find_first_prime(const uint8_t *coll, int64_t cs) {
  if (coll[0] != 0) return 0;
  return ref_find_next_non_zero(coll, -1, cs);
}

/* The whole distributed run in its race-free order:
 * machine m leads only after machine m-1 appointed it (sieve.clj:145-150,
 * 167-171); every prime it reports reaches its own chunk (sieve.clj:141) and
 * every machine numbered above it (core.clj:122-126 -> sieve.clj:164).
 * flags: P*cs bytes, caller-allocated; byte j of chunk k (offset (k-1)*cs+j)
 * ends 1 iff element j of chunk k is non-zero before finish (value 3+2((k-1)cs+j)).
 * msgs (nullable): number of [mi ps p] prime messages broadcast. */
int ref_sieve_flags(int64_t n, int32_t P, uint8_t *flags, uint64_t *msgs) {
  int64_t cs;
  int rc = ref_spread_work(n, P, NULL, &cs);
  if (rc) return rc;
  if (cs < 1) return REF_EINVAL; /* find-first-prime NPEs on an empty chunk */
  memset(flags, 1, (size_t)P * (size_t)cs); /* gen-table: every element non-zero */
  uint64_t nmsg = 0;
  for (int64_t m = 1; m <= P; ++m) {
    uint8_t *own = flags + (size_t)(m - 1) * (size_t)cs;
    int64_t start = ref_find_first_prime(own, cs); /* sieve.clj:131 */
    for (;;) {
      int64_t n_start = ref_find_next_non_zero(own, start, cs); /* :134 */
      if (n_start < 0) break;                                   /* :135 -> appoint */
      if (start >= cs || own[start] == 0) return REF_EINTERNAL; /* a zero "prime" would hang the reference */
      int64_t prime = 3 + 2 * ((m - 1) * cs + start);           /* (get chunk start) */
      ++nmsg;                                                   /* :139 >!! [my-num start prime] */
      for (int64_t k = m; k <= P; ++k)                          /* own chunk (:141) + followers (:164) */
        ref_mark_composites(m, cs, start, prime, k, flags + (size_t)(k - 1) * (size_t)cs);
      start = n_start; /* :143 */
    }
  }
  if (msgs) *msgs = nmsg;
  return REF_OK;
}

static uint64_t popcount_flags_to_mask(const uint8_t *f, int64_t cs, uint64_t *mask) {
  int64_t words = (cs + 63) / 64;
  uint64_t cnt = 0;
  for (int64_t w = 0; w < words; ++w) {
    uint64_t v = 0;
    int64_t base = w * 64;
    int64_t lim = cs - base < 64 ? cs - base : 64;
    for (int64_t b = 0; b < lim; ++b) v |= (uint64_t)(f[base + b] != 0) << b;
    if (mask) mask[w] = v;
    cnt += (uint64_t)__builtin_popcountll(v);
  }
  return cnt;
}

/* Faithful run, packed: masks = P * ceil(cs/64) little-endian uint64 words,
 * bit j of chunk k = 1 iff element j is non-zero before finish; counts[k-1] =
 * popcount of chunk k. Returns cs via cs_out. */
int ref_sieve(int64_t n, int32_t P, uint64_t *masks, uint64_t *counts, int64_t *cs_out,
              uint64_t *msgs) {
  int64_t cs;
  int rc = ref_spread_work(n, P, NULL, &cs);
  if (rc) return rc;
  if (cs_out) *cs_out = cs;
  if (cs < 1) return REF_EINVAL;
  uint8_t *flags = (uint8_t *)malloc((size_t)P * (size_t)cs);
  if (!flags) return REF_ENOMEM;
  rc = ref_sieve_flags(n, P, flags, msgs);
  if (rc) { free(flags); return rc; }
  int64_t words = (cs + 63) / 64;
  for (int32_t k = 0; k < P; ++k) {
    uint64_t c = popcount_flags_to_mask(flags + (size_t)k * (size_t)cs, cs,
                                        masks ? masks + (size_t)k * (size_t)words : NULL);
    if (counts) counts[k] = c;
  }
  free(flags);
  return REF_OK;
}

/* java.lang.Double.toString for an integer-valued double v, 1 <= v < 2^53:
 * "<int>.0" below 1e7, otherwise "d.dddE<exp>" with the integer's significant
 * digits (trailing zeros dropped, at least one fraction digit). */
static int java_double_str(uint64_t v, char *out) {
  if (v < 10000000ull) return sprintf(out, "%llu.0", (unsigned long long)v);
  char d[32];
  int len = sprintf(d, "%llu", (unsigned long long)v);
  int sig = len;
  while (sig > 1 && d[sig - 1] == '0') --sig;
  int o = 0;
  out[o++] = d[0];
  out[o++] = '.';
  if (sig == 1) out[o++] = '0';
  else { memcpy(out + o, d + 1, (size_t)(sig - 1)); o += sig - 1; }
  o += sprintf(out + o, "E%d", len - 1);
  return o;
}

/* sieve.clj:82-108 finish, applied to chunk my_num's packed mask: chunk 1
 * elements are Doubles (gen-table over [3.0 ..), core.clj:152) and get the
 * 2/3/5/7 hack at positions 0..3 (:93-96); other chunks hold Longs
 * (core.clj:191 mapv int). Non-zero values, 10 per line, ", "-joined, each
 * line ended by line.separator (LF). Requires cs >= 4 as the hack does. */
int ref_finish(const char *path, int32_t my_num, int64_t n, int32_t P, const uint64_t *mask) {
  int64_t cs;
  int rc = ref_spread_work(n, P, NULL, &cs);
  if (rc) return rc;
  if (my_num < 1 || my_num > P || cs < 4) return REF_EINVAL;
  FILE *f = fopen(path, "wb");
  if (!f) return REF_EIO;
  int64_t base = (int64_t)(my_num - 1) * cs;
  int per_line = 0;
  char buf[48];
  for (int64_t j = 0; j < cs; ++j) {
    uint64_t v;
    if (my_num == 1 && j < 4) v = (uint64_t)(j == 0 ? 2 : j == 1 ? 3 : j == 2 ? 5 : 7);
    else {
      if (!((mask[j >> 6] >> (j & 63)) & 1)) continue;
      v = (uint64_t)(3 + 2 * (base + j));
    }
    int len = (my_num == 1) ? java_double_str(v, buf) : sprintf(buf, "%llu", (unsigned long long)v);
    if (per_line) fputs(", ", f);
    fwrite(buf, 1, (size_t)len, f);
    if (++per_line == 10) { fputc('\n', f); per_line = 0; }
  }
  if (per_line) fputc('\n', f);
  return fclose(f) == 0 ? REF_OK : REF_EIO;
}

/* ---------------------------------------------------------------------
 * fast_*: independent OpenMP segmented sieve over global odd indices
 * [g0, g0+nbits) (value 3+2g). Output uses the same packed layout as
 * ref_sieve (bit j <-> index g0+j; 1 = prime).
 * --------------------------------------------------------------------- */
static uint32_t *fast_base_primes(uint64_t limit, uint64_t *np_out) {
  /* odd primes <= limit by a plain sieve */
  uint64_t m = limit / 2 + 1;
  uint8_t *c = (uint8_t *)calloc(m + 1, 1);
  uint64_t cap = 1024, np = 0;
  uint32_t *pr = (uint32_t *)malloc(cap * sizeof(uint32_t));
  for (uint64_t v = 3; v <= limit; v += 2) {
    if (c[v / 2]) continue;
    if (np == cap) { cap *= 2; pr = (uint32_t *)realloc(pr, cap * sizeof(uint32_t)); }
    pr[np++] = (uint32_t)v;
    for (uint64_t w = v * v; w <= limit; w += 2 * v) c[w / 2] = 1;
  }
  free(c);
  *np_out = np;
  return pr;
}

static uint64_t isqrt_u64(uint64_t x) {
  uint64_t r = (uint64_t)sqrtl((long double)x);
  while (r * r > x) --r;
  while ((r + 1) * (r + 1) <= x) ++r;
  return r;
}

int fast_sieve_range(uint64_t g0, uint64_t nbits, uint64_t *mask, uint64_t *count) {
  if (nbits == 0) { if (count) *count = 0; return REF_OK; }
  uint64_t vmax = 3 + 2 * (g0 + nbits - 1);
  uint64_t np;
  uint32_t *pr = fast_base_primes(isqrt_u64(vmax), &np);
  const uint64_t SEG = 1ull << 18; /* bits per segment, multiple of 64 */
  uint64_t nseg = (nbits + SEG - 1) / SEG;
  uint64_t total = 0;
#pragma omp parallel reduction(+ : total)
  {
    uint8_t *s = (uint8_t *)malloc(SEG);
#pragma omp for schedule(dynamic, 4)
    for (uint64_t sg = 0; sg < nseg; ++sg) {
      uint64_t b0 = sg * SEG, len = nbits - b0 < SEG ? nbits - b0 : SEG;
      uint64_t G = g0 + b0;
      memset(s, 1, len);
      for (uint64_t i = 0; i < np; ++i) {
        uint64_t p = pr[i];
        uint64_t gq = (p * p - 3) / 2; /* index of p^2 */
        if (gq >= G + len) break;
        uint64_t off = gq >= G ? gq - G : (p - (G - gq) % p) % p;
        for (; off < len; off += p) s[off] = 0;
      }
      for (uint64_t w = 0; w < (len + 63) / 64; ++w) {
        uint64_t v = 0;
        uint64_t lim = len - w * 64 < 64 ? len - w * 64 : 64;
        for (uint64_t b = 0; b < lim; ++b) v |= (uint64_t)s[w * 64 + b] << b;
        if (mask) mask[b0 / 64 + w] = v;
        total += (uint64_t)__builtin_popcountll(v);
      }
    }
    free(s);
  }
  free(pr);
  if (count) *count = total;
  return REF_OK;
}

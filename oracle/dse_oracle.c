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
 * The checkers that live here:
 *   ref_*   a faithful, single-threaded restatement of sieve.clj: the same
 *           spread-work bounds, the same survivor scan with its end-of-chunk
 *           sentinel, the same per-prime lead/follower marking walk (including
 *           the early-indices skip), processed in the race-free order.
 *   ref_sieve_threaded  the same machines as P threads exchanging [mi ps p]
 *           messages through in-process queues, with machine 1's relay
 *           (core.clj:118-134) as a thread of its own: the reference's
 *           lead/follower run on one host's cores, timed by bench.py's
 *           cpu_baseline leg (no JVM in the image).
 *   fast_*  an OpenMP odd-only segmented sieve used only to produce golden
 *           hashes at sizes the faithful restatement cannot reach; it is itself
 *           cross-checked against ref_* in tests/test_oracle.py.
 *   fast_count_window  an independent OpenMP count of the primes in a high
 *           window (outside the reference's semantics).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

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

/* ---------------------------------------------------------------------
 * ref_sieve_threaded: the lead/follower run (core.clj:136-205,
 * sieve.clj:118-172) as P machine threads plus machine 1's relay thread.
 *   machine 1 leads first; for every survivor of its chunk it sends
 *     [1 start prime] to every follower (send-chan broadcast,
 *     core.clj:93-95), then marks its own chunk (sieve.clj:139-141);
 *     at the end it sends the appoint [1 -1 0] to every follower (:148);
 *   machine m >= 2 follows: it marks its chunk for every [mi ps p] it
 *     receives (sieve.clj:156-164) until the appoint [m-1 -1 0], then leads,
 *     sending its lines to the relay (its out-channel is the socket to
 *     machine 1), which forwards each line to the machines > mi
 *     (core.clj:122-126); the appoint from machine P ends the run (:132-134).
 * FIFO queues give the race-free order of SURVEY.md section 5 (i), so the
 * result equals ref_sieve's. Same outputs as ref_sieve.
 * --------------------------------------------------------------------- */
typedef struct {
  int64_t mi, ps, p;
} ref_msg;

typedef struct {
  ref_msg *buf;
  size_t head, tail, cap;
  int closed; /* set by rq_close: pops of an empty queue return REF_MSG_CLOSED */
  pthread_mutex_t mu;
  pthread_cond_t cv;
} ref_queue;

static const ref_msg REF_MSG_CLOSED = {-2, -2, 0};

static int rq_init(ref_queue *q) {
  q->cap = 1024;
  q->head = q->tail = 0;
  q->closed = 0;
  q->buf = (ref_msg *)malloc(q->cap * sizeof(ref_msg));
  if (!q->buf) return REF_ENOMEM;
  pthread_mutex_init(&q->mu, NULL);
  pthread_cond_init(&q->cv, NULL);
  return REF_OK;
}

static void rq_free(ref_queue *q) {
  free(q->buf);
  pthread_mutex_destroy(&q->mu);
  pthread_cond_destroy(&q->cv);
}

static int rq_push(ref_queue *q, ref_msg m) {
  pthread_mutex_lock(&q->mu);
  if (q->tail == q->cap) {
    if (q->head > 0) {
      memmove(q->buf, q->buf + q->head, (q->tail - q->head) * sizeof(ref_msg));
      q->tail -= q->head;
      q->head = 0;
    }
    if (q->tail == q->cap) {
      ref_msg *nb = (ref_msg *)realloc(q->buf, 2 * q->cap * sizeof(ref_msg));
      if (!nb) { pthread_mutex_unlock(&q->mu); return REF_ENOMEM; }
      q->buf = nb;
      q->cap *= 2;
    }
  }
  q->buf[q->tail++] = m;
  pthread_cond_signal(&q->cv);
  pthread_mutex_unlock(&q->mu);
  return REF_OK;
}

static ref_msg rq_pop(ref_queue *q) {
  pthread_mutex_lock(&q->mu);
  while (q->head == q->tail && !q->closed) pthread_cond_wait(&q->cv, &q->mu);
  const ref_msg m = q->head < q->tail ? q->buf[q->head++] : REF_MSG_CLOSED;
  pthread_mutex_unlock(&q->mu);
  return m;
}

static void rq_close(ref_queue *q) {
  pthread_mutex_lock(&q->mu);
  q->closed = 1;
  pthread_cond_broadcast(&q->cv);
  pthread_mutex_unlock(&q->mu);
}

typedef struct ref_run ref_run;
typedef struct {
  ref_run *run;
  int64_t my_num;
} ref_machine;

struct ref_run {
  int64_t cs;
  int32_t P;
  uint8_t *flags;
  ref_queue *q;   /* q[0] = relay (machine 1's transfer-primes), q[k-1] = machine k */
  uint64_t nmsg;  /* prime messages (all leads) */
  pthread_mutex_t nmsg_mu;
  int err;        /* first failure (under nmsg_mu); non-zero closes every queue */
};

/* A failed push, thread start or invariant: record the first error and close
 * every queue, so each machine and the relay return instead of waiting for a
 * message that will never come. */
static void ref_fail(ref_run *r, int code) {
  pthread_mutex_lock(&r->nmsg_mu);
  if (!r->err) r->err = code;
  pthread_mutex_unlock(&r->nmsg_mu);
  for (int32_t k = 0; k < r->P; ++k) rq_close(&r->q[k]);
}

static int ref_failed(ref_run *r) {
  pthread_mutex_lock(&r->nmsg_mu);
  const int e = r->err;
  pthread_mutex_unlock(&r->nmsg_mu);
  return e;
}

/* Send a lead's message to machines 2..P (machine 1) or to the relay. */
static int ref_send(ref_run *r, int64_t m, ref_msg msg) {
  if (m == 1) {
    for (int64_t k = 2; k <= r->P; ++k)
      if (rq_push(&r->q[k - 1], msg)) return REF_ENOMEM;
    return REF_OK;
  }
  return rq_push(&r->q[0], msg);
}

/* Lead phase of machine m (sieve.clj:131-150). */
static void ref_lead(ref_run *r, int64_t m) {
  const int64_t cs = r->cs;
  uint8_t *own = r->flags + (size_t)(m - 1) * (size_t)cs;
  uint64_t sent = 0;
  int64_t start = ref_find_first_prime(own, cs);
  for (;;) {
    int64_t n_start = ref_find_next_non_zero(own, start, cs);
    if (n_start < 0) break;
    if (start >= cs || own[start] == 0) { ref_fail(r, REF_EINTERNAL); return; }
    ref_msg msg = {m, start, 3 + 2 * ((m - 1) * cs + start)};
    if (ref_send(r, m, msg)) { ref_fail(r, REF_ENOMEM); return; }
    ++sent;
    ref_mark_composites(m, cs, start, msg.p, m, own);
    start = n_start;
    if ((sent & 1023) == 0 && ref_failed(r)) return;
  }
  ref_msg appoint = {m, -1, 0};
  if (ref_send(r, m, appoint)) { ref_fail(r, REF_ENOMEM); return; }
  pthread_mutex_lock(&r->nmsg_mu);
  r->nmsg += sent;
  pthread_mutex_unlock(&r->nmsg_mu);
}

static void *ref_machine_main(void *arg) {
  ref_machine *mc = (ref_machine *)arg;
  ref_run *r = mc->run;
  const int64_t m = mc->my_num;
  uint8_t *own = r->flags + (size_t)(m - 1) * (size_t)r->cs;
  if (m > 1) {
    for (;;) { /* follower loop, sieve.clj:154-171 */
      ref_msg msg = rq_pop(&r->q[m - 1]);
      if (msg.mi == REF_MSG_CLOSED.mi) return NULL; /* the run failed elsewhere */
      if (msg.ps == -1) {
        if (msg.mi == m - 1) break; /* appointed */
        continue;
      }
      ref_mark_composites(msg.mi, r->cs, msg.ps, msg.p, m, own);
    }
  }
  ref_lead(r, m);
  return NULL;
}

/* machine 1's transfer-primes handler (core.clj:118-134) */
static void *ref_relay_main(void *arg) {
  ref_run *r = (ref_run *)arg;
  for (;;) {
    ref_msg msg = rq_pop(&r->q[0]);
    if (msg.mi == REF_MSG_CLOSED.mi) return NULL;
    for (int64_t k = msg.mi + 1; k <= r->P; ++k)
      if (rq_push(&r->q[k - 1], msg)) { ref_fail(r, REF_ENOMEM); return NULL; }
    if (msg.ps == -1 && msg.mi == r->P) break;
  }
  return NULL;
}

int ref_sieve_threaded(int64_t n, int32_t P, uint64_t *masks, uint64_t *counts, int64_t *cs_out,
                       uint64_t *msgs) {
  int64_t cs;
  int rc = ref_spread_work(n, P, NULL, &cs);
  if (rc) return rc;
  if (cs_out) *cs_out = cs;
  if (cs < 1) return REF_EINVAL;
  ref_run r;
  memset(&r, 0, sizeof(r));
  r.cs = cs;
  r.P = P;
  r.flags = (uint8_t *)malloc((size_t)P * (size_t)cs);
  r.q = (ref_queue *)calloc((size_t)P, sizeof(ref_queue));
  ref_machine *mc = (ref_machine *)calloc((size_t)P, sizeof(ref_machine));
  pthread_t *th = (pthread_t *)calloc((size_t)P + 1, sizeof(pthread_t));
  if (!r.flags || !r.q || !mc || !th) { free(r.flags); free(r.q); free(mc); free(th); return REF_ENOMEM; }
  memset(r.flags, 1, (size_t)P * (size_t)cs); /* gen-table */
  int32_t nq = 0;
  while (nq < P && rq_init(&r.q[nq]) == REF_OK) ++nq;
  if (nq < P) {
    for (int32_t k = 0; k < nq; ++k) rq_free(&r.q[k]);
    free(r.flags); free(r.q); free(mc); free(th);
    return REF_ENOMEM;
  }
  pthread_mutex_init(&r.nmsg_mu, NULL);
  /* st[k]: thread k is running and must be joined (st[P] = the relay) */
  uint8_t *st = (uint8_t *)calloc((size_t)P + 1, 1);
  if (!st) ref_fail(&r, REF_ENOMEM);
  for (int32_t k = 0; st && k < P; ++k) {
    mc[k].run = &r;
    mc[k].my_num = k + 1;
    if (pthread_create(&th[k], NULL, ref_machine_main, &mc[k]) != 0) { ref_fail(&r, REF_EINTERNAL); break; }
    st[k] = 1;
  }
  if (st && P > 1 && !ref_failed(&r)) {
    if (pthread_create(&th[P], NULL, ref_relay_main, &r) != 0) ref_fail(&r, REF_EINTERNAL);
    else st[P] = 1;
  }
  for (int32_t k = 0; st && k <= P; ++k)
    if (st[k]) pthread_join(th[k], NULL);
  free(st);
  rc = r.err;
  if (!rc) {
    int64_t words = (cs + 63) / 64;
    for (int32_t k = 0; k < P; ++k) {
      uint64_t c = popcount_flags_to_mask(r.flags + (size_t)k * (size_t)cs, cs,
                                          masks ? masks + (size_t)k * (size_t)words : NULL);
      if (counts) counts[k] = c;
    }
    if (msgs) *msgs = r.nmsg;
  }
  for (int32_t k = 0; k < P; ++k) rq_free(&r.q[k]);
  pthread_mutex_destroy(&r.nmsg_mu);
  free(r.flags);
  free(r.q);
  free(mc);
  free(th);
  return rc;
}

/* ---------------------------------------------------------------------
 * fast_count_window: number of primes among the odd values in [lo, hi]
 * (lo >= 3), for high windows such as [1e18, 1e18 + 1e10] (SURVEY.md
 * 8(a) a11). Independent of the GPU path: threads own contiguous slices of
 * the window as plain bit arrays; primes below 2^22 are sieved in
 * cache-sized segments with offsets carried from segment to segment, the
 * larger ones (up to 1e9 for that window) mark their multiples directly.
 * --------------------------------------------------------------------- */
static uint64_t mulmod_u64(uint64_t a, uint64_t b, uint64_t m) {
  return (uint64_t)(((unsigned __int128)a * b) % m);
}

/* first odd-index offset >= 0 (value a + 2*off) divisible by p, p odd, values
 * a odd; the multiple must be >= p*p */
static uint64_t first_off(uint64_t a, uint64_t p) {
  uint64_t v = a;
  uint64_t p2 = p * p;
  if (v < p2) v = p2;
  uint64_t r = v % p;
  uint64_t w = r ? v + (p - r) : v;
  if (!(w & 1)) w += p;
  return (w - a) / 2;
}

int fast_count_window(uint64_t lo, uint64_t hi, uint64_t *count) {
  if (!count) return REF_EINVAL;
  *count = 0;
  uint64_t a = lo < 3 ? 3 : lo;
  if (!(a & 1)) ++a;
  if (hi < a) return REF_OK;
  uint64_t b = (hi & 1) ? hi : hi - 1;
  uint64_t nb = (b - a) / 2 + 1; /* odd values a, a+2, ..., b */
  uint64_t np;
  uint32_t *pr = fast_base_primes(isqrt_u64(b), &np);
  if (!pr) return REF_ENOMEM;
  const uint64_t SMALL = 1ull << 22, SEG = 1ull << 21; /* bits */
  uint64_t nsmall = 0;
  while (nsmall < np && pr[nsmall] < SMALL) ++nsmall;
  uint64_t total = 0;
  int err = 0;
  (void)mulmod_u64;
#pragma omp parallel reduction(+ : total)
  {
    int nt = 1, t = 0;
#ifdef _OPENMP
    nt = omp_get_num_threads();
    t = omp_get_thread_num();
#endif
    uint64_t per = (nb + (uint64_t)nt - 1) / (uint64_t)nt;
    per = (per + 63) & ~63ull;
    uint64_t s0 = per * (uint64_t)t, s1 = s0 + per < nb ? s0 + per : nb;
    if (s0 < s1) {
      uint64_t len = s1 - s0, words = (len + 63) / 64;
      uint64_t *bits = (uint64_t *)calloc(words, 8); /* 1 = composite */
      uint64_t *off = (uint64_t *)malloc((nsmall ? nsmall : 1) * 8);
      if (!bits || !off) {
#pragma omp atomic write
        err = REF_ENOMEM;
      } else {
        const uint64_t va = a + 2 * s0; /* value of bit 0 */
        for (uint64_t i = 0; i < nsmall; ++i) off[i] = first_off(va, pr[i]);
        for (uint64_t g = 0; g < len; g += SEG) { /* small primes, segment by segment */
          uint64_t ge = g + SEG < len ? g + SEG : len;
          for (uint64_t i = 0; i < nsmall; ++i) {
            uint64_t o = off[i], p = pr[i];
            for (; o < ge; o += p) bits[o >> 6] |= 1ull << (o & 63);
            off[i] = o;
          }
        }
        for (uint64_t i = nsmall; i < np; ++i) { /* large primes: direct */
          uint64_t p = pr[i];
          if (p * p > va + 2 * (len - 1)) break;
          for (uint64_t o = first_off(va, p); o < len; o += p) bits[o >> 6] |= 1ull << (o & 63);
        }
        uint64_t c = 0;
        for (uint64_t w = 0; w < words; ++w) {
          uint64_t v = ~bits[w];
          if (w == words - 1 && (len & 63)) v &= (1ull << (len & 63)) - 1;
          c += (uint64_t)__builtin_popcountll(v);
        }
        /* values that are small primes themselves (windows starting below
         * sqrt(hi)): first_off starts at p*p, so p stays unmarked; 1 is not odd
         * prime but a >= 3 excludes it */
        total += c;
      }
      free(bits);
      free(off);
    }
  }
  free(pr);
  if (err) return err;
  *count = total;
  return REF_OK;
}

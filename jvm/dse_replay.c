/*
 * dse_replay.c -- replays, from C, exactly the libdse.so calls that the JVM
 * glue (jvm/src/mail_sieve_e/dse.clj, the drop-in for mail-sieve-e.sieve)
 * makes for one machine of the reference's run, in its order:
 *   s/spread-work (core.clj:151)      dse_spread_work -> the machine's [lo hi]
 *                                     (the lead hands it out; core.clj:154-161)
 *   s/gen-table   (core.clj:152,192)  g_start = (lo-3)/2, nbits = (hi-lo)/2
 *   s/sieve-e     (core.clj:163,196)  dse_device_count -> dse_init_device((my-num-1) mod count)
 *                                     -> dse_sieve_odd_range(g_start, nbits), then the lead's lines
 *                                     [my-num j prime] + [my-num -1 0] (sieve.clj:131-148)
 *   finish        (sieve.clj:150)     dse_write_range_file(primes{my-num}.txt)
 *   close!                            dse_destroy
 *
 * usage: dse_replay lead   <n> <P> <out-dir> [lines-file]
 *        dse_replay client <n> <P> <my-num> <out-dir> [lines-file]
 * lines-file receives the lines the glue puts on out-channel, as the
 * reference's write-handler prints them (str of the vector; the prime is a
 * Java Double in chunk 1). Prints "<my-num> <count>" on success; exits
 * non-zero with dse_last_error().
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dse.h"

static int die(const char *where) {
  fprintf(stderr, "%s: %s\n", where, dse_last_error());
  return 1;
}

/* java.lang.Double.toString of an integer-valued double 1 <= v < 2^53, as
 * Clojure's str prints it: "4999.0", "1.0000019E7". */
static void java_double(uint64_t v, char *out) {
  char d[24];
  int len = snprintf(d, sizeof d, "%llu", (unsigned long long)v);
  if (v < 10000000ull) {
    snprintf(out, 32, "%s.0", d);
    return;
  }
  int sig = len;
  while (sig > 1 && d[sig - 1] == '0') --sig;
  int n = 0;
  out[n++] = d[0];
  out[n++] = '.';
  if (sig == 1) out[n++] = '0';
  for (int i = 1; i < sig; ++i) out[n++] = d[i];
  snprintf(out + n, 32 - (size_t)n, "E%d", len - 1);
}

int main(int argc, char **argv) {
  const int lead = (argc == 5 || argc == 6) && strcmp(argv[1], "lead") == 0;
  const int client = (argc == 6 || argc == 7) && strcmp(argv[1], "client") == 0;
  if (!lead && !client) {
    fprintf(stderr, "usage: %s lead <n> <P> <dir> [lines] | client <n> <P> <my-num> <dir> [lines]\n", argv[0]);
    return 2;
  }
  const int64_t n = strtoll(argv[2], NULL, 10);
  const int32_t P = (int32_t)strtol(argv[3], NULL, 10);
  const int32_t my_num = lead ? 1 : (int32_t)strtol(argv[4], NULL, 10);
  const char *dir = argv[lead ? 4 : 5];
  const char *lines_path = argc == (lead ? 6 : 7) ? argv[lead ? 5 : 6] : NULL;
  if (P < 1 || my_num < 1 || my_num > P) {
    fprintf(stderr, "my-num must be in 1..P\n");
    return 2;
  }

  /* s/spread-work: the bounds the lead computes and writes to machine my_num */
  int64_t cs = 0;
  int64_t *lo_hi = (int64_t *)calloc(2 * (size_t)P, sizeof(int64_t));
  if (!lo_hi) return 1;
  if (dse_spread_work(n, P, lo_hi, &cs) != DSE_OK) return die("dse_spread_work");
  const int64_t lo = lo_hi[2 * (my_num - 1)], hi = lo_hi[2 * (my_num - 1) + 1];
  /* s/gen-table */
  const uint64_t g_start = (uint64_t)((lo - 3) / 2), nbits = hi > lo ? (uint64_t)((hi - lo) / 2) : 0;
  /* s/sieve-e: the machine's GPU, the chunk from its bounds */
  const int32_t ndev = dse_device_count();
  dse_ctx *ctx = dse_init_device((my_num - 1) % (ndev > 0 ? ndev : 1));
  if (!ctx) return die("dse_init_device");
  const size_t words = (size_t)(nbits + 63) / 64;
  uint64_t *mask = (uint64_t *)calloc(words ? words : 1, sizeof(uint64_t));
  if (!mask) return 1;
  uint64_t count = 0;
  if (dse_sieve_odd_range(ctx, g_start, nbits, mask, &count) != DSE_OK) return die("dse_sieve_odd_range");
  if (lines_path) { /* lead!: what sieve-e puts on out-channel while it leads */
    FILE *lf = fopen(lines_path, "wb");
    if (!lf) return 1;
    char v[32];
    for (size_t w = 0; w < words; ++w)
      for (uint64_t b = mask[w]; b; b &= b - 1) {
        const uint64_t j = 64 * w + (uint64_t)__builtin_ctzll(b);
        if (j >= nbits) break;
        const uint64_t p = (uint64_t)lo + 2 * j;
        if (my_num == 1) java_double(p, v);
        else snprintf(v, sizeof v, "%llu", (unsigned long long)p);
        fprintf(lf, "[%d %llu %s]\n", (int)my_num, (unsigned long long)j, v);
      }
    fprintf(lf, "[%d -1 0]\n", (int)my_num);
    if (fclose(lf) != 0) return 1;
  }
  /* finish */
  char path[4096];
  snprintf(path, sizeof path, "%s/primes%d.txt", dir, (int)my_num);
  if (dse_write_range_file(path, my_num, g_start, nbits, mask) != DSE_OK) return die("dse_write_range_file");
  dse_destroy(ctx);
  printf("%d %llu\n", (int)my_num, (unsigned long long)count);
  free(mask);
  free(lo_hi);
  return 0;
}

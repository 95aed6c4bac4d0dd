/*
 * dse_replay.c -- replays, from C, exactly the libdse.so calls that the JVM
 * glue (jvm/src/mail_sieve_e/dse.clj, run-machine!) makes for one machine of
 * the reference's run:
 *   lead-start   (core.clj:151-152,163 -> sieve.clj:150):  my_num = 1
 *   client-start (core.clj:192,196     -> sieve.clj:150):  my_num = k
 * call sequence: dse_init -> dse_spread_work -> dse_sieve_chunk ->
 * dse_write_primes_file -> dse_destroy.
 *
 * usage: dse_replay lead   <num-primes> <num-expected> <out-dir>
 *        dse_replay client <num-primes> <num-expected> <my-num> <out-dir>
 * Prints "<my-num> <count>" on success; exits non-zero with dse_last_error().
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

int main(int argc, char **argv) {
  int lead = argc == 5 && strcmp(argv[1], "lead") == 0;
  int client = argc == 6 && strcmp(argv[1], "client") == 0;
  if (!lead && !client) {
    fprintf(stderr, "usage: %s lead <n> <P> <dir> | client <n> <P> <my-num> <dir>\n", argv[0]);
    return 2;
  }
  const int64_t n = strtoll(argv[2], NULL, 10);
  const int32_t P = (int32_t)strtol(argv[3], NULL, 10);
  const int32_t my_num = lead ? 1 : (int32_t)strtol(argv[4], NULL, 10);
  const char *dir = argv[lead ? 4 : 5];

  dse_ctx *ctx = dse_init(1);
  if (!ctx) return die("dse_init");
  int64_t cs = 0;
  int64_t *lo_hi = (int64_t *)calloc(2 * (size_t)P, sizeof(int64_t));
  if (!lo_hi) return 1;
  if (dse_spread_work(n, P, lo_hi, &cs) != DSE_OK) return die("dse_spread_work");
  uint64_t *mask = (uint64_t *)calloc(((size_t)cs + 63) / 64 + 1, sizeof(uint64_t));
  if (!mask) return 1;
  uint64_t count = 0;
  if (dse_sieve_chunk(ctx, n, P, my_num, mask, &count) != DSE_OK) return die("dse_sieve_chunk");
  char path[4096];
  snprintf(path, sizeof path, "%s/primes%d.txt", dir, (int)my_num);
  if (dse_write_primes_file(path, my_num, n, P, mask) != DSE_OK) return die("dse_write_primes_file");
  dse_destroy(ctx);
  printf("%d %llu\n", (int)my_num, (unsigned long long)count);
  free(mask);
  free(lo_hi);
  return 0;
}

/*
 * gen_hll_redo.c -- TEST INFRASTRUCTURE (run by make_hll_redo_values.py, never shipped).
 *
 * Searches for values whose Spark XXH64 (seed 42) has bits 54..32 all zero: for those the HLL rank
 * pw = nlz((x << 9) | 256) + 1 (StatefulHyperloglogPlus.scala:96-113) is not determined by the hash's
 * high word alone, so the GPU kernels take their exact-rank redo path (p = 2^-23 per random value).
 * XXH64 comes from the oracle's C restatement (oracle/c/dq_oracle.c), included as source.
 *
 *   gen_hll_redo i64 <start> <count> <want>        int64 values start, start + 1, ...
 *   gen_hll_redo f64 <start> <count> <want>        finite doubles with bit patterns mix(k)
 *   gen_hll_redo i32 <start> <count> <want>        int32 values (int32_t)k, k = start, start + 1, ... (hashInt)
 *   gen_hll_redo str <len> <start> <count> <want>  strings of <len> bytes from counter k
 * Prints one hit per line (the value, or the string as hex).
 */
#include "../../oracle/c/dq_oracle.c"

#include <stdio.h>

static int redo(uint64_t h) { return ((h >> 32) & 0x7FFFFFu) == 0; }

/* splitmix64: spreads counter k over all 64 bits */
static uint64_t mix(uint64_t k) {
  uint64_t z = k + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* string k of len bytes: printable base-64 digits of mix(k) (and of mix(k + 2^40) past 10 bytes) */
static void make_str(uint64_t k, int len, uint8_t* out) {
  static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
  uint64_t a = mix(k), b = mix(k + (1ull << 40)), c = mix(k + (2ull << 40)), d = mix(k + (3ull << 40));
  uint64_t w[4] = {a, b, c, d};
  for (int i = 0; i < len; ++i) out[i] = (uint8_t)A[(w[(i / 10) & 3] >> (6 * (i % 10))) & 63];
}

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  int found = 0;
  if (!strcmp(argv[1], "i32")) {
    const uint64_t start = strtoull(argv[2], 0, 0), count = strtoull(argv[3], 0, 0);
    const int want = atoi(argv[4]);
    for (uint64_t k = start; k < start + count && found < want; ++k) {
      if (redo(dqo_xxh64_int((int32_t)(uint32_t)k, 42))) {
        printf("%d\n", (int32_t)(uint32_t)k);
        ++found;
      }
    }
  } else if (!strcmp(argv[1], "i64") || !strcmp(argv[1], "f64")) {
    const int is_f = argv[1][0] == 'f';
    const uint64_t start = strtoull(argv[2], 0, 0), count = strtoull(argv[3], 0, 0);
    const int want = atoi(argv[4]);
    for (uint64_t k = start; k < start + count && found < want; ++k) {
      uint64_t v = is_f ? mix(k) : k;
      if (is_f) {
        double d;
        memcpy(&d, &v, 8);
        if (!isfinite(d)) continue;
      }
      if (redo(dqo_xxh64_long((int64_t)v, 42))) {
        if (is_f) printf("%016llx\n", (unsigned long long)v);
        else printf("%lld\n", (long long)v);
        ++found;
      }
    }
  } else {
    if (argc < 6) return 2;
    const int len = atoi(argv[2]);
    const uint64_t start = strtoull(argv[3], 0, 0), count = strtoull(argv[4], 0, 0);
    const int want = atoi(argv[5]);
    uint8_t buf[64];
    for (uint64_t k = start; k < start + count && found < want; ++k) {
      make_str(k, len, buf);
      if (redo(dqo_xxh64_bytes(buf, len, 42))) {
        for (int i = 0; i < len; ++i) printf("%02x", buf[i]);
        printf("\n");
        ++found;
      }
    }
  }
  fflush(stdout);
  return 0;
}

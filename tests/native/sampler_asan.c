/* Host sanitizer driver for the legacy-MT19937 sampler (csrc/sampler.cpp): exercises
 * every argument path of dopt_mt_choice / dopt_mt_choice_rounds / dopt_mt_advance_rounds under
 * -fsanitize=address,undefined (tests/test_sanitizers.py builds and runs it). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dopt.h"

static void seed_key(uint32_t* key, int32_t* pos, uint32_t s) {
  for (int i = 0; i < 624; ++i) key[i] = s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
  *pos = 624;
}

int main(void) {
  uint32_t key[624];
  int32_t pos;
  seed_key(key, &pos, 203u);
  const int64_t ms[] = {0, 1, 2, 7, 500, 4096, 70000};
  const int64_t bs[] = {0, 1, 16, 500, 100000};
  for (size_t a = 0; a < sizeof(ms) / sizeof(ms[0]); ++a)
    for (size_t b = 0; b < sizeof(bs) / sizeof(bs[0]); ++b) {
      const int64_t m = ms[a], bb = bs[b];
      const int64_t eb = m < bb ? m : bb;
      int64_t* out = (int64_t*)malloc((size_t)(eb > 0 ? eb : 1) * sizeof(int64_t));
      if (dopt_mt_choice(key, &pos, m, bb, out) != DOPT_OK) return 1;
      for (int64_t k = 0; k < eb && m > 0; ++k)
        if (out[k] < 0 || out[k] >= m) return 2;
      free(out);
    }
  /* rounds: ragged and empty shards, -1 padding */
  const int64_t rows[] = {3, 0, 500, 17, 1};
  const int64_t T = 5, n = 5, b = 8;
  int32_t* idx = (int32_t*)malloc((size_t)(T * n * b) * sizeof(int32_t));
  if (dopt_mt_choice_rounds(key, &pos, T, n, rows, b, idx) != DOPT_OK) return 3;
  for (int64_t t = 0; t < T; ++t)
    for (int64_t i = 0; i < n; ++i)
      for (int64_t k = 0; k < b; ++k) {
        const int32_t v = idx[(t * n + i) * b + k];
        const int64_t eb = rows[i] < b ? rows[i] : b;
        if (k < eb ? (v < 0 || v >= rows[i]) : v != -1) return 4;
      }
  free(idx);
  /* the parallel stream advance (uniform shards), small segments so every stitch path runs;
   * compared with the sequential advance of the same stream */
  {
    uint32_t k1[624], k2[624];
    int32_t p1 = pos, p2 = pos;
    memcpy(k1, key, sizeof(k1));
    memcpy(k2, key, sizeof(k2));
    const int64_t urows[] = {512, 0, 512, 1, 512, 512};
    setenv("DOPT_MT_SEG_BLOCKS", "40", 1);
    setenv("DOPT_MT_WIN_BLOCKS", "12", 1);
    setenv("DOPT_MT_THREADS", "3", 1);
    if (dopt_mt_advance_rounds(k1, &p1, 30, 6, urows) != DOPT_OK) return 9;
    setenv("DOPT_MT_THREADS", "0", 1);
    if (dopt_mt_advance_rounds(k2, &p2, 30, 6, urows) != DOPT_OK) return 10;
    if (p1 != p2 || memcmp(k1, k2, sizeof(k1)) != 0) return 11;
    /* minibatch draws through the parallel path vs the sequential one */
    {
      int32_t* i1 = (int32_t*)malloc(30 * 6 * 4 * sizeof(int32_t));
      int32_t* i2 = (int32_t*)malloc(30 * 6 * 4 * sizeof(int32_t));
      memcpy(k2, k1, sizeof(k1));
      p2 = p1;
      setenv("DOPT_MT_THREADS", "3", 1);
      if (dopt_mt_choice_rounds(k1, &p1, 30, 6, urows, 4, i1) != DOPT_OK) return 12;
      setenv("DOPT_MT_THREADS", "0", 1);
      if (dopt_mt_choice_rounds(k2, &p2, 30, 6, urows, 4, i2) != DOPT_OK) return 13;
      if (p1 != p2 || memcmp(k1, k2, sizeof(k1)) != 0 || memcmp(i1, i2, 30 * 6 * 4 * sizeof(int32_t)) != 0) return 14;
      free(i1);
      free(i2);
    }
    unsetenv("DOPT_MT_SEG_BLOCKS");
    unsetenv("DOPT_MT_WIN_BLOCKS");
    unsetenv("DOPT_MT_THREADS");
  }
  /* invalid arguments are rejected, not dereferenced */
  if (dopt_mt_choice(NULL, &pos, 5, 2, NULL) == DOPT_OK) return 5;
  int32_t bad = 625;
  int64_t one;
  if (dopt_mt_choice(key, &bad, 5, 1, &one) == DOPT_OK) return 6;
  if (dopt_mt_choice_rounds(key, &pos, 1, 2, NULL, 1, NULL) == DOPT_OK) return 7;
  const int64_t neg[] = {-1};
  int32_t o1;
  if (dopt_mt_choice_rounds(key, &pos, 1, 1, neg, 1, &o1) == DOPT_OK) return 8;
  puts("sampler asan ok");
  return 0;
}

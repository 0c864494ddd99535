/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. A standalone driver that runs every oracle entry point over
 * seeded random inputs (empty, ragged, sentinel-holding, duplicate-holding) so that the oracle can be
 * built and run under AddressSanitizer + UndefinedBehaviorSanitizer, and its multi-thread forms under
 * ThreadSanitizer (tests/test_sanitizers.py, oracle/Makefile targets asan / tsan). It checks a few
 * invariants on the way; the sanitizers check the rest. Exit status 0 = clean.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (uint32_t)(rs >> 16);
}

#define CHECK(x)                                                  \
  do {                                                            \
    if (!(x)) {                                                   \
      fprintf(stderr, "check failed: %s (line %d)\n", #x, __LINE__); \
      exit(1);                                                    \
    }                                                             \
  } while (0)

static int cmp_u32(const void* a, const void* b) {
  const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return (x > y) - (x < y);
}

/* a random corpus: n covers of up to maxlen sorted unique PCs below space (some with the sentinel) */
static void corpus(size_t n, uint32_t maxlen, uint32_t space, uint32_t G, uint32_t** pcs, uint64_t** off,
                   uint32_t** group) {
  *off = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
  *group = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  uint32_t* buf = (uint32_t*)malloc(((size_t)n * maxlen + 1) * sizeof(uint32_t));
  uint64_t L = 0;
  (*off)[0] = 0;
  for (size_t i = 0; i < n; i++) {
    const uint32_t len = maxlen ? rnd() % (maxlen + 1) : 0;
    uint32_t* c = buf + L;
    for (uint32_t k = 0; k < len; k++) c[k] = rnd() % space;
    qsort(c, len, 4, cmp_u32);
    size_t u = 0;
    for (uint32_t k = 0; k < len; k++)
      if (!u || c[u - 1] != c[k]) c[u++] = c[k];
    if (u && rnd() % 17 == 0) c[u - 1] = 0xFFFFFFFFu;
    L += u;
    (*off)[i + 1] = L;
    (*group)[i] = rnd() % G;
  }
  *pcs = buf;
}

static void run_setops(void) {
  for (int it = 0; it < 200; it++) {
    const size_t na = rnd() % 50, nb = rnd() % 50;
    uint32_t a[64], b[64], out[128];
    for (size_t i = 0; i < na; i++) a[i] = rnd() % 80;
    for (size_t i = 0; i < nb; i++) b[i] = rnd() % 80;
    qsort(a, na, 4, cmp_u32);
    qsort(b, nb, 4, cmp_u32);
    for (int op = 0; op < 4; op++) {
      size_t n = 0;
      CHECK(oracle_setop(op, a, na, b, nb, out, na + nb, &n) == 0);
      CHECK(n <= na + nb);
    }
    size_t n = 0;
    CHECK(oracle_canonicalize(a, na, &n) == 0 && n <= na);
  }
}

static void run_minimize(void) {
  for (int it = 0; it < 20; it++) {
    const size_t n = rnd() % 3000;
    const uint32_t G = 1 + rnd() % 40;
    uint32_t *pcs, *group;
    uint64_t* off;
    corpus(n, 1 + rnd() % 200, 1 + rnd() % 5000, G, &pcs, &off, &group);
    int64_t* out = (int64_t*)malloc((n + 1) * 8);
    int64_t* out2 = (int64_t*)malloc((n + 1) * 8);
    uint64_t* goff = (uint64_t*)malloc((G + 1) * 8);
    uint64_t* goff2 = (uint64_t*)malloc((G + 1) * 8);
    size_t m = 0;
    CHECK(oracle_minimize(pcs, off, n, out, &m) == 0 && m <= n);
    CHECK(oracle_minimize_grouped(pcs, off, group, n, G, out, goff) == 0);
    CHECK(oracle_minimize_grouped_mt(pcs, off, group, n, G, 1 + it % 5, out2, goff2) == 0);
    CHECK(memcmp(goff, goff2, (G + 1) * 8) == 0 && memcmp(out, out2, goff[G] * 8) == 0);
    uint64_t* lens = (uint64_t*)malloc((n + 1) * 8);
    for (size_t i = 0; i < n; i++) lens[i] = off[i + 1] - off[i];
    CHECK(oracle_minimize_order(lens, n, out) == 0);
    /* novelty, literal and first-occurrence forms, against the corpus's first half as maxCover */
    const size_t h = n / 2;
    uint32_t* mc = (uint32_t*)malloc((off[h] + 1) * 4);
    uint64_t* mco = (uint64_t*)calloc(G + 1, 8);
    size_t p = 0;
    for (uint32_t g = 0; g < G; g++) {
      const size_t p0 = p;
      for (size_t i = 0; i < h; i++)
        if (group[i] == g)
          for (uint64_t k = off[i]; k < off[i + 1]; k++) mc[p++] = pcs[k];
      qsort(mc + p0, p - p0, 4, cmp_u32);
      size_t u = p0;
      for (size_t k = p0; k < p; k++)
        if (u == p0 || mc[u - 1] != mc[k]) mc[u++] = mc[k];
      p = u;
      mco[g + 1] = p;
    }
    uint32_t flakes[8];
    for (int f = 0; f < 8; f++) flakes[f] = rnd() % 5000;
    qsort(flakes, 8, 4, cmp_u32);
    const size_t cap = p + off[n] + 1;
    uint8_t* nw = (uint8_t*)malloc(n + 1);
    uint8_t* nw2 = (uint8_t*)malloc(n + 1);
    uint32_t* om = (uint32_t*)malloc(cap * 4);
    uint32_t* om2 = (uint32_t*)malloc(cap * 4);
    uint64_t* oo = (uint64_t*)malloc((G + 1) * 8);
    uint64_t* oo2 = (uint64_t*)malloc((G + 1) * 8);
    CHECK(oracle_novelty(pcs, off, group, n, G, mc, mco, flakes, 8, nw, om, oo, cap) == 0);
    CHECK(oracle_novelty_mt(pcs, off, group, n, G, mc, mco, flakes, 8, 3, nw2, om2, oo2, cap) == 0);
    CHECK(memcmp(nw, nw2, n) == 0 && memcmp(oo, oo2, (G + 1) * 8) == 0 && memcmp(om, om2, oo[G] * 4) == 0);
    /* html.go analytics */
    uint64_t *ci = (uint64_t*)malloc(G * 8), *cc = (uint64_t*)malloc(G * 8), *cu = (uint64_t*)malloc(G * 8);
    uint64_t tot[3];
    uint32_t* iu = (uint32_t*)malloc((n + 1) * 4);
    CHECK(oracle_cover_stats(pcs, off, group, n, G, ci, cc, cu, tot, iu) == 0);
    uint32_t* lst = (uint32_t*)malloc((off[n] + 1) * 4);
    size_t ln = 0;
    CHECK(oracle_corpus_cover(pcs, off, group, n, G, -1, 1, lst, off[n] + 1, &ln) == 0);
    free(ci), free(cc), free(cu), free(iu), free(lst);
    free(nw), free(nw2), free(om), free(om2), free(oo), free(oo2), free(mc), free(mco);
    free(pcs), free(off), free(group), free(out), free(out2), free(goff), free(goff2), free(lens);
  }
}

static void run_prio(void) {
  for (int it = 0; it < 10; it++) {
    const int32_t C = 1 + rnd() % 70;
    const size_t np = rnd() % 500, nk = rnd() % 60;
    uint16_t* pl = (uint16_t*)malloc((np + 1) * 2);
    for (size_t i = 0; i < np; i++) pl[i] = (uint16_t)(rnd() % (C + 1));
    float* st = (float*)malloc((size_t)C * C * 4);
    float* pr = (float*)malloc((size_t)C * C * 4);
    float* uses = (float*)calloc(nk * C + 1, 4);
    static const float w[4] = {0.1f, 0.2f, 0.5f, 1.0f};
    for (size_t i = 0; i < nk * (size_t)C; i++)
      if (rnd() % 5 == 0) uses[i] = w[rnd() % 4];
    CHECK(oracle_static_priorities(uses, nk, C, NULL, 0, st) == 0);
    CHECK(oracle_static_priorities(uses, nk, C, NULL, 1, pr) == 0);
    CHECK(oracle_dynamic_prio(pl, np, C, pr) == 0);
    CHECK(oracle_calculate_priorities(st, pl, np, C, pr) == 0);
    int64_t* run = (int64_t*)malloc((size_t)C * C * 8);
    uint8_t* en = (uint8_t*)malloc(C);
    uint8_t* pres = (uint8_t*)malloc(C);
    for (int32_t i = 0; i < C; i++) en[i] = rnd() % 3 != 0;
    CHECK(oracle_build_choice_table(pr, en, C, run, pres) == 0);
    CHECK(oracle_build_choice_table(pr, NULL, C, run, pres) == 0);
    free(pl), free(st), free(pr), free(uses), free(run), free(en), free(pres);
  }
}

static void run_text(void) {
  static const char* progs[] = {"", "\n", "mmap(&(0x7f0000000000/0x1000)=nil)\n", "r0 = open()\nclose(r0)",
                                "a()\r\nb()\r\n\n", "no bracket\n", "(x)\n", "foo("};
  uint8_t sig[20];
  for (size_t i = 0; i < sizeof(progs) / sizeof(progs[0]); i++) {
    uint32_t nc = 0;
    uint8_t stt = 0;
    oracle_prog_scan((const uint8_t*)progs[i], strlen(progs[i]), &nc, &stt);
    oracle_sha1((const uint8_t*)progs[i], strlen(progs[i]), sig);
  }
  const size_t big = 70 * 1024;  /* a line past bufio.Scanner's 64 KiB token limit */
  uint8_t* b = (uint8_t*)malloc(big);
  memset(b, 'a', big);
  uint32_t nc = 0;
  uint8_t stt = 0;
  oracle_prog_scan(b, big, &nc, &stt);
  oracle_sha1(b, big, sig);
  free(b);
}

int main(int argc, char** argv) {
  const int only_mt = argc > 1 && strcmp(argv[1], "mt") == 0;
  if (!only_mt) {
    run_setops();
    run_prio();
    run_text();
  }
  run_minimize();
  printf("oracle sanitizer run ok\n");
  return 0;
}

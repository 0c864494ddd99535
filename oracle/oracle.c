/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). Plain C restatement of
 *   cover/cover.go            (set algebra, Canonicalize, Minimize)
 *   prog/prio.go              (calcDynamicPrio, normalizePrio, CalculatePriorities, BuildChoiceTable)
 *   syz-manager/manager.go    (minimizeCorpus grouping, NewInput novelty)
 *   syz-fuzzer/fuzzer.go      (execute novelty vs maxCover/flakes)
 * Compiled with -ffp-contract=off and without fast-math: Go on amd64 rounds every float32 op
 * separately.
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "gosort.h"

#define SENT 0xFFFFFFFFu /* cover/cover.go:17 */

/* ---- sort.Sort instantiations ------------------------------------------------------------- */

/* cover/cover.go:13-15  Cover.Less(i, j) = a[i] < a[j] */
#define COVER_LESS(x, y) ((x) < (y))
GOSORT_DEFINE(gosort_cover, uint32_t, COVER_LESS)

/* cover/cover.go:133-143  minInput{idx, cov}; Less(i, j) = len(a[i].cov) > len(a[j].cov) */
typedef struct {
  int64_t idx;
  uint64_t len;
  const uint32_t* cov;
} min_input;
#define MININPUT_LESS(x, y) ((x).len > (y).len)
GOSORT_DEFINE(gosort_mininput, min_input, MININPUT_LESS)

/* ---- cover/cover.go ------------------------------------------------------------------------ */

int oracle_canonicalize(uint32_t* cov, size_t n, size_t* out_n) {
  /* cover.go:29 sort.Sort(Cover(cov)); :30-38 dedup with last = sent */
  gosort_cover(cov, (long)n);
  size_t i = 0;
  uint32_t last = SENT;
  for (size_t k = 0; k < n; k++) {
    uint32_t pc = cov[k];
    if (pc != last) {
      last = pc;
      cov[i++] = pc;
    }
  }
  *out_n = i;
  return 0;
}

static inline uint32_t apply_op(int op, uint32_t v0, uint32_t v1) {
  switch (op) {
    case 0: /* Difference cover.go:42-49 */
      return v0 < v1 ? v0 : SENT;
    case 1: /* SymmetricDifference cover.go:51-61 */
      if (v0 < v1) return v0;
      if (v1 < v0) return v1;
      return SENT;
    case 2: /* Union cover.go:63-70 */
      return v0 <= v1 ? v0 : v1;
    default: /* Intersection cover.go:72-79 */
      return v0 == v1 ? v0 : SENT;
  }
}

int oracle_setop(int op, const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out,
                 size_t cap, size_t* out_n) {
  if (op < 0 || op > 3) return 1;
  /* cover.go:81-102 foreach */
  size_t n = 0;
  for (size_t i0 = 0, i1 = 0; i0 < na || i1 < nb;) {
    uint32_t v0 = SENT, v1 = SENT;
    if (i0 < na) v0 = a[i0];
    if (i1 < nb) v1 = b[i1];
    if (v0 <= v1) i0++;
    if (v1 <= v0) i1++;
    uint32_t v = apply_op(op, v0, v1);
    if (v != SENT) {
      if (n >= cap) return 6;
      out[n++] = v;
    }
  }
  *out_n = n;
  return 0;
}

/* Open-addressing uint32 set standing in for Go's map[uint32]struct{} (cover.go:115). Slots hold
 * key+1 so that every uint32 (including 0 and 0xFFFFFFFF, both legal map keys) is storable. */
typedef struct {
  uint64_t* slot;
  size_t mask, count;
} u32set;

static void u32set_init(u32set* s, size_t hint) {
  size_t cap = 64;
  while (cap < hint * 2) cap <<= 1;
  s->slot = (uint64_t*)calloc(cap, sizeof(uint64_t));
  s->mask = cap - 1;
  s->count = 0;
}
static inline size_t u32hash(uint32_t k) {
  uint64_t h = (uint64_t)k * 0x9E3779B97F4A7C15ull;
  return (size_t)(h >> 32);
}
static void u32set_grow(u32set* s);
static inline int u32set_has(const u32set* s, uint32_t k) {
  for (size_t i = u32hash(k) & s->mask;; i = (i + 1) & s->mask) {
    uint64_t v = s->slot[i];
    if (v == 0) return 0;
    if (v == (uint64_t)k + 1) return 1;
  }
}
static inline void u32set_add(u32set* s, uint32_t k) {
  if ((s->count + 1) * 2 > s->mask + 1) u32set_grow(s);
  for (size_t i = u32hash(k) & s->mask;; i = (i + 1) & s->mask) {
    uint64_t v = s->slot[i];
    if (v == 0) {
      s->slot[i] = (uint64_t)k + 1;
      s->count++;
      return;
    }
    if (v == (uint64_t)k + 1) return;
  }
}
static void u32set_grow(u32set* s) {
  u32set n;
  u32set_init(&n, (s->mask + 1));
  for (size_t i = 0; i <= s->mask; i++)
    if (s->slot[i]) u32set_add(&n, (uint32_t)(s->slot[i] - 1));
  free(s->slot);
  *s = n;
}

static int minimize_core(min_input* inputs, size_t n, int64_t* out_idx, size_t* out_n) {
  /* cover.go:113 sort.Sort(minInputArray(inputs)) */
  gosort_mininput(inputs, (long)n);
  /* cover.go:114-129 greedy selection against a covered-PC map */
  size_t total = 0;
  for (size_t i = 0; i < n; i++) total += inputs[i].len;
  u32set covered;
  u32set_init(&covered, total < 1024 ? 1024 : total / 4);
  size_t m = 0;
  for (size_t i = 0; i < n; i++) {
    int hit = 0;
    const uint32_t* cov = inputs[i].cov;
    for (uint64_t k = 0; k < inputs[i].len; k++) {
      uint32_t pc = cov[k];
      if (!hit) {
        if (!u32set_has(&covered, pc)) {
          hit = 1;
          out_idx[m++] = inputs[i].idx;
        }
      }
      if (hit) u32set_add(&covered, pc);
    }
  }
  free(covered.slot);
  *out_n = m;
  return 0;
}

int oracle_minimize(const uint32_t* pcs, const uint64_t* off, size_t ncov, int64_t* out_idx,
                    size_t* out_n) {
  /* cover.go:106-112 inputs[i] = &minInput{idx: i, cov: cov} */
  min_input* inputs = (min_input*)malloc((ncov ? ncov : 1) * sizeof(min_input));
  for (size_t i = 0; i < ncov; i++) {
    inputs[i].idx = (int64_t)i;
    inputs[i].len = off[i + 1] - off[i];
    inputs[i].cov = pcs + off[i];
  }
  int rc = minimize_core(inputs, ncov, out_idx, out_n);
  free(inputs);
  return rc;
}

/* the leaf form of the restated Go quickSort (gosort.h): 12 (default) or 7; -1 for another value */
int oracle_set_go_sort_leaf(int leaf) {
  if (leaf != 12 && leaf != 7) return -1;
  gosort_leaf = leaf;
  return 0;
}

int oracle_minimize_order(const uint64_t* lens, size_t n, int64_t* perm) {
  min_input* inputs = (min_input*)malloc((n ? n : 1) * sizeof(min_input));
  for (size_t i = 0; i < n; i++) {
    inputs[i].idx = (int64_t)i;
    inputs[i].len = lens[i];
    inputs[i].cov = NULL;
  }
  gosort_mininput(inputs, (long)n);
  for (size_t i = 0; i < n; i++) perm[i] = inputs[i].idx;
  free(inputs);
  return 0;
}

int oracle_minimize_grouped(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                            size_t n, uint32_t ngroups, int64_t* out_idx, uint64_t* group_out_off) {
  /* manager.go:514-520: bucket inputs per call, keeping corpus order inside a bucket */
  uint64_t* cnt = (uint64_t*)calloc((size_t)ngroups + 1, sizeof(uint64_t));
  for (size_t i = 0; i < n; i++) {
    if (group[i] >= ngroups) {
      free(cnt);
      return 1;
    }
    cnt[group[i] + 1]++;
  }
  for (uint32_t g = 0; g < ngroups; g++) cnt[g + 1] += cnt[g];
  uint64_t* fill = (uint64_t*)malloc(((size_t)ngroups + 1) * sizeof(uint64_t));
  memcpy(fill, cnt, ((size_t)ngroups + 1) * sizeof(uint64_t));
  int64_t* members = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
  for (size_t i = 0; i < n; i++) members[fill[group[i]]++] = (int64_t)i;
  min_input* inputs = (min_input*)malloc((n ? n : 1) * sizeof(min_input));
  int64_t* sel = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
  size_t outp = 0;
  group_out_off[0] = 0;
  /* manager.go:522-527: Minimize each bucket, append the kept inputs */
  for (uint32_t g = 0; g < ngroups; g++) {
    size_t ng = (size_t)(cnt[g + 1] - cnt[g]);
    for (size_t i = 0; i < ng; i++) {
      int64_t e = members[cnt[g] + i];
      inputs[i].idx = (int64_t)i;
      inputs[i].len = off[e + 1] - off[e];
      inputs[i].cov = pcs + off[e];
    }
    size_t m = 0;
    minimize_core(inputs, ng, sel, &m);
    for (size_t k = 0; k < m; k++) out_idx[outp++] = members[cnt[g] + sel[k]];
    group_out_off[g + 1] = outp;
  }
  free(cnt);
  free(fill);
  free(members);
  free(inputs);
  free(sel);
  return 0;
}

/* The same minimizeCorpus with the call groups spread over nthreads host threads (SURVEY.md §8d's
 * "stronger" CPU baseline: the groups are independent, manager.go:522-527). Groups are taken largest
 * first from a shared counter; each writes its kept inputs into its own slice, then the slices are
 * concatenated in group order, so the output equals oracle_minimize_grouped's. */
typedef struct {
  const uint32_t* pcs;
  const uint64_t* off;
  const uint64_t* cnt;
  const int64_t* members;
  const uint32_t* order;
  uint32_t ngroups;
  int64_t* sel;      /* group g's kept members at [cnt[g], cnt[g] + kept[g]) */
  uint64_t* kept;
  uint32_t next;     /* next index into order (atomic) */
} mt_job;

static void* mt_worker(void* arg) {
  mt_job* J = (mt_job*)arg;
  size_t cap = 0;
  min_input* inputs = NULL;
  int64_t* loc = NULL;
  for (;;) {
    const uint32_t t = __atomic_fetch_add(&J->next, 1u, __ATOMIC_RELAXED);
    if (t >= J->ngroups) break;
    const uint32_t g = J->order[t];
    const size_t ng = (size_t)(J->cnt[g + 1] - J->cnt[g]);
    if (ng > cap) {
      cap = ng;
      inputs = (min_input*)realloc(inputs, cap * sizeof(min_input));
      loc = (int64_t*)realloc(loc, cap * sizeof(int64_t));
    }
    for (size_t i = 0; i < ng; i++) {
      const int64_t e = J->members[J->cnt[g] + i];
      inputs[i].idx = (int64_t)i;
      inputs[i].len = J->off[e + 1] - J->off[e];
      inputs[i].cov = J->pcs + J->off[e];
    }
    size_t m = 0;
    if (ng) minimize_core(inputs, ng, loc, &m);
    for (size_t k = 0; k < m; k++) J->sel[J->cnt[g] + k] = J->members[J->cnt[g] + loc[k]];
    J->kept[g] = m;
  }
  free(inputs);
  free(loc);
  return NULL;
}

/* (size, group) pairs: a stateless comparator, so concurrent callers share nothing (qsort has no
 * context argument); largest first, ties by group id */
typedef struct {
  uint64_t size;
  uint32_t g;
} group_size;
static int cmp_group_size(const void* a, const void* b) {
  const group_size *x = (const group_size*)a, *y = (const group_size*)b;
  return x->size < y->size ? 1 : x->size > y->size ? -1 : (x->g > y->g) - (x->g < y->g);
}

/* groups in decreasing size order (the LPT order both multi-thread oracles take them in) */
static uint32_t* groups_by_size(const uint64_t* cnt, uint32_t ngroups) {
  group_size* gs = (group_size*)malloc(((size_t)ngroups + 1) * sizeof(group_size));
  for (uint32_t g = 0; g < ngroups; g++) {
    gs[g].size = cnt[g + 1] - cnt[g];
    gs[g].g = g;
  }
  qsort(gs, ngroups, sizeof(group_size), cmp_group_size);
  uint32_t* order = (uint32_t*)malloc(((size_t)ngroups + 1) * sizeof(uint32_t));
  for (uint32_t g = 0; g < ngroups; g++) order[g] = gs[g].g;
  free(gs);
  return order;
}

int oracle_minimize_grouped_mt(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                               uint32_t ngroups, int nthreads, int64_t* out_idx, uint64_t* group_out_off) {
  uint64_t* cnt = (uint64_t*)calloc((size_t)ngroups + 1, sizeof(uint64_t));
  for (size_t i = 0; i < n; i++) {
    if (group[i] >= ngroups) {
      free(cnt);
      return 1;
    }
    cnt[group[i] + 1]++;
  }
  for (uint32_t g = 0; g < ngroups; g++) cnt[g + 1] += cnt[g];
  uint64_t* fill = (uint64_t*)malloc(((size_t)ngroups + 1) * sizeof(uint64_t));
  memcpy(fill, cnt, ((size_t)ngroups + 1) * sizeof(uint64_t));
  int64_t* members = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
  for (size_t i = 0; i < n; i++) members[fill[group[i]]++] = (int64_t)i;
  uint32_t* order = groups_by_size(cnt, ngroups);
  mt_job J = {pcs, off, cnt, members, order, ngroups, (int64_t*)malloc((n ? n : 1) * sizeof(int64_t)),
              (uint64_t*)calloc((size_t)ngroups + 1, sizeof(uint64_t)), 0};
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc((size_t)nthreads * sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, mt_worker, &J);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  size_t outp = 0;
  group_out_off[0] = 0;
  for (uint32_t g = 0; g < ngroups; g++) {
    memcpy(out_idx + outp, J.sel + cnt[g], J.kept[g] * sizeof(int64_t));
    outp += J.kept[g];
    group_out_off[g + 1] = outp;
  }
  free(th);
  free(J.sel);
  free(J.kept);
  free(order);
  free(cnt);
  free(fill);
  free(members);
  return 0;
}

/* ---- prog/prio.go -------------------------------------------------------------------------- */

void oracle_normalize_prio(float* prios, int32_t C) {
  /* prio.go:158-192, every op rounded to float32 separately */
  for (int32_t r = 0; r < C; r++) {
    float* prio = prios + (size_t)r * C;
    float max = 0.0f;
    float min = 1e10f;
    long nzero = 0;
    for (int32_t i = 0; i < C; i++) {
      float p = prio[i];
      if (max < p) max = p;
      if (p != 0 && min > p) min = p;
      if (p == 0) nzero++;
    }
    if (nzero != 0) {
      volatile float den = 2.0f * (float)nzero;
      min /= den;
    }
    for (int32_t i = 0; i < C; i++) {
      float p = prio[i];
      if (max == 0) {
        prio[i] = 1;
        continue;
      }
      if (p == 0) p = min;
      volatile float t1 = p - min;
      volatile float t2 = max - min;
      volatile float t3 = t1 / t2;
      volatile float t4 = t3 * 0.9f;
      p = t4 + 0.1f;
      if (p > 1) p = 1;
      prio[i] = p;
    }
  }
}

int oracle_dynamic_prio(const uint16_t* prog_len, size_t nprogs, int32_t C, float* out) {
  if (C <= 0) return 1;
  for (size_t p = 0; p < nprogs; p++)
    if ((int32_t)prog_len[p] > C) return 1; /* Go: index out of range panic (prio.go:148) */
  memset(out, 0, sizeof(float) * (size_t)C * (size_t)C);
  /* prio.go:142-151: += 1.0 for every ordered pair of call *positions*  */
  for (size_t p = 0; p < nprogs; p++) {
    int32_t L = prog_len[p];
    for (int32_t i0 = 0; i0 < L; i0++)
      for (int32_t i1 = 0; i1 < L; i1++) {
        if (i0 == i1) continue;
        out[(size_t)i0 * C + i1] += 1.0f;
      }
  }
  oracle_normalize_prio(out, C); /* prio.go:152 */
  return 0;
}

/* The call-ID form of prio.go:142-151 (not the reference's quantity): for every
 * program, += 1 at [calls[i0]][calls[i1]] for every ordered pair of distinct positions i0 != i1. The
 * literal loop, exact int32 counts; the checker of syzgpu_call_cooccurrence. */
int oracle_call_cooccurrence(const uint16_t* calls, const uint64_t* off, size_t nprogs, int32_t C, int32_t* out) {
  if (C <= 0) return 1;
  memset(out, 0, sizeof(int32_t) * (size_t)C * (size_t)C);
  for (size_t p = 0; p < nprogs; p++) {
    const uint64_t b = off[p], e = off[p + 1];
    for (uint64_t i0 = b; i0 < e; i0++) {
      if ((int32_t)calls[i0] >= C) return 1;
      for (uint64_t i1 = b; i1 < e; i1++) {
        if (i0 == i1) continue;
        out[(size_t)calls[i0] * C + calls[i1]] += 1;
      }
    }
  }
  return 0;
}

int oracle_calculate_priorities(const float* static_prios, const uint16_t* prog_len, size_t nprogs,
                                int32_t C, float* out) {
  int rc = oracle_dynamic_prio(prog_len, nprogs, C, out); /* prio.go:31 */
  if (rc) return rc;
  /* prio.go:32-36 dynamic[i][j] *= static[i][j] */
  for (size_t k = 0; k < (size_t)C * (size_t)C; k++) {
    volatile float v = out[k] * static_prios[k];
    out[k] = v;
  }
  return 0;
}

/* prio.go:40-135 calcStaticPriorities from its `uses` map as a dense nkeys x C matrix (0 = unused).
 * exact == 0: the Go loop (:110-120) with the keys taken in key_order (NULL: 0..nkeys-1) standing in
 *   for Go's map iteration order, which Go randomises per run: float32 products added into float32
 *   sums, so results differ in the last bits between orders, as Go's own runs do.
 * exact == 1: the sum every such order approximates: per pair of weight classes (distinct non-zero
 *   weights, ascending) the count of keys, times the float32 product of the two weights, added in
 *   float64 in (class, class) order and rounded once (what syzgpu_static_priorities computes).
 * Then self-priority = row max (:124-132) and normalizePrio (:133). */
#define ST_KMAX 8
int oracle_static_priorities(const float* uses, size_t nkeys, int32_t C, const int64_t* key_order, int exact,
                             float* out) {
  if (C <= 0) return 1;
  const size_t CC = (size_t)C * C;
  memset(out, 0, CC * sizeof(float));
  if (!exact) {
    for (size_t t = 0; t < nkeys; t++) {
      const size_t k = key_order ? (size_t)key_order[t] : t;
      if (k >= nkeys) return 1;
      const float* w = uses + k * (size_t)C;
      for (int32_t c0 = 0; c0 < C; c0++) {
        if (w[c0] == 0) continue;
        for (int32_t c1 = 0; c1 < C; c1++) {
          if (w[c1] == 0 || c0 == c1) continue; /* :113-116 */
          volatile float prod = w[c0] * w[c1];
          volatile float sum = out[(size_t)c0 * C + c1] + prod;
          out[(size_t)c0 * C + c1] = sum;
        }
      }
    }
  } else {
    float cls[ST_KMAX];
    int nk = 0;
    for (size_t i = 0; i < nkeys * (size_t)C; i++) {
      const float w = uses[i];
      if (w == 0) continue;
      if (!isfinite(w)) return 1;
      int j = 0;
      while (j < nk && cls[j] != w) j++;
      if (j == nk) {
        if (nk == ST_KMAX) return 1;
        cls[nk++] = w;
      }
    }
    for (int i = 1; i < nk; i++)
      for (int j = i; j > 0 && cls[j - 1] > cls[j]; j--) {
        const float t = cls[j];
        cls[j] = cls[j - 1];
        cls[j - 1] = t;
      }
    uint32_t* cnt = (uint32_t*)calloc((size_t)nk * nk * CC + 1, sizeof(uint32_t));
    int32_t* kc = (int32_t*)malloc(((size_t)C + 1) * sizeof(int32_t));
    int8_t* ka = (int8_t*)malloc(((size_t)C + 1) * sizeof(int8_t));
    for (size_t k = 0; k < nkeys; k++) {
      const float* w = uses + k * (size_t)C;
      int m = 0;
      for (int32_t c = 0; c < C; c++) {
        if (w[c] == 0) continue;
        int a = 0;
        while (cls[a] != w[c]) a++;
        kc[m] = c;
        ka[m] = (int8_t)a;
        m++;
      }
      for (int x = 0; x < m; x++)
        for (int y = 0; y < m; y++)
          if (x != y) cnt[((size_t)ka[x] * nk + ka[y]) * CC + (size_t)kc[x] * C + kc[y]]++;
    }
    for (size_t e = 0; e < CC; e++) {
      double acc = 0.0;
      for (int a = 0; a < nk; a++)
        for (int b = 0; b < nk; b++) {
          volatile float p = cls[a] * cls[b];
          acc += (double)cnt[((size_t)a * nk + b) * CC + e] * (double)p;
        }
      out[e] = (float)acc;
    }
    free(cnt);
    free(kc);
    free(ka);
  }
  for (int32_t c0 = 0; c0 < C; c0++) { /* :124-132 */
    float* pp = out + (size_t)c0 * C;
    float max = 0;
    for (int32_t j = 0; j < C; j++)
      if (max < pp[j]) max = pp[j];
    pp[c0] = max;
  }
  oracle_normalize_prio(out, C);
  return 0;
}

/* Go on amd64 converts float32 -> int with CVTTSS2SQ: truncation toward zero; NaN and
 * out-of-range values give the "integer indefinite" 0x8000000000000000. */
static inline int64_t go_f32_to_int(float x) {
  if (x != x) return INT64_MIN;
  if (x >= 9223372036854775808.0f || x < -9223372036854775808.0f) return INT64_MIN;
  return (int64_t)x;
}

int oracle_build_choice_table(const float* prios, const uint8_t* enabled, int32_t C, int64_t* run,
                              uint8_t* row_present) {
  if (C <= 0) return 1;
  /* prio.go:213-226 */
  for (int32_t i = 0; i < C; i++) {
    int64_t* row = run + (size_t)i * C;
    if (enabled && !enabled[i]) {
      row_present[i] = 0;
      memset(row, 0, sizeof(int64_t) * (size_t)C);
      continue;
    }
    row_present[i] = 1;
    uint64_t sum = 0; /* Go int arithmetic wraps */
    for (int32_t j = 0; j < C; j++) {
      if (!enabled || enabled[j]) {
        volatile float t = prios[(size_t)i * C + j] * 1000.0f;
        sum += (uint64_t)go_f32_to_int(t);
      }
      row[j] = (int64_t)sum;
    }
  }
  return 0;
}

/* ---- syz-fuzzer/fuzzer.go:446-470 execute (novelty vs maxCover/flakes) ---------------------- */

int oracle_novelty(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                   uint32_t ngroups, const uint32_t* mc, const uint64_t* mc_off,
                   const uint32_t* flakes, size_t nflakes, uint8_t* is_new, uint32_t* out_mc,
                   uint64_t* out_mc_off, size_t out_cap) {
  /* per-group maxCover tables as growable arrays */
  uint32_t** tab = (uint32_t**)calloc(ngroups ? ngroups : 1, sizeof(uint32_t*));
  size_t* tlen = (size_t*)calloc(ngroups ? ngroups : 1, sizeof(size_t));
  int rc = 0;
  for (uint32_t g = 0; g < ngroups; g++) {
    tlen[g] = (size_t)(mc_off[g + 1] - mc_off[g]);
    tab[g] = (uint32_t*)malloc((tlen[g] ? tlen[g] : 1) * sizeof(uint32_t));
    memcpy(tab[g], mc + mc_off[g], tlen[g] * sizeof(uint32_t));
  }
  for (size_t k = 0; k < n && !rc; k++) {
    uint32_t g = group[k];
    if (g >= ngroups) {
      rc = 1;
      break;
    }
    const uint32_t* cov = pcs + off[k];
    size_t L = (size_t)(off[k + 1] - off[k]);
    is_new[k] = 0;
    if (L == 0) continue; /* fuzzer.go:451-453 */
    /* diff := Difference(cov, maxCover[c.CallID]); diff = Difference(diff, flakes) */
    uint32_t* d1 = (uint32_t*)malloc(L * sizeof(uint32_t));
    uint32_t* d2 = (uint32_t*)malloc(L * sizeof(uint32_t));
    size_t n1 = 0, n2 = 0;
    oracle_setop(0, cov, L, tab[g], tlen[g], d1, L, &n1);
    oracle_setop(0, d1, n1, flakes, nflakes, d2, L, &n2);
    if (n2 != 0) {
      /* maxCover[c.CallID] = Union(maxCover[c.CallID], diff) */
      uint32_t* u = (uint32_t*)malloc((tlen[g] + n2) * sizeof(uint32_t));
      size_t nu = 0;
      oracle_setop(2, tab[g], tlen[g], d2, n2, u, tlen[g] + n2, &nu);
      free(tab[g]);
      tab[g] = u;
      tlen[g] = nu;
      is_new[k] = 1;
    }
    free(d1);
    free(d2);
  }
  size_t p = 0;
  out_mc_off[0] = 0;
  for (uint32_t g = 0; g < ngroups; g++) {
    if (!rc) {
      if (p + tlen[g] > out_cap) {
        rc = 6;
      } else {
        memcpy(out_mc + p, tab[g], tlen[g] * sizeof(uint32_t));
        p += tlen[g];
      }
    }
    out_mc_off[g + 1] = p;
    free(tab[g]);
  }
  free(tab);
  free(tlen);
  return rc;
}

/* The same batch as oracle_novelty, as a first-occurrence characterisation for canonical inputs
 * (sorted covers, sorted duplicate-free tables, sorted flakes): per call, a cover is new iff one of
 * its PCs other than the sentinel is in neither maxCover[call] nor flakes nor an earlier cover of the
 * batch; a call's table becomes the sorted union of its old table and those PCs, without the
 * sentinel (Union drops it, cover.go:63-70), and stays as it was when no cover of the call is new.
 * A hash set per call instead of Go's per-cover merges makes it O(total PCs), and calls spread over
 * nthreads host threads (largest first), so the full configs[2] batch (1M covers) checks in seconds.
 * tests/test_oracle.py pins it to oracle_novelty on canonical random batches. */
typedef struct {
  const uint32_t *pcs, *mc, *flk;
  const uint64_t *off, *mc_off, *cnt;
  const int64_t* members;
  const uint32_t* order;
  size_t nflakes;
  uint32_t ngroups, next;
  uint8_t* is_new;
  uint32_t** tab; /* per call: the new table (NULL: unchanged) */
  size_t* tlen;
} nov_job;

static int cmp_u32(const void* a, const void* b) {
  const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return (x > y) - (x < y);
}

static int in_sorted(const uint32_t* a, size_t n, uint32_t k) {
  size_t lo = 0, hi = n;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (a[mid] < k)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < n && a[lo] == k;
}

static void* nov_worker(void* arg) {
  nov_job* J = (nov_job*)arg;
  for (;;) {
    const uint32_t t = __atomic_fetch_add(&J->next, 1u, __ATOMIC_RELAXED);
    if (t >= J->ngroups) break;
    const uint32_t g = J->order[t];
    const uint32_t* old = J->mc + J->mc_off[g];
    const size_t nold = (size_t)(J->mc_off[g + 1] - J->mc_off[g]);
    const size_t ng = (size_t)(J->cnt[g + 1] - J->cnt[g]);
    u32set seen;
    u32set_init(&seen, nold + 1024);
    for (size_t i = 0; i < nold; i++) u32set_add(&seen, old[i]);
    size_t nnew = 0, cap = 0;
    uint32_t* fresh = NULL;
    for (size_t i = 0; i < ng; i++) {
      const int64_t e = J->members[J->cnt[g] + i];
      const uint32_t* cov = J->pcs + J->off[e];
      const size_t L = (size_t)(J->off[e + 1] - J->off[e]);
      for (size_t k = 0; k < L; k++) {
        const uint32_t pc = cov[k];
        if (pc == SENT || u32set_has(&seen, pc) || in_sorted(J->flk, J->nflakes, pc)) continue;
        u32set_add(&seen, pc);
        if (nnew == cap) {
          cap = cap ? 2 * cap : 1024;
          fresh = (uint32_t*)realloc(fresh, cap * sizeof(uint32_t));
        }
        fresh[nnew++] = pc;
        J->is_new[e] = 1;
      }
    }
    free(seen.slot);
    if (nnew) {
      qsort(fresh, nnew, sizeof(uint32_t), cmp_u32);
      uint32_t* u = (uint32_t*)malloc((nold + nnew) * sizeof(uint32_t));
      size_t nu = 0;
      oracle_setop(2, old, nold, fresh, nnew, u, nold + nnew, &nu); /* drops the sentinel */
      J->tab[g] = u;
      J->tlen[g] = nu;
    }
    free(fresh);
  }
  return NULL;
}

int oracle_novelty_mt(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                      uint32_t ngroups, const uint32_t* mc, const uint64_t* mc_off, const uint32_t* flakes,
                      size_t nflakes, int nthreads, uint8_t* is_new, uint32_t* out_mc, uint64_t* out_mc_off,
                      size_t out_cap) {
  uint64_t* cnt = (uint64_t*)calloc((size_t)ngroups + 1, sizeof(uint64_t));
  for (size_t i = 0; i < n; i++) {
    if (group[i] >= ngroups) {
      free(cnt);
      return 1;
    }
    cnt[group[i] + 1]++;
  }
  for (uint32_t g = 0; g < ngroups; g++) cnt[g + 1] += cnt[g];
  uint64_t* fill = (uint64_t*)malloc(((size_t)ngroups + 1) * sizeof(uint64_t));
  memcpy(fill, cnt, ((size_t)ngroups + 1) * sizeof(uint64_t));
  int64_t* members = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
  for (size_t i = 0; i < n; i++) members[fill[group[i]]++] = (int64_t)i;
  memset(is_new, 0, n);
  nov_job J = {pcs, mc, flakes, off, mc_off, cnt, members, groups_by_size(cnt, ngroups), nflakes, ngroups, 0,
               is_new, (uint32_t**)calloc((size_t)ngroups + 1, sizeof(uint32_t*)),
               (size_t*)calloc((size_t)ngroups + 1, sizeof(size_t))};
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc((size_t)nthreads * sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, nov_worker, &J);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  int rc = 0;
  size_t p = 0;
  out_mc_off[0] = 0;
  for (uint32_t g = 0; g < ngroups; g++) {
    const uint32_t* src = J.tab[g] ? J.tab[g] : mc + mc_off[g];
    const size_t len = J.tab[g] ? J.tlen[g] : (size_t)(mc_off[g + 1] - mc_off[g]);
    if (!rc && p + len > out_cap) rc = 6;
    if (!rc) {
      memcpy(out_mc + p, src, len * sizeof(uint32_t));
      p += len;
    }
    out_mc_off[g + 1] = p;
    free(J.tab[g]);
  }
  free(th);
  free(J.tab);
  free(J.tlen);
  free((void*)J.order);
  free(cnt);
  free(fill);
  free(members);
  return rc;
}

/* ---- prog/encoding.go: Deserialize's call count and CallSet's checks ------------------------- */

/* bufio.ScanLines (Go stdlib bufio/scan.go): a token is the bytes up to '\n' with one trailing '\r'
 * dropped; a final unterminated line is returned at EOF; a token that needs 64 KiB or more of buffer
 * stops the scanner with ErrTooLong (MaxScanTokenSize = 64*1024). Third-party dependency: Go stdlib
 * bufio, version not pinned (README.md:67 requires Go >= 1.7); restated from its published source. */
#define SCAN_MAX_TOKEN (64 * 1024)

void oracle_prog_scan(const uint8_t* data, size_t len, uint32_t* ncalls, uint8_t* status) {
  uint32_t calls = 0;
  uint8_t st = 0;
  size_t i = 0;
  while (i < len) { /* for s.Scan() */
    size_t e = i;
    while (e < len && data[e] != '\n') e++;
    size_t line_len = e - i;
    if (line_len >= SCAN_MAX_TOKEN) {
      st |= 4; /* Scan() returns false: both Deserialize and CallSet stop here */
      break;
    }
    size_t tok = line_len;
    if (tok > 0 && data[i + tok - 1] == '\r') tok--; /* dropCR */
    const uint8_t* ln = data + i;
    /* encoding.go:124 `if p.EOF() || p.Char() == '#' { continue }`;
     * encoding.go:527 `if len(ln) == 0 || ln[0] == '#' { continue }` */
    if (tok > 0 && ln[0] != '#') {
      calls++;
      size_t bracket = 0;
      while (bracket < tok && ln[bracket] != '(') bracket++; /* bytes.IndexByte(ln, '(') */
      if (bracket == tok) {
        st |= 1; /* "line does not contain opening bracket" */
      } else {
        size_t b = 0; /* call := ln[:bracket] */
        size_t eq = 0;
        while (eq < bracket && ln[eq] != '=') eq++;
        if (eq < bracket) { /* if eq := bytes.IndexByte(call, '='); eq != -1 */
          eq++;
          while (eq < bracket && ln[eq] == ' ') eq++;
          b = eq;
        }
        if (bracket - b == 0) st |= 2; /* "call name is empty" */
      }
    }
    i = e + 1; /* past '\n' (or past the end for the final unterminated line) */
  }
  if (calls == 0) st |= 8; /* "program does not contain any calls" */
  *ncalls = calls;
  *status = st;
}

/* ---- hash/hash.go: sha1.Sum ------------------------------------------------------------------ */

static uint32_t rol32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

static void sha1_compress(uint32_t h[5], const uint8_t blk[64]) {
  uint32_t w[80];
  for (int t = 0; t < 16; t++)
    w[t] = (uint32_t)blk[4 * t] << 24 | (uint32_t)blk[4 * t + 1] << 16 | (uint32_t)blk[4 * t + 2] << 8 |
           (uint32_t)blk[4 * t + 3];
  for (int t = 16; t < 80; t++) w[t] = rol32(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
  for (int t = 0; t < 80; t++) {
    uint32_t f, k;
    if (t < 20) {
      f = (b & c) | (~b & d);
      k = 0x5A827999u;
    } else if (t < 40) {
      f = b ^ c ^ d;
      k = 0x6ED9EBA1u;
    } else if (t < 60) {
      f = (b & c) | (b & d) | (c & d);
      k = 0x8F1BBCDCu;
    } else {
      f = b ^ c ^ d;
      k = 0xCA62C1D6u;
    }
    uint32_t tmp = rol32(a, 5) + f + e + k + w[t];
    e = d;
    d = c;
    c = rol32(b, 30);
    b = a;
    a = tmp;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
}

void oracle_sha1(const uint8_t* data, size_t len, uint8_t* sig) {
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  size_t i = 0;
  for (; i + 64 <= len; i += 64) sha1_compress(h, data + i);
  uint8_t tail[128];
  memset(tail, 0, sizeof(tail));
  size_t r = len - i;
  memcpy(tail, data + i, r);
  tail[r] = 0x80;
  size_t tl = r + 1 + 8 <= 64 ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int k = 0; k < 8; k++) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
  sha1_compress(h, tail);
  if (tl == 128) sha1_compress(h, tail + 64);
  for (int k = 0; k < 5; k++) {
    sig[4 * k] = (uint8_t)(h[k] >> 24);
    sig[4 * k + 1] = (uint8_t)(h[k] >> 16);
    sig[4 * k + 2] = (uint8_t)(h[k] >> 8);
    sig[4 * k + 3] = (uint8_t)h[k];
  }
}

/* ---- syz-manager/html.go: cover analytics over mgr.corpus ----------------------------------- */

/* Open-addressing uint32 -> count map standing in for Go's map[uint32]int (html.go:214). */
typedef struct {
  uint64_t* slot; /* key + 1, 0 = free */
  int64_t* cnt;
  size_t mask, count;
} u32map;

static void u32map_init(u32map* m, size_t hint) {
  size_t cap = 64;
  while (cap < hint * 2) cap <<= 1;
  m->slot = (uint64_t*)calloc(cap, sizeof(uint64_t));
  m->cnt = (int64_t*)calloc(cap, sizeof(int64_t));
  m->mask = cap - 1;
  m->count = 0;
}
static void u32map_free(u32map* m) {
  free(m->slot);
  free(m->cnt);
}
static void u32map_inc(u32map* m, uint32_t k);
static void u32map_grow(u32map* m) {
  u32map n;
  u32map_init(&n, m->mask + 1);
  for (size_t i = 0; i <= m->mask; i++)
    if (m->slot[i]) {
      size_t j = u32hash((uint32_t)(m->slot[i] - 1)) & n.mask;
      while (n.slot[j]) j = (j + 1) & n.mask;
      n.slot[j] = m->slot[i];
      n.cnt[j] = m->cnt[i];
      n.count++;
    }
  u32map_free(m);
  *m = n;
}
static void u32map_inc(u32map* m, uint32_t k) {
  if ((m->count + 1) * 2 > m->mask + 1) u32map_grow(m);
  for (size_t i = u32hash(k) & m->mask;; i = (i + 1) & m->mask) {
    if (m->slot[i] == 0) {
      m->slot[i] = (uint64_t)k + 1;
      m->cnt[i] = 1;
      m->count++;
      return;
    }
    if (m->slot[i] == (uint64_t)k + 1) {
      m->cnt[i]++;
      return;
    }
  }
}

/* html.go:213-237 uniqueCover(perCall). Returns a malloc'ed, Canonicalized list in *out. */
static size_t unique_cover(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                           uint32_t ngroups, int per_call, uint32_t** out) {
  u32map total;
  u32map_init(&total, 1024);
  u32set* call_cover = NULL;
  if (per_call) {
    call_cover = (u32set*)calloc(ngroups ? ngroups : 1, sizeof(u32set));
    for (uint32_t g = 0; g < ngroups; g++) u32set_init(&call_cover[g], 16);
  }
  for (size_t e = 0; e < n; e++) {
    for (uint64_t j = off[e]; j < off[e + 1]; j++) {
      const uint32_t pc = pcs[j];
      if (per_call) {
        if (u32set_has(&call_cover[group[e]], pc)) continue;
        u32set_add(&call_cover[group[e]], pc);
      }
      u32map_inc(&total, pc);
    }
  }
  size_t k = 0;
  uint32_t* cov = (uint32_t*)malloc((total.count ? total.count : 1) * sizeof(uint32_t));
  for (size_t i = 0; i <= total.mask; i++) /* map order: arbitrary, as in Go */
    if (total.slot[i] && total.cnt[i] == 1) cov[k++] = (uint32_t)(total.slot[i] - 1);
  size_t nk = 0;
  oracle_canonicalize(cov, k, &nk);
  u32map_free(&total);
  if (per_call) {
    for (uint32_t g = 0; g < ngroups; g++) free(call_cover[g].slot);
    free(call_cover);
  }
  *out = cov;
  return nk;
}

/* cc.cov = cover.Union(cc.cov, inp.Cover) for the inputs of group g (all inputs when g < 0). */
static size_t union_of(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n, int64_t g,
                       uint32_t** out) {
  uint32_t* acc = (uint32_t*)malloc(sizeof(uint32_t));
  size_t na = 0;
  for (size_t e = 0; e < n; e++) {
    if (g >= 0 && group[e] != (uint32_t)g) continue;
    const size_t L = (size_t)(off[e + 1] - off[e]);
    uint32_t* u = (uint32_t*)malloc((na + L + 1) * sizeof(uint32_t));
    size_t nu = 0;
    oracle_setop(2, acc, na, pcs + off[e], L, u, na + L + 1, &nu);
    free(acc);
    acc = u;
    na = nu;
  }
  *out = acc;
  return na;
}

static size_t intersection_len(const uint32_t* a, size_t na, const uint32_t* b, size_t nb) {
  uint32_t* tmp = (uint32_t*)malloc((na < nb ? na : nb) * sizeof(uint32_t) + 4);
  size_t k = 0;
  oracle_setop(3, a, na, b, nb, tmp, (na < nb ? na : nb) + 1, &k);
  free(tmp);
  return k;
}

int oracle_cover_stats(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                       uint32_t ngroups, uint64_t* call_inputs, uint64_t* call_cover, uint64_t* call_unique,
                       uint64_t* totals, uint32_t* input_unique) {
  for (size_t e = 0; e < n; e++)
    if (group[e] >= ngroups) return 1;
  uint32_t *uc_call = NULL, *uc_input = NULL;
  const size_t nuc_call = unique_cover(pcs, off, group, n, ngroups, 1, &uc_call);
  const size_t nuc_input = unique_cover(pcs, off, group, n, ngroups, 0, &uc_input);
  /* html.go:67-97: calls[inp.Call].count / .cov, cov = Union over calls (map order; Union commutes) */
  uint32_t* cov = (uint32_t*)malloc(sizeof(uint32_t));
  size_t ncov = 0;
  for (uint32_t g = 0; g < ngroups; g++) {
    uint64_t cnt = 0;
    for (size_t e = 0; e < n; e++) cnt += group[e] == g;
    uint32_t* cc = NULL;
    const size_t ncc = union_of(pcs, off, group, n, g, &cc);
    call_inputs[g] = cnt;
    call_cover[g] = ncc;
    call_unique[g] = intersection_len(cc, ncc, uc_call, nuc_call);
    uint32_t* u = (uint32_t*)malloc((ncov + ncc + 1) * sizeof(uint32_t));
    size_t nu = 0;
    oracle_setop(2, cov, ncov, cc, ncc, u, ncov + ncc + 1, &nu);
    free(cov);
    cov = u;
    ncov = nu;
    free(cc);
  }
  totals[0] = ncov;
  totals[1] = nuc_call;
  totals[2] = nuc_input;
  /* html.go:158-170 httpCorpus: len(cover.Intersection(inp.Cover, totalUnique)) */
  for (size_t e = 0; e < n; e++)
    input_unique[e] = (uint32_t)intersection_len(pcs + off[e], (size_t)(off[e + 1] - off[e]), uc_input, nuc_input);
  free(cov);
  free(uc_call);
  free(uc_input);
  return 0;
}

int oracle_corpus_cover(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                        uint32_t ngroups, int64_t call, int unique, uint32_t* out, size_t cap, size_t* out_n) {
  if (call >= (int64_t)ngroups || unique < 0 || unique > 2) return 1;
  uint32_t* res = NULL;
  size_t nres = 0;
  if (call < 0 && unique) {
    nres = unique_cover(pcs, off, group, n, ngroups, unique == 1, &res);
  } else {
    nres = union_of(pcs, off, group, n, call, &res);
    if (unique) {
      uint32_t* uc = NULL;
      const size_t nuc = unique_cover(pcs, off, group, n, ngroups, unique == 1, &uc);
      uint32_t* x = (uint32_t*)malloc((nres + 1) * sizeof(uint32_t));
      size_t nx = 0;
      oracle_setop(3, res, nres, uc, nuc, x, nres + 1, &nx);
      free(res);
      free(uc);
      res = x;
      nres = nx;
    }
  }
  *out_n = nres;
  int rc = 0;
  if (nres > cap)
    rc = 6;
  else
    memcpy(out, res, nres * sizeof(uint32_t));
  free(res);
  return rc;
}

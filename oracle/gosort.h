/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, called by, or shipped with the product
 * (libsyzgpu.so). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * Restatement of the Go standard library's sort.Sort (Go 1.6 .. 1.18 algorithm) as a C macro
 * template. The reference (no go.mod; README.md:67 asks for Go >= 1.7) sorts with this algorithm in
 *   cover/cover.go:29   Canonicalize  -> sort.Sort(Cover(cov))
 *   cover/cover.go:113  Minimize      -> sort.Sort(minInputArray(inputs))   (unstable! tie order
 *                                        decides which inputs Minimize keeps)
 * Third-party dependency: Go stdlib "sort" (version not pinned by the reference; Go 1.7 era).
 * Algorithm restated from the published Go sources of that era (sort/sort.go):
 *   quickSort(data, a, b, maxDepth):   while b-a > 12 { heapSort at depth 0; doPivot; recurse on the
 *                                      smaller side }  then a gap-6 shell pass + insertionSort.
 *   Leaf form (gosort_leaf, oracle_set_go_sort_leaf): 12 as above (the default), or 7: `while b-a > 7`
 *   and insertionSort alone. The reference pins neither (it asks for Go >= 1.7; its tests hold no tie of
 *   more than three equal keys), so both are restated, as in the GPU sort (syzgpu_set_go_sort_leaf).
 *   doPivot: Tukey ninther for hi-lo > 40, medianOfThree(lo, m, hi-1), Hoare-style partition with
 *            the "protect" duplicate pass, pivot swapped into the middle.
 *   maxDepth(n) = 2 * ceil(lg(n+1)).
 * Go >= 1.19 switched to pdqsort (different tie order); not restated here.
 *
 * PARITY STATUS: the tie order for n > 12 equal keys is "parity unpinned" — no Go toolchain exists
 * in this environment and the reference tests (cover/cover_test.go:104-168) only contain ties at
 * n = 3. Everything else in the oracle is pinned by cover_test.go's tables.
 *
 * GOSORT_DEFINE(name, T, LESS) defines  void name(T* data, long n);
 * LESS(x, y) must be an expression on two element *values* equal to Go's data.Less(i, j).
 */
#ifndef SYZ_ORACLE_GOSORT_H
#define SYZ_ORACLE_GOSORT_H

static int gosort_leaf = 12; /* 12 or 7, see above */

#define GOSORT_DEFINE(name, T, LESS)                                                             \
  static inline int name##_less(T* d, long i, long j) { return (LESS(d[i], d[j])); }            \
  static inline void name##_swap(T* d, long i, long j) {                                        \
    T t = d[i];                                                                                 \
    d[i] = d[j];                                                                                \
    d[j] = t;                                                                                   \
  }                                                                                             \
  static void name##_insertion(T* d, long a, long b) {                                          \
    for (long i = a + 1; i < b; i++)                                                            \
      for (long j = i; j > a && name##_less(d, j, j - 1); j--) name##_swap(d, j, j - 1);       \
  }                                                                                             \
  static void name##_siftdown(T* d, long lo, long hi, long first) {                             \
    long root = lo;                                                                             \
    for (;;) {                                                                                  \
      long child = 2 * root + 1;                                                                \
      if (child >= hi) break;                                                                   \
      if (child + 1 < hi && name##_less(d, first + child, first + child + 1)) child++;         \
      if (!name##_less(d, first + root, first + child)) return;                                 \
      name##_swap(d, first + root, first + child);                                              \
      root = child;                                                                             \
    }                                                                                           \
  }                                                                                             \
  static void name##_heapsort(T* d, long a, long b) {                                           \
    long first = a, lo = 0, hi = b - a;                                                         \
    for (long i = (hi - 1) / 2; i >= 0; i--) name##_siftdown(d, i, hi, first);                \
    for (long i = hi - 1; i >= 0; i--) {                                                        \
      name##_swap(d, first, first + i);                                                         \
      name##_siftdown(d, lo, i, first);                                                         \
    }                                                                                           \
  }                                                                                             \
  /* medianOfThree moves the median of data[m0], data[m1], data[m2] into data[m1]. */           \
  static void name##_mo3(T* d, long m1, long m0, long m2) {                                     \
    if (name##_less(d, m1, m0)) name##_swap(d, m1, m0);                                         \
    if (name##_less(d, m2, m1)) {                                                               \
      name##_swap(d, m2, m1);                                                                   \
      if (name##_less(d, m1, m0)) name##_swap(d, m1, m0);                                       \
    }                                                                                           \
  }                                                                                             \
  static void name##_dopivot(T* d, long lo, long hi, long* midlo, long* midhi) {                \
    long m = (long)(((unsigned long)(lo + hi)) >> 1);                                           \
    if (hi - lo > 40) {                                                                         \
      long s = (hi - lo) / 8;                                                                   \
      name##_mo3(d, lo, lo + s, lo + 2 * s);                                                    \
      name##_mo3(d, m, m - s, m + s);                                                           \
      name##_mo3(d, hi - 1, hi - 1 - s, hi - 1 - 2 * s);                                        \
    }                                                                                           \
    name##_mo3(d, lo, m, hi - 1);                                                               \
    long pivot = lo, a = lo + 1, c = hi - 1;                                                    \
    for (; a < c && name##_less(d, a, pivot); a++) {                                            \
    }                                                                                           \
    long b = a;                                                                                 \
    for (;;) {                                                                                  \
      for (; b < c && !name##_less(d, pivot, b); b++) {                                         \
      }                                                                                         \
      for (; b < c && name##_less(d, pivot, c - 1); c--) {                                      \
      }                                                                                         \
      if (b >= c) break;                                                                        \
      name##_swap(d, b, c - 1);                                                                 \
      b++;                                                                                      \
      c--;                                                                                      \
    }                                                                                           \
    int protect = hi - c < 5;                                                                   \
    if (!protect && hi - c < (hi - lo) / 4) {                                                   \
      int dups = 0;                                                                             \
      if (!name##_less(d, pivot, hi - 1)) {                                                     \
        name##_swap(d, c, hi - 1);                                                              \
        c++;                                                                                    \
        dups++;                                                                                 \
      }                                                                                         \
      if (!name##_less(d, b - 1, pivot)) {                                                      \
        b--;                                                                                    \
        dups++;                                                                                 \
      }                                                                                         \
      if (!name##_less(d, m, pivot)) {                                                          \
        name##_swap(d, m, b - 1);                                                               \
        b--;                                                                                    \
        dups++;                                                                                 \
      }                                                                                         \
      protect = dups > 1;                                                                       \
    }                                                                                           \
    if (protect) {                                                                              \
      for (;;) {                                                                                \
        for (; a < b && !name##_less(d, b - 1, pivot); b--) {                                   \
        }                                                                                       \
        for (; a < b && name##_less(d, a, pivot); a++) {                                        \
        }                                                                                       \
        if (a >= b) break;                                                                      \
        name##_swap(d, a, b - 1);                                                               \
        a++;                                                                                    \
        b--;                                                                                    \
      }                                                                                         \
    }                                                                                           \
    name##_swap(d, pivot, b - 1);                                                               \
    *midlo = b - 1;                                                                             \
    *midhi = c;                                                                                 \
  }                                                                                             \
  static void name##_quick(T* d, long a, long b, int maxDepth) {                                \
    while (b - a > gosort_leaf) {                                                               \
      if (maxDepth == 0) {                                                                      \
        name##_heapsort(d, a, b);                                                               \
        return;                                                                                 \
      }                                                                                         \
      maxDepth--;                                                                               \
      long mlo, mhi;                                                                            \
      name##_dopivot(d, a, b, &mlo, &mhi);                                                      \
      if (mlo - a < b - mhi) {                                                                  \
        name##_quick(d, a, mlo, maxDepth);                                                      \
        a = mhi;                                                                                \
      } else {                                                                                  \
        name##_quick(d, mhi, b, maxDepth);                                                      \
        b = mlo;                                                                                \
      }                                                                                         \
    }                                                                                           \
    if (b - a > 1) {                                                                            \
      if (gosort_leaf == 12)                                                                    \
        for (long i = a + 6; i < b; i++)                                                        \
          if (name##_less(d, i, i - 6)) name##_swap(d, i, i - 6);                               \
      name##_insertion(d, a, b);                                                                \
    }                                                                                           \
  }                                                                                             \
  static inline int name##_maxdepth(long n) {                                                   \
    int depth = 0;                                                                              \
    for (long i = n; i > 0; i >>= 1) depth++;                                                   \
    return depth * 2;                                                                           \
  }                                                                                             \
  static void name(T* d, long n) { name##_quick(d, 0, n, name##_maxdepth(n)); }

#endif

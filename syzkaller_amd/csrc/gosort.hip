// The permutation Go's sort.Sort (Go 1.7 quickSort) produces for cover.Minimize's input array
// (cover/cover.go:106-113, minInputArray.Less = len(a[i].cov) > len(a[j].cov), :140-143),
// computed on the GPU for every call group at once, in ONE persistent launch.
//
// sort.Sort is unstable: among equal lengths the order depends on the exact sequence of swaps, and
// that order decides which inputs Minimize keeps. The simulation performs exactly the
// swaps of the sequential algorithm, with each doPivot's O(n) loops run in parallel:
//   * the Hoare loop pairs the k-th element > pivot from the left with the k-th element <= pivot
//     from the right for every k below the number of misplaced elements: both lists are built by
//     ordered compaction (prefix scans / ballots) and swapped pairwise;
//   * the "protect" duplicate pass is the same pairing with (== pivot) vs (< pivot);
//   * the O(1) parts (Tukey ninther + medianOfThree, the dups probe) gather their <= 9 elements in
//     parallel and evaluate the sequential decision logic on registers in every lane;
//   * leaves (<= 12 elements: gap-6 shell pass + insertionSort) are six disjoint compare-swaps plus
//     a STABLE sort — insertionSort only moves an element past strictly greater ones — done as a
//     lane-parallel rank computation.
// Disjoint subranges are independent, so nodes are scheduled through a global work queue:
//   segment > T_LDS   one 1024-thread workgroup partitions it in place in HBM, pushes the children;
//   segment <= T_LDS  one workgroup sorts it to completion in LDS (1024-thread cooperative
//                     partitions above WAVE_MAX, then one wave per sub-segment) and writes the
//                     local permutation to perm[].
// Elements are (len << 32) | member index in HBM and (len << 14) | local index in LDS; Less only
// compares the length field.
#include <type_traits>

#include "pipeline.hpp"

namespace syz {

#ifdef SYZ_GS_DEBUG
#define GSD(...) printf(__VA_ARGS__)
#else
#define GSD(...)
#endif

constexpr int GS_BLOCK = 1024;
constexpr int GS_WAVES = GS_BLOCK / 64;
constexpr uint32_t T_LDS = 16384;     // segment sorted entirely in LDS (u32 packed elements)
constexpr uint32_t WAVE_MAX = 1024;   // sub-segments handled by a single wave
constexpr uint32_t LDS_SHIFT = 14;    // local index bits
constexpr uint32_t LEN_LIMIT = 1u << 18;
constexpr uint32_t STACK_A = 64;
constexpr uint32_t LIST_B = 128;   // phase-A leaves: <= 2 per cooperative partition
constexpr uint32_t STACK_W = 64;   // >= sort.Sort maxDepth budget + 1

template <int SH, class T>
__device__ __forceinline__ bool LT(T x, T y) {  // Go's Less: longer cover first
  return (x >> SH) > (y >> SH);
}
template <int SH, class T>
__device__ __forceinline__ uint32_t KEY(T x) {
  return (uint32_t)(x >> SH);
}

template <class P>
__device__ __forceinline__ void swp(P d, uint32_t i, uint32_t j) {
  auto t = d[i];
  d[i] = d[j];
  d[j] = t;
}

// medianOfThree(data, m1, m0, m2) on values: moves the median into a1 (= data[m1]).
template <int SH, class T>
__device__ __forceinline__ void mo3v(T& a1, T& a0, T& a2) {
  if (LT<SH>(a1, a0)) {
    T t = a1;
    a1 = a0;
    a0 = t;
  }
  if (LT<SH>(a2, a1)) {
    T t = a2;
    a2 = a1;
    a1 = t;
    if (LT<SH>(a1, a0)) {
      t = a1;
      a1 = a0;
      a0 = t;
    }
  }
}

// doPivot's pivot selection, executed by a full wave (all lanes compute redundantly on registers).
// Leaves the pivot at d[lo]; returns m.
template <int SH, class P>
__device__ uint32_t wave_pivot(P d, uint32_t lo, uint32_t hi) {
  using T = typename std::remove_reference<decltype(d[0])>::type;
  const unsigned lane = __lane_id();
  const uint32_t m = (uint32_t)(((uint64_t)lo + hi) >> 1);
  if (hi - lo > 40) {
    const uint32_t s = (hi - lo) / 8;
    uint32_t pos = lo;
    switch (lane) {
      case 1: pos = lo + s; break;
      case 2: pos = lo + 2 * s; break;
      case 3: pos = m - s; break;
      case 4: pos = m; break;
      case 5: pos = m + s; break;
      case 6: pos = hi - 1 - 2 * s; break;
      case 7: pos = hi - 1 - s; break;
      case 8: pos = hi - 1; break;
      default: break;
    }
    T mine = lane < 9 ? d[pos] : T(0);
    T v0 = __shfl(mine, 0), v1 = __shfl(mine, 1), v2 = __shfl(mine, 2), v3 = __shfl(mine, 3),
      v4 = __shfl(mine, 4), v5 = __shfl(mine, 5), v6 = __shfl(mine, 6), v7 = __shfl(mine, 7),
      v8 = __shfl(mine, 8);
    mo3v<SH>(v0, v1, v2);  // medianOfThree(lo, lo+s, lo+2s)
    mo3v<SH>(v4, v3, v5);  // medianOfThree(m, m-s, m+s)
    mo3v<SH>(v8, v7, v6);  // medianOfThree(hi-1, hi-1-s, hi-1-2s)
    mo3v<SH>(v0, v4, v8);  // medianOfThree(lo, m, hi-1)
    T out = v0;
    switch (lane) {
      case 1: out = v1; break;
      case 2: out = v2; break;
      case 3: out = v3; break;
      case 4: out = v4; break;
      case 5: out = v5; break;
      case 6: out = v6; break;
      case 7: out = v7; break;
      case 8: out = v8; break;
      default: break;
    }
    if (lane < 9 && out != mine) d[pos] = out;
  } else {
    const uint32_t pos = lane == 0 ? lo : (lane == 1 ? m : hi - 1);
    T mine = lane < 3 ? d[pos] : T(0);
    T v0 = __shfl(mine, 0), v1 = __shfl(mine, 1), v2 = __shfl(mine, 2);
    mo3v<SH>(v0, v1, v2);  // medianOfThree(lo, m, hi-1)
    T out = lane == 0 ? v0 : (lane == 1 ? v1 : v2);
    if (lane < 3 && out != mine) d[pos] = out;
  }
  return m;
}

// doPivot's dups probe after the main partition (b == c == bnd on entry), one full wave.
// The five positions it may touch are cached by position, so aliasing (m == b-1) is exact.
template <int SH, class P>
__device__ bool wave_probe(P d, uint32_t lo, uint32_t hi, uint32_t m, uint32_t bnd, uint32_t* bout,
                           uint32_t* cout) {
  using T = typename std::remove_reference<decltype(d[0])>::type;
  uint32_t b = bnd, c = bnd;
  bool protect = hi - c < 5;
  if (!protect && hi - c < (hi - lo) / 4) {
    const unsigned lane = __lane_id();
    const uint32_t p0 = hi - 1, p1 = bnd, p2 = bnd - 1, p3 = bnd - 2, p4 = m;
    const uint32_t pos = lane == 0 ? p0 : lane == 1 ? p1 : lane == 2 ? p2 : lane == 3 ? p3 : lane == 4 ? p4 : lo;
    T mine = lane < 6 ? d[pos] : T(0);
    T v0 = __shfl(mine, 0), v1 = __shfl(mine, 1), v2 = __shfl(mine, 2), v3 = __shfl(mine, 3),
      v4 = __shfl(mine, 4), pv = __shfl(mine, 5);
    auto get = [&](uint32_t p) -> T {
      return p == p0 ? v0 : p == p1 ? v1 : p == p2 ? v2 : p == p3 ? v3 : v4;
    };
    auto set = [&](uint32_t p, T x) {
      if (p == p0) v0 = x;
      if (p == p1) v1 = x;
      if (p == p2) v2 = x;
      if (p == p3) v3 = x;
      if (p == p4) v4 = x;
    };
    int dups = 0;
    if (!LT<SH>(pv, get(hi - 1))) {  // data[hi-1] = pivot: swap(c, hi-1); c++
      T t = get(c);
      set(c, get(hi - 1));
      set(hi - 1, t);
      c++;
      dups++;
    }
    if (!LT<SH>(get(b - 1), pv)) {  // data[b-1] = pivot
      b--;
      dups++;
    }
    if (!LT<SH>(get(m), pv)) {  // data[m] = pivot: swap(m, b-1); b--
      T t = get(m);
      set(m, get(b - 1));
      set(b - 1, t);
      b--;
      dups++;
    }
    protect = dups > 1;
    T out = lane == 0 ? v0 : lane == 1 ? v1 : lane == 2 ? v2 : lane == 3 ? v3 : v4;
    if (lane < 5 && out != mine) d[pos] = out;
  }
  *bout = b;
  *cout = c;
  return protect;
}

// quickSort's tail for 2..12 elements: gap-6 shell pass (six disjoint compare-swaps) then
// insertionSort (= a stable sort under Less), one full wave.
template <int SH, class P>
__device__ void wave_leaf(P d, uint32_t lo, uint32_t hi) {
  using T = typename std::remove_reference<decltype(d[0])>::type;
  const uint32_t n = hi - lo;
  const unsigned lane = __lane_id();
  T x = lane < n ? d[lo + lane] : T(0);
  const unsigned partner = lane < 6 ? lane + 6 : lane - 6;
  T y = __shfl(x, partner < 64 ? partner : 0);
  if (lane < n && partner < n && lane < 12) {
    if (lane >= 6) {
      if (LT<SH>(x, y)) x = y;  // Less(i, i-6): lane i takes data[i-6]
    } else {
      if (LT<SH>(y, x)) x = y;  // Less(j+6, j): lane j takes data[j+6]
    }
  }
  uint32_t rank = 0;
  for (uint32_t j = 0; j < n; j++) {
    const T xj = __shfl(x, j);
    if (LT<SH>(xj, x) || (j < lane && KEY<SH>(xj) == KEY<SH>(x))) rank++;
  }
  wave_sync();
  if (lane < n) d[lo + rank] = x;
  wave_sync();
}

template <int SH, class P>
__device__ void sift_down(P d, uint32_t lo, uint32_t hi, uint32_t first) {
  uint32_t root = lo;
  for (;;) {
    uint32_t child = 2 * root + 1;
    if (child >= hi) break;
    if (child + 1 < hi && LT<SH>(d[first + child], d[first + child + 1])) child++;
    if (!LT<SH>(d[first + root], d[first + child])) return;
    swp(d, first + root, first + child);
    root = child;
  }
}

template <int SH, class P>
__device__ void heap_sort(P d, uint32_t a, uint32_t b) {  // one thread
  const uint32_t first = a, hi = b - a;
  for (int64_t i = ((int64_t)hi - 1) / 2; i >= 0; i--) sift_down<SH>(d, (uint32_t)i, hi, first);
  for (int64_t i = (int64_t)hi - 1; i >= 0; i--) {
    swp(d, first, first + (uint32_t)i);
    sift_down<SH>(d, 0, (uint32_t)i, first);
  }
}

// ---- ordered compaction helpers ----------------------------------------------------------------
template <class Pred, class Q>
__device__ uint32_t wave_collect(uint32_t beg, uint32_t end, Pred pred, Q out) {
  uint32_t k = 0;
  for (uint32_t base = beg; base < end; base += 64) {
    const uint32_t p = base + __lane_id();
    const bool f = p < end && pred(p);
    const uint64_t mask = __ballot(f);
    if (f) out[k + __popcll(mask & lanemask_lt())] = p;
    k += __popcll(mask);
  }
  return k;
}

// Block-wide: every thread takes a contiguous run of the range; counts, scans, then writes in order.
template <class Pred, class Q>
__device__ uint32_t block_collect(uint32_t beg, uint32_t end, Pred pred, Q out, uint32_t* red) {
  const uint32_t n = end > beg ? end - beg : 0;
  const uint32_t per = (n + GS_BLOCK - 1) / GS_BLOCK;
  const uint32_t s = beg + threadIdx.x * per;
  const uint32_t e = min(end, s + per);
  uint32_t cnt = 0;
  for (uint32_t p = s; p < e; p++) cnt += pred(p) ? 1u : 0u;
  uint32_t tot;
  uint32_t k = block_excl_scan<GS_BLOCK>(cnt, red, &tot);
  for (uint32_t p = s; p < e; p++)
    if (pred(p)) out[k++] = p;
  __syncthreads();
  return tot;
}

template <class Pred>
__device__ uint32_t block_count(uint32_t beg, uint32_t end, Pred pred, uint32_t* red) {
  uint32_t c = 0;
  for (uint32_t p = beg + threadIdx.x; p < end; p += GS_BLOCK) c += pred(p) ? 1u : 0u;
  return block_sum<GS_BLOCK>(c, red);
}

// ---- one doPivot by the whole workgroup on an array in LDS (u32) or HBM (u64) ----------------------
// A/B: position scratch (tA/tB + lo indexing). Returns false if depth was exhausted (caller sorts).
template <int SH, class P, class Q>
__device__ void block_dopivot(P d, Q A, Q B, uint32_t lo, uint32_t hi, uint32_t* red, uint32_t* sh,
                              uint32_t* mlo, uint32_t* mhi) {
  if (threadIdx.x < 64) {
    const uint32_t m = wave_pivot<SH>(d, lo, hi);
    if (threadIdx.x == 0) {
      sh[0] = KEY<SH>(d[lo]);
      sh[1] = m;
    }
  }
  __syncthreads();
  const uint32_t plen = sh[0], m = sh[1];
  auto key = [&](uint32_t p) { return KEY<SH>(d[p]); };
  const uint32_t bnd = lo + 1 + block_count(lo + 1, hi - 1, [&](uint32_t p) { return key(p) >= plen; }, red);
  const uint32_t nG = block_collect(lo + 1, bnd, [&](uint32_t p) { return key(p) < plen; }, A + lo, red);
  (void)block_collect(bnd, hi - 1, [&](uint32_t p) { return key(p) >= plen; }, B + lo, red);
  for (uint32_t k = threadIdx.x; k < nG; k += GS_BLOCK) swp(d, A[lo + k], B[lo + nG - 1 - k]);
  __syncthreads();
  if (threadIdx.x < 64) {
    uint32_t b, c;
    const bool protect = wave_probe<SH>(d, lo, hi, m, bnd, &b, &c);
    if (threadIdx.x == 0) {
      sh[2] = b;
      sh[3] = c;
      sh[4] = protect;
    }
  }
  __syncthreads();
  uint32_t b = sh[2];
  const uint32_t c = sh[3];
  if (sh[4]) {
    // protect pass over [lo+1, b): len > plen stays left, len <= plen goes right
    const uint32_t b2 = lo + 1 + block_count(lo + 1, b, [&](uint32_t p) { return key(p) > plen; }, red);
    const uint32_t nE = block_collect(lo + 1, b2, [&](uint32_t p) { return key(p) <= plen; }, A + lo, red);
    (void)block_collect(b2, b, [&](uint32_t p) { return key(p) > plen; }, B + lo, red);
    for (uint32_t k = threadIdx.x; k < nE; k += GS_BLOCK) swp(d, A[lo + k], B[lo + nE - 1 - k]);
    __syncthreads();
    b = b2;
  }
  if (threadIdx.x == 0) swp(d, lo, b - 1);
  __syncthreads();
  *mlo = b - 1;
  *mhi = c;
}

// One doPivot by a single wave on LDS.
template <class P, class Q>
__device__ void wave_dopivot(P d, Q A, Q B, uint32_t lo, uint32_t hi, uint32_t* mlo, uint32_t* mhi) {
  constexpr int SH = LDS_SHIFT;
  const uint32_t m = wave_pivot<SH>(d, lo, hi);
  wave_sync();
  const uint32_t plen = KEY<SH>(d[lo]);
  auto key = [&](uint32_t p) { return KEY<SH>(d[p]); };
  uint32_t lc = 0;
  for (uint32_t p = lo + 1 + __lane_id(); p < hi - 1; p += 64) lc += key(p) >= plen;
  const uint32_t bnd = lo + 1 + wave_sum(lc);
  const uint32_t nG = wave_collect(lo + 1, bnd, [&](uint32_t p) { return key(p) < plen; }, A + lo);
  (void)wave_collect(bnd, hi - 1, [&](uint32_t p) { return key(p) >= plen; }, B + lo);
  wave_sync();
  for (uint32_t k = __lane_id(); k < nG; k += 64) swp(d, A[lo + k], B[lo + nG - 1 - k]);
  wave_sync();
  uint32_t b, c;
  const bool protect = wave_probe<SH>(d, lo, hi, m, bnd, &b, &c);
  wave_sync();
  if (protect) {
    uint32_t xc = 0;
    for (uint32_t p = lo + 1 + __lane_id(); p < b; p += 64) xc += key(p) > plen;
    const uint32_t b2 = lo + 1 + wave_sum(xc);
    const uint32_t nE = wave_collect(lo + 1, b2, [&](uint32_t p) { return key(p) <= plen; }, A + lo);
    (void)wave_collect(b2, b, [&](uint32_t p) { return key(p) > plen; }, B + lo);
    wave_sync();
    for (uint32_t k = __lane_id(); k < nE; k += 64) swp(d, A[lo + k], B[lo + nE - 1 - k]);
    wave_sync();
    b = b2;
  }
  if (__lane_id() == 0) swp(d, lo, b - 1);
  wave_sync();
  *mlo = b - 1;
  *mhi = c;
}

// quickSort(d, lo, hi, depth) entirely by one wave (sub-segment <= WAVE_MAX in LDS).
__device__ void wave_quicksort(uint32_t* d, uint16_t* A, uint16_t* B, uint32_t* stk, uint32_t lo, uint32_t hi,
                               int32_t depth) {
  constexpr int SH = LDS_SHIFT;
  int sp = 0;
  if (__lane_id() == 0) {
    stk[0] = lo;
    stk[1] = hi;
    stk[2] = (uint32_t)depth;
  }
  sp = 1;
  wave_sync();
  while (sp > 0) {
    sp--;
    const uint32_t a = stk[3 * sp], b = stk[3 * sp + 1];
    const int32_t dep = (int32_t)stk[3 * sp + 2];
    wave_sync();
    if (__lane_id() == 0) GSD("wq pop [%u,%u) dep %d sp %d\n", a, b, dep, sp);
    if (b - a <= 12) {
      if (b - a > 1) wave_leaf<SH>(d, a, b);
      if (__lane_id() == 0) GSD("leaf done\n");
      continue;
    }
    if (dep == 0) {
      if (__lane_id() == 0) heap_sort<SH>(d, a, b);
      wave_sync();
      continue;
    }
    uint32_t mlo, mhi;
    wave_dopivot(d, A, B, a, b, &mlo, &mhi);
    if (__lane_id() == 0) {
      stk[3 * sp] = a;
      stk[3 * sp + 1] = mlo;
      stk[3 * sp + 2] = (uint32_t)(dep - 1);
      stk[3 * sp + 3] = mhi;
      stk[3 * sp + 4] = b;
      stk[3 * sp + 5] = (uint32_t)(dep - 1);
    }
    sp += 2;
    wave_sync();
  }
}

struct QCtl {
  uint32_t head, tail, pending, err;
};

struct GsLds {
  uint32_t d[T_LDS];
  uint16_t A[T_LDS];
  uint16_t B[T_LDS];
  uint32_t red[GS_BLOCK / 64 + 1];
  uint32_t sh[8];
  uint32_t stackA[STACK_A * 3];
  uint32_t listB[LIST_B * 3];
  uint32_t stackW[GS_WAVES][STACK_W * 3];
  uint32_t nA, nB, flag;
};

// Sort el[lo, lo+n) (n <= T_LDS) completely in LDS; writes perm[lo + p] = lo + source offset.
// Returns false (nothing written) if a length does not fit the packed LDS format.
__device__ bool lds_sort(const uint64_t* __restrict__ el, uint32_t* __restrict__ perm, uint32_t lo, uint32_t n,
                         int32_t depth, GsLds& L) {
  constexpr int SH = LDS_SHIFT;
  if (threadIdx.x == 0) {
    L.flag = 0;
    L.nA = 0;
    L.nB = 0;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += GS_BLOCK) {
    const uint64_t len = el[lo + i] >> 32;
    if (len >= LEN_LIMIT) L.flag = 1;
    L.d[i] = ((uint32_t)len << SH) | i;
  }
  __syncthreads();
  if (threadIdx.x == 0) GSD("lds loaded n %u flag %u\n", n, L.flag);
  if (L.flag) return false;
  // phase A: cooperative partitions of sub-segments larger than one wave's share
  if (threadIdx.x == 0) {
    if (n > WAVE_MAX && depth > 0) {
      L.stackA[0] = 0;
      L.stackA[1] = n;
      L.stackA[2] = (uint32_t)depth;
      L.nA = 1;
    } else {
      L.listB[0] = 0;
      L.listB[1] = n;
      L.listB[2] = (uint32_t)depth;
      L.nB = 1;
    }
  }
  __syncthreads();
  while (L.nA > 0) {
    const uint32_t top = L.nA - 1;
    const uint32_t a = L.stackA[3 * top], b = L.stackA[3 * top + 1];
    const int32_t dep = (int32_t)L.stackA[3 * top + 2];
    __syncthreads();
    if (threadIdx.x == 0) L.nA = top;
    uint32_t mlo, mhi;
    block_dopivot<SH>(L.d, L.A, L.B, a, b, L.red, L.sh, &mlo, &mhi);
    if (threadIdx.x == 0) {
      const uint32_t ca[2] = {a, mhi}, cb[2] = {mlo, b};
      for (int k = 0; k < 2; k++) {
        const uint32_t s = cb[k] - ca[k];
        if (s <= 1) continue;
        if (s > WAVE_MAX && dep - 1 > 0) {
          L.stackA[3 * L.nA] = ca[k];
          L.stackA[3 * L.nA + 1] = cb[k];
          L.stackA[3 * L.nA + 2] = (uint32_t)(dep - 1);
          L.nA++;
        } else {
          L.listB[3 * L.nB] = ca[k];
          L.listB[3 * L.nB + 1] = cb[k];
          L.listB[3 * L.nB + 2] = (uint32_t)(dep - 1);
          L.nB++;
        }
      }
    }
    __syncthreads();
  }
  // phase B: one wave per remaining sub-segment
  const int w = threadIdx.x >> 6;
  if (threadIdx.x == 0) GSD("phase B nB %u\n", L.nB);
  for (uint32_t i = w; i < L.nB; i += GS_WAVES) {
    const uint32_t a = L.listB[3 * i], b = L.listB[3 * i + 1];
    const int32_t dep = (int32_t)L.listB[3 * i + 2];
    if (b - a > WAVE_MAX && dep == 0) {
      if (__lane_id() == 0) heap_sort<SH>(L.d, a, b);  // depth-exhausted large sub-segment
      wave_sync();
    } else {
      wave_quicksort(L.d, L.A, L.B, L.stackW[w], a, b, dep);
    }
  }
  if (__lane_id() == 0) GSD("wave %d phase B done\n", w);
  __syncthreads();
  if (threadIdx.x == 0) GSD("perm write\n");
  for (uint32_t i = threadIdx.x; i < n; i += GS_BLOCK) perm[lo + i] = lo + (L.d[i] & ((1u << SH) - 1));
  return true;
}

// ---- kernels -------------------------------------------------------------------------------------
// Level kernel: one workgroup per segment larger than T_LDS, partitioned in place in HBM; children
// are routed to the next level (large) or to the LDS list.
__device__ __forceinline__ void route(Seg s, uint32_t* cnt, Seg* big, Seg* lds, Seg* heap) {
  const uint32_t n = s.hi - s.lo;
  if (n <= 1) return;
  if (n <= T_LDS) {
    lds[atomicAdd(&cnt[1], 1u)] = s;
  } else if (s.depth == 0) {
    heap[atomicAdd(&cnt[2], 1u)] = s;
  } else {
    big[atomicAdd(&cnt[0], 1u)] = s;
  }
}

__global__ __launch_bounds__(GS_BLOCK) void k_gs_level(uint64_t* __restrict__ el, uint32_t* __restrict__ tmpA,
                                                       uint32_t* __restrict__ tmpB, const Seg* segs,
                                                       uint32_t nsegs, uint32_t* cnt, Seg* big, Seg* lds,
                                                       Seg* heap) {
  __shared__ uint32_t red[GS_BLOCK / 64 + 1];
  __shared__ uint32_t sh[8];
  for (uint32_t si = blockIdx.x; si < nsegs; si += gridDim.x) {
    const Seg sg = segs[si];
    uint32_t mlo, mhi;
    block_dopivot<32>(el, tmpA, tmpB, sg.lo, sg.hi, red, sh, &mlo, &mhi);
    if (threadIdx.x == 0) {
      route(Seg{sg.lo, mlo, sg.depth - 1, 0}, cnt, big, lds, heap);
      route(Seg{mhi, sg.hi, sg.depth - 1, 0}, cnt, big, lds, heap);
    }
    __syncthreads();
  }
}

// LDS kernel: one workgroup per segment of at most T_LDS elements, sorted to completion.
__global__ __launch_bounds__(GS_BLOCK) void k_gs_lds(uint64_t* __restrict__ el, uint32_t* __restrict__ perm,
                                                     const Seg* segs, uint32_t nsegs, uint32_t* cnt,
                                                     Seg* heap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  GsLds& L = *reinterpret_cast<GsLds*>(smem);
  for (uint32_t si = blockIdx.x; si < nsegs; si += gridDim.x) {
    const Seg sg = segs[si];
    const bool ok = lds_sort(el, perm, sg.lo, sg.hi - sg.lo, sg.depth, L);
    if (!ok && threadIdx.x == 0) heap[atomicAdd(&cnt[3], 1u)] = sg;  // lengths >= 2^18: HBM path
    __syncthreads();
  }
}

// Fallbacks in HBM: depth-exhausted heapSort (one thread per segment), and segments whose lengths do
// not fit the packed LDS format (quickSort by one workgroup, sequentially with cached pivots).
__global__ void k_gs_heap(uint64_t* el, const Seg* segs, uint32_t nsegs) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsegs; i += gridDim.x * blockDim.x)
    heap_sort<32>(el, segs[i].lo, segs[i].hi);
}

__global__ __launch_bounds__(GS_BLOCK) void k_gs_wide(uint64_t* __restrict__ el, uint32_t* __restrict__ tmpA,
                                                      uint32_t* __restrict__ tmpB, const Seg* segs,
                                                      uint32_t nsegs) {
  __shared__ uint32_t red[GS_BLOCK / 64 + 1];
  __shared__ uint32_t sh[8];
  __shared__ uint32_t stk[3 * 256];
  __shared__ uint32_t sp;
  for (uint32_t si = blockIdx.x; si < nsegs; si += gridDim.x) {
    if (threadIdx.x == 0) {
      stk[0] = segs[si].lo;
      stk[1] = segs[si].hi;
      stk[2] = (uint32_t)segs[si].depth;
      sp = 1;
    }
    __syncthreads();
    while (sp > 0) {
      const uint32_t a = stk[3 * (sp - 1)], b = stk[3 * (sp - 1) + 1];
      const int32_t dep = (int32_t)stk[3 * (sp - 1) + 2];
      __syncthreads();
      if (threadIdx.x == 0) sp--;
      if (b - a <= 12) {
        if (b - a > 1 && threadIdx.x < 64) wave_leaf<32>(el, a, b);
      } else if (dep == 0) {
        if (threadIdx.x == 0) heap_sort<32>(el, a, b);
      } else {
        uint32_t mlo, mhi;
        block_dopivot<32>(el, tmpA, tmpB, a, b, red, sh, &mlo, &mhi);
        if (threadIdx.x == 0) {
          stk[3 * sp] = a;
          stk[3 * sp + 1] = mlo;
          stk[3 * sp + 2] = (uint32_t)(dep - 1);
          stk[3 * sp + 3] = mhi;
          stk[3 * sp + 4] = b;
          stk[3 * sp + 5] = (uint32_t)(dep - 1);
          sp += 2;
        }
      }
      __syncthreads();
    }
  }
}

__global__ void k_gs_init(const uint64_t* gstart, uint32_t ngroups, uint32_t* perm, size_t n, uint32_t* cnt,
                          Seg* big, Seg* lds, Seg* heap) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    perm[i] = (uint32_t)i;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += gridDim.x * blockDim.x) {
    const uint32_t lo = (uint32_t)gstart[g], hi = (uint32_t)gstart[g + 1];
    uint32_t depth = 0;
    for (uint32_t i = hi - lo; i > 0; i >>= 1) depth++;  // maxDepth = 2*ceil(lg(n+1))
    route(Seg{lo, hi, (int32_t)(2 * depth), 0}, cnt, big, lds, heap);
  }
}

// Sorts every group's [gstart[g], gstart[g+1]) range with Go's sort.Sort semantics.
// Result: the element at sorted position r is el[perm[r]].
void gosort_groups(uint64_t* el, uint32_t* perm, size_t n, const uint64_t* gstart_dev, uint32_t ngroups,
                   hipStream_t s) {
  Context& c = ctx();
  const size_t maxseg = n / 2 + ngroups + 16;
  Seg* bigA = c.scratch.get<Seg>("gs_bigA", maxseg);
  Seg* bigB = c.scratch.get<Seg>("gs_bigB", maxseg);
  Seg* lds = c.scratch.get<Seg>("gs_lds", maxseg);
  Seg* heap = c.scratch.get<Seg>("gs_heap", maxseg);
  Seg* wide = c.scratch.get<Seg>("gs_wide", maxseg);
  uint32_t* tmpA = c.scratch.get<uint32_t>("gs_tmpA", n + 1);
  uint32_t* tmpB = c.scratch.get<uint32_t>("gs_tmpB", n + 1);
  uint32_t* cnt = c.scratch.get<uint32_t>("gs_cnt", 8);  // big, lds, heap, wide
  uint32_t* hcnt = c.pinned.get<uint32_t>(8);
  static bool attr_set = false;
  if (!attr_set) {
    SYZ_HIP(hipFuncSetAttribute((const void*)k_gs_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sizeof(GsLds)));
    attr_set = true;
  }
  SYZ_HIP(hipMemsetAsync(cnt, 0, 8 * sizeof(uint32_t), s));
  {
    ProfScope ps("gosort_init", s, (uint64_t)n * 4);
    k_gs_init<<<grid_for(std::max<size_t>(n, ngroups), 256, 2048), 256, 0, s>>>(gstart_dev, ngroups, perm, n, cnt,
                                                                                bigA, lds, heap);
    SYZ_LAUNCHED();
  }
  SYZ_HIP(hipMemcpyAsync(hcnt, cnt, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  // levels of segments larger than T_LDS (only the biggest call groups have any)
  for (int level = 0; hcnt[0] > 0; level++) {
    const uint32_t nbig = hcnt[0];
    SYZ_HIP(hipMemsetAsync(cnt, 0, sizeof(uint32_t), s));
    {
      ProfScope ps("gosort_level", s, 0);
      k_gs_level<<<std::min<uint32_t>(nbig, 2048), GS_BLOCK, 0, s>>>(el, tmpA, tmpB, bigA, nbig, cnt, bigB, lds,
                                                                     heap);
      SYZ_LAUNCHED();
    }
    std::swap(bigA, bigB);
    SYZ_HIP(hipMemcpyAsync(hcnt, cnt, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (level > 256) fail(SYZGPU_EINTERNAL, "gosort: level limit");
  }
  const uint32_t nlds = hcnt[1], nheap = hcnt[2];
  if (nheap) {
    k_gs_heap<<<grid_for(nheap, 64, 4096), 64, 0, s>>>(el, heap, nheap);
    SYZ_LAUNCHED();
  }
  if (nlds) {
    ProfScope ps("gosort_lds", s, (uint64_t)n * 12);
    SYZ_HIP(hipMemsetAsync(cnt + 3, 0, sizeof(uint32_t), s));
    k_gs_lds<<<std::min<uint32_t>(nlds, 4096), GS_BLOCK, sizeof(GsLds), s>>>(el, perm, lds, nlds, cnt, wide);
    SYZ_LAUNCHED();
    SYZ_HIP(hipMemcpyAsync(hcnt + 3, cnt + 3, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (hcnt[3]) {  // lengths beyond the packed LDS format: sort those segments in HBM
      k_gs_wide<<<std::min<uint32_t>(hcnt[3], 2048), GS_BLOCK, 0, s>>>(el, tmpA, tmpB, wide, hcnt[3]);
      SYZ_LAUNCHED();
    }
  }
}

}  // namespace syz

static_assert(sizeof(syz::GsLds) <= 160 * 1024, "gosort LDS budget");

// The permutation Go's sort.Sort (Go 1.6 .. 1.18 quickSort) produces for cover.Minimize's input array
// (cover/cover.go:106-113, minInputArray.Less = len(a[i].cov) > len(a[j].cov), :140-143), computed
// on the GPU for every call group at once.
//
// sort.Sort is unstable: among equal lengths the order depends on the exact sequence of swaps, and
// that order decides which inputs Minimize keeps. The simulation performs exactly the
// swaps of the sequential algorithm (Go 1.6-1.18 sort/sort.go quickSort, doPivot, insertionSort):
//   * the O(1) decisions of doPivot (Tukey ninther + medianOfThree, the dups probe) and the leaves
//     (gap-6 shell pass + insertionSort on <= 12 elements) and heapSort run as the SAME sequential
//     code, one thread per segment;
//   * the two O(n) loops of doPivot are replaced by their closed form: the Hoare loop swaps the k-th
//     misplaced element from the left (len < pivot len, left of the final boundary) with the k-th
//     misplaced element from the right, and the boundary is lo+1 + #(len >= pivot len); the
//     "protect" duplicate loop is the same pairing with (len <= pivot) vs (len > pivot) on [lo+1, b).
//     Counting and ordered compaction are data-parallel.
// Quicksort nodes of one level are independent, so they are processed LEVEL-SYNCHRONOUSLY:
//   segment > T_SEG   global levels: every segment of the level split into 4096-element tiles,
//                     one kernel per step (pivot / count / tile counts / lists / swap / probe /
//                     protect x4 / finish), children routed by size;
//   segment <= T_SEG  one workgroup per pack of segments in LDS (call groups <= T_SEG are packed
//                     up to T_SEG elements; global-level children get a workgroup each); inside, all
//                     active segments advance one doPivot per level with workgroup-wide scans.
// Elements are (len << 32) | position in HBM and (len << SH) | local index in LDS (u32 when every
// length of the pack fits, otherwise a u64 instantiation); Less only compares the length field.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "pipeline.hpp"

namespace syz {

#ifdef SYZ_GS_STATS
// diagnostic build only: [0] packs [1] levels [2] cycles total [3] pivot [4] part0 [5] probe [6] part1
// [7] children [8] heap sorts [9] heap elements [10] max active segments [11] leaves
__device__ unsigned long long g_gs_stats[24];
#define GS_STAT_ADD(i, v) atomicAdd(&g_gs_stats[i], (unsigned long long)(v))
#define GS_STAT_MAX(i, v) atomicMax(&g_gs_stats[i], (unsigned long long)(v))
#define GS_T() __builtin_amdgcn_s_memtime()
#else
#define GS_STAT_ADD(i, v)
#define GS_STAT_MAX(i, v)
#define GS_T() 0ull
#endif

constexpr uint32_t T_SEG = GS_T_SEG;  // largest segment sorted in LDS
// (GS_PACK_DIV, the pack size cap n / GS_PACK_DIV, and the packs themselves: plan_host.cpp gosort_segments)
#ifndef GS_T_CHILD_DEFAULT
#define GS_T_CHILD_DEFAULT T_SEG
#endif
#ifndef SYZ_LS_BLOCK
#define SYZ_LS_BLOCK 1024
#endif
constexpr int LS_BLOCK = SYZ_LS_BLOCK;  // LDS workgroup (1024: 16 waves, the wave sorter runs 16 segments at once)
constexpr int LS_ITEMS = T_SEG / LS_BLOCK;  // elements per thread chunk
constexpr int LS_ISH = LS_ITEMS == 8 ? 3 : LS_ITEMS == 16 ? 4 : -1;  // log2(LS_ITEMS)
static_assert((1 << LS_ISH) == LS_ITEMS, "LS_ISH");
constexpr int LS_SH = 13;  // local index bits of the packed u32 LDS element (T_SEG = 2^13)
static_assert((1u << LS_SH) == T_SEG, "LS_SH");
// Go's quickSort leaf form (gosort_leaf, syzgpu_set_go_sort_leaf): GO_LEAF12 = `for b-a > 12`, then a
// gap-6 shell pass + insertionSort (the default); GO_LEAF7 = `for b-a > 7`, then insertionSort alone.
// Which one the reference's Go release used is not pinned by anything in the reference.
constexpr int GO_LEAF12 = 12, GO_LEAF7 = 7;
template <int LEAF>
constexpr uint32_t ls_maxs() {  // active segments (> LEAF elements) per pack
  return T_SEG / (LEAF + 1) + 4;
}
// Children of the global rounds at most this long go to the LDS sorter; longer ones take another
// global round. Below T_SEG this trades one more (latency-bound) round for a shorter post-round LDS
// launch. Measured at config 4 (step ms): 8192 0.850, 4096 0.892, 2048 0.931 - the LDS launch barely
// shrinks (its per-level costs are mostly fixed), so T_SEG stays. SYZGPU_GS_T_CHILD overrides.
__constant__ uint32_t g_t_child = T_SEG;
static uint32_t t_child_host() {
  static const uint32_t v = [] {
    uint32_t x = GS_T_CHILD_DEFAULT;
    if (const char* e = dev_env("SYZGPU_GS_T_CHILD")) x = (uint32_t)atoi(e);
    if (x < 64) x = 64;
    if (x > T_SEG) x = T_SEG;
    SYZ_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_t_child), &x, sizeof(x)));
    return x;
  }();
  return v;
}
#ifndef SYZ_GL_BLOCK
#define SYZ_GL_BLOCK 256
#endif
#ifndef SYZ_GL_ITEMS
#define SYZ_GL_ITEMS 4
#endif
// Global-level tiles of 1024 elements: the rounds are latency-bound, so more, shorter tiles finish
// sooner (config 4 step: 4096-element tiles 0.841 ms, 2048 0.770, 1024 0.748, 512 0.761).
constexpr int GL_BLOCK = SYZ_GL_BLOCK;  // global-level tile workgroup
constexpr int GL_ITEMS = SYZ_GL_ITEMS;
constexpr uint32_t GL_TILE = GL_BLOCK * GL_ITEMS;

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

// ---- sequential pieces, exactly as Go sort/sort.go -------------------------------------------------
template <int SH, class P>
__device__ void seq_mo3(P d, uint32_t m1, uint32_t m0, uint32_t m2) {
  if (LT<SH>(d[m1], d[m0])) swp(d, m1, m0);
  if (LT<SH>(d[m2], d[m1])) {
    swp(d, m2, m1);
    if (LT<SH>(d[m1], d[m0])) swp(d, m1, m0);
  }
}

// doPivot's pivot choice; leaves the pivot at d[lo], returns m.
template <int SH, class P>
__device__ uint32_t seq_pivot(P d, uint32_t lo, uint32_t hi) {
  const uint32_t m = (uint32_t)(((uint64_t)lo + hi) >> 1);
  if (hi - lo > 40) {
    const uint32_t s = (hi - lo) / 8;
    seq_mo3<SH>(d, lo, lo + s, lo + 2 * s);
    seq_mo3<SH>(d, m, m - s, m + s);
    seq_mo3<SH>(d, hi - 1, hi - 1 - s, hi - 1 - 2 * s);
  }
  seq_mo3<SH>(d, lo, m, hi - 1);
  return m;
}

// doPivot after the Hoare loop (b == c == bnd): the dups probe. Returns protect.
template <int SH, class P>
__device__ bool seq_probe(P d, uint32_t lo, uint32_t hi, uint32_t m, uint32_t bnd, uint32_t* bout, uint32_t* cout) {
  uint32_t b = bnd, c = bnd;
  bool protect = hi - c < 5;
  if (!protect && hi - c < (hi - lo) / 4) {
    int dups = 0;
    if (!LT<SH>(d[lo], d[hi - 1])) {
      swp(d, c, hi - 1);
      c++;
      dups++;
    }
    if (!LT<SH>(d[b - 1], d[lo])) {
      b--;
      dups++;
    }
    if (!LT<SH>(d[m], d[lo])) {
      swp(d, m, b - 1);
      b--;
      dups++;
    }
    protect = dups > 1;
  }
  *bout = b;
  *cout = c;
  return protect;
}

// medianOfThree(data, m1, m0, m2) on register values: moves the median into a1 (= data[m1]).
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

// seq_pivot by a whole wave: the (at most 9, distinct) positions are loaded by 9 lanes at once, the
// medianOfThree network runs on registers in every lane, and the changed positions are stored back.
// One memory round trip each way instead of a dependent chain (used on el[] in HBM / L2).
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
    const T mine = lane < 9 ? d[pos] : T(0);
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
    const T mine = lane < 3 ? d[pos] : T(0);
    T v0 = __shfl(mine, 0), v1 = __shfl(mine, 1), v2 = __shfl(mine, 2);
    mo3v<SH>(v0, v1, v2);  // medianOfThree(lo, m, hi-1)
    const T out = lane == 0 ? v0 : (lane == 1 ? v1 : v2);
    if (lane < 3 && out != mine) d[pos] = out;
  }
  return m;
}

// seq_probe by a whole wave. Its positions hi-1, bnd, bnd-1, bnd-2, m are distinct whenever the
// probe runs (bnd > hi - (hi-lo)/4 and hi - bnd >= 5), and are cached by position.
template <int SH, class P>
__device__ bool wave_probe(P d, uint32_t lo, uint32_t hi, uint32_t m, uint32_t bnd, uint32_t* bout, uint32_t* cout) {
  using T = typename std::remove_reference<decltype(d[0])>::type;
  uint32_t b = bnd, c = bnd;
  bool protect = hi - c < 5;
  if (!protect && hi - c < (hi - lo) / 4) {
    const unsigned lane = __lane_id();
    const uint32_t p0 = hi - 1, p1 = bnd, p2 = bnd - 1, p3 = bnd - 2, p4 = m;
    const uint32_t pos = lane == 0 ? p0 : lane == 1 ? p1 : lane == 2 ? p2 : lane == 3 ? p3 : lane == 4 ? p4 : lo;
    const T mine = lane < 6 ? d[pos] : T(0);
    T v0 = __shfl(mine, 0), v1 = __shfl(mine, 1), v2 = __shfl(mine, 2), v3 = __shfl(mine, 3),
      v4 = __shfl(mine, 4);
    const T pv = __shfl(mine, 5);
    auto get = [&](uint32_t p) -> T { return p == p0 ? v0 : p == p1 ? v1 : p == p2 ? v2 : p == p3 ? v3 : v4; };
    auto set = [&](uint32_t p, T x) {
      if (p == p0) v0 = x;
      if (p == p1) v1 = x;
      if (p == p2) v2 = x;
      if (p == p3) v3 = x;
      if (p == p4) v4 = x;
    };
    int dups = 0;
    if (!LT<SH>(pv, get(hi - 1))) {  // data[hi-1] = pivot: swap(c, hi-1); c++
      const T t = get(c);
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
      const T t = get(m);
      set(m, get(b - 1));
      set(b - 1, t);
      b--;
      dups++;
    }
    protect = dups > 1;
    const T out = lane == 0 ? v0 : lane == 1 ? v1 : lane == 2 ? v2 : lane == 3 ? v3 : v4;
    if (lane < 5 && out != mine) d[pos] = out;
  }
  *bout = b;
  *cout = c;
  return protect;
}

// quickSort's tail for 2..12 elements (the LEAF 12 form): gap-6 shell pass, then insertionSort.
template <int SH, class P>
__device__ void seq_leaf(P d, uint32_t a, uint32_t b) {
  for (uint32_t i = a + 6; i < b; i++)
    if (LT<SH>(d[i], d[i - 6])) swp(d, i, i - 6);
  for (uint32_t i = a + 1; i < b; i++)
    for (uint32_t j = i; j > a && LT<SH>(d[j], d[j - 1]); j--) swp(d, j, j - 1);
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
__device__ void heap_sort(P d, uint32_t a, uint32_t b) {
  const uint32_t first = a, hi = b - a;
  for (int64_t i = ((int64_t)hi - 1) / 2; i >= 0; i--) sift_down<SH>(d, (uint32_t)i, hi, first);
  for (int64_t i = (int64_t)hi - 1; i >= 0; i--) {
    swp(d, first, first + (uint32_t)i);
    sift_down<SH>(d, 0, (uint32_t)i, first);
  }
}

// The same leaf in registers: the shell pass (LEAF 12 only) swaps the disjoint pairs (i-6, i), and
// insertionSort only moves an element past strictly Less ones, so it is the STABLE sort by Less: the
// element at i lands at #{j : Less(j, i)} + #{j < i : equal}. Loads and stores are independent (no LDS
// chains).
template <int SH, int LEAF, class P>
__device__ void reg_leaf(P d, uint32_t a, uint32_t n) {
  using E = typename std::remove_reference<decltype(d[0])>::type;
  E x[12];
#pragma unroll
  for (uint32_t i = 0; i < 12; i++) x[i] = i < n ? d[a + i] : (E)0;
#pragma unroll
  for (uint32_t i = 6; i < 12; i++)
    if (LEAF == GO_LEAF12 && i < n && LT<SH>(x[i], x[i - 6])) {
      const E t = x[i];
      x[i] = x[i - 6];
      x[i - 6] = t;
    }
#pragma unroll
  for (uint32_t i = 0; i < 12; i++) {
    if (i >= n) break;
    const uint32_t ki = KEY<SH>(x[i]);
    uint32_t r = 0;
#pragma unroll
    for (uint32_t j = 0; j < 12; j++) {
      const uint32_t kj = KEY<SH>(x[j]);
      r += (j < n && (kj > ki || (j < i && kj == ki))) ? 1u : 0u;
    }
    d[a + r] = x[i];
  }
}

// A node of quickSort(data, lo, hi, depth) that is not a doPivot: leaf or depth-exhausted heapSort.
template <int SH, int LEAF, class P>
__device__ void seq_terminal(P d, uint32_t lo, uint32_t hi, int32_t depth) {
  if (hi - lo <= LEAF) {
    if (hi - lo > 1) reg_leaf<SH, LEAF>(d, lo, hi - lo);
  } else if (depth == 0) {
    GS_STAT_ADD(8, 1);
    GS_STAT_ADD(9, hi - lo);
    heap_sort<SH>(d, lo, hi);
  }
}

// (go_max_depth: plan_host.hpp)

// =====================================================================================================
// LDS level-synchronous sorter: one workgroup per pack.
// =====================================================================================================
// (Pack: plan_host.hpp)

// LDS view of the pack's elements with one pad word per chunk: a thread's contiguous LS_ITEMS-element
// chunk then starts on its own bank, so chunk walks are conflict-free (a plain array is 8-way).
template <class E>
struct PadRef {
  E* v;
  __device__ __forceinline__ E& operator[](uint32_t i) const { return v[i + (i >> LS_ISH)]; }
};

template <class E, int LEAF>
struct LsLds {
  static constexpr uint32_t LS_MAXS = ls_maxs<LEAF>();
  E dv[T_SEG + T_SEG / LS_ITEMS];
  __device__ __forceinline__ PadRef<E> D() { return PadRef<E>{dv}; }
  uint16_t bl[T_SEG];               // misplaced-right positions, at lo + rank from the right
  uint32_t cpre[LS_BLOCK + 1];      // #left before each chunk (pass scan), [LS_BLOCK] = total
  uint32_t cmask[LS_BLOCK];         // left bits of each chunk
  uint16_t lo[2][LS_MAXS], hi[2][LS_MAXS];
  int8_t dep[2][LS_MAXS];
  uint32_t pl[LS_MAXS], cnt[LS_MAXS];  // cnt: T | (#left before the range << 16) of the pass
  uint16_t m[LS_MAXS], bnd[LS_MAXS], b[LS_MAXS], c[LS_MAXS];
  uint8_t prot[LS_MAXS];
  uint32_t wl[LS_MAXS];  // segments of LEAF+1..WQ elements for the wave sorter: lo | hi << 16
  int8_t wd[LS_MAXS];    // and their depth budget
  uint32_t red[LS_BLOCK / 64 + 1];
  uint32_t na, tot, flag, anyprot, nw;
};

// first active segment with hi > p (segments sorted, disjoint)
template <class L>
__device__ __forceinline__ uint32_t seg_at(const L& S, int cur, uint32_t na, uint32_t p) {
  uint32_t a = 0, z = na;
  while (a < z) {
    const uint32_t mid = (a + z) >> 1;
    if (S.hi[cur][mid] <= p)
      a = mid + 1;
    else
      z = mid;
  }
  return a;
}

// One pass of doPivot's O(n) loop over every active segment of the pack: mode 0 = Hoare pass
// (stays left: len >= pivot len, on [lo+1, hi-1)), mode 1 = protect pass (stays left: len > pivot
// len, on [lo+1, b)).
// Closed form (as in the global rounds): with L(p) = #left in [a, p) and T = #left in [a, e), the
// boundary is a + T; a misplaced-left element (not left, p < bnd) has rank (p - a) - L(p) from the
// left, a misplaced-right one (left, p >= bnd) has rank T - 1 - L(p) from the right, and the loop
// swaps equal ranks. L comes from ONE workgroup scan of per-chunk left counts (no atomics); the
// misplaced-right positions go to a list indexed inside the segment's own range, and each
// misplaced-left element fetches its partner from it and performs the swap.
// Thread t owns the chunk [8t, 8t+8). Active segments have more than WQ elements, so a chunk meets at
// most 2 of them (the code allows 3: sf .. sf+2).
// bits j of a chunk starting at i0 whose position lies in [a, e)
__device__ __forceinline__ uint32_t chunk_range(uint32_t i0, uint32_t a, uint32_t e) {
  const int32_t lo = max(0, min((int32_t)LS_ITEMS, (int32_t)a - (int32_t)i0));
  const int32_t hi = max(0, min((int32_t)LS_ITEMS, (int32_t)e - (int32_t)i0));
  return (uint32_t)((1ull << hi) - 1ull) & ~(uint32_t)((1ull << lo) - 1ull);  // 0 when hi <= lo
}

// #left in [0, p) of the pack (p <= T_SEG), from the chunk prefixes and masks
template <class L>
__device__ __forceinline__ uint32_t ls_lpre(const L& S, uint32_t p) {
  const uint32_t t = p >> LS_ISH, j = p & (LS_ITEMS - 1u);
  return j ? S.cpre[t] + __popc(S.cmask[t] & ((1u << j) - 1u)) : S.cpre[t];
}

template <int SH, class E, class L>
__device__ void ls_partition(L& S, int cur, uint32_t na, uint32_t n, int mode) {
  unsigned long long tq0 = GS_T();
  (void)tq0;
  const uint32_t i0 = threadIdx.x * LS_ITEMS;
  uint32_t sf = 0, mseg[3] = {0, 0, 0}, slo[3] = {0, 0, 0}, inr = 0, left = 0;
  bool live = i0 < n && na > 0;
  if (live) {
    sf = seg_at(S, cur, na, i0);
    live = sf < na && S.lo[cur][sf] < i0 + LS_ITEMS;
  }
  if (live) {
    uint32_t key[LS_ITEMS];
#pragma unroll
    for (int i = 0; i < LS_ITEMS; i++) key[i] = KEY<SH>(S.D()[i0 + i]);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const uint32_t ss = sf + k;
      if (ss >= na) break;
      const uint32_t lo = S.lo[cur][ss];
      if (lo >= i0 + LS_ITEMS) break;
      slo[k] = lo;
      mseg[k] = chunk_range(i0, lo, S.hi[cur][ss]);
      if (mode == 1 && !S.prot[ss]) continue;
      const uint32_t r = chunk_range(i0, lo + 1, mode == 0 ? S.hi[cur][ss] - 1u : (uint32_t)S.b[ss]);
      if (!r) continue;
      const uint32_t pl = S.pl[ss];
      uint32_t ge = 0;
#pragma unroll
      for (int i = 0; i < LS_ITEMS; i++) ge |= ((mode == 0 ? key[i] >= pl : key[i] > pl) ? 1u : 0u) << i;
      inr |= r;
      left |= r & ge;
    }
  }
  uint32_t tot;
  const uint32_t pre = block_excl_scan<LS_BLOCK>((uint32_t)__popc(left), S.red, &tot);
  S.cpre[threadIdx.x] = pre;
  S.cmask[threadIdx.x] = left;
  if (threadIdx.x == 0) S.cpre[LS_BLOCK] = tot;
  __syncthreads();
  unsigned long long tq1 = GS_T();
  // per segment: the boundary and the left count before the range
  for (uint32_t q = threadIdx.x; q < na; q += LS_BLOCK) {
    if (mode == 1 && !S.prot[q]) continue;
    const uint32_t a = S.lo[cur][q] + 1u, e = mode == 0 ? S.hi[cur][q] - 1u : (uint32_t)S.b[q];
    if (a >= e) {
      S.bnd[q] = (uint16_t)a;
      S.cnt[q] = 0;
      continue;
    }
    const uint32_t la = ls_lpre(S, a), T = ls_lpre(S, e) - la;
    S.bnd[q] = (uint16_t)(a + T);
    S.cnt[q] = T | (la << 16);
  }
  __syncthreads();
  unsigned long long tq2 = GS_T();
  // misplaced-right: B[lo + rank from the right] = p; misplaced-left: remembered in ml
  uint32_t ml = 0;
  uint32_t sbd[3] = {0, 0, 0}, sT[3] = {0, 0, 0}, sla[3] = {0, 0, 0};
  if (inr) {
#pragma unroll
    for (int k = 0; k < 3; k++)
      if (mseg[k] & inr) {
        const uint32_t cv = S.cnt[sf + k];
        sbd[k] = S.bnd[sf + k];
        sT[k] = cv & 0xFFFFu;
        sla[k] = cv >> 16;
      }
    uint32_t lp = pre;
#pragma unroll
    for (int i = 0; i < LS_ITEMS; i++) {
      if ((inr >> i) & 1u) {
        const uint32_t p = i0 + i;
        const uint32_t k = ((mseg[0] >> i) & 1u) ? 0u : (((mseg[1] >> i) & 1u) ? 1u : 2u);
        const uint32_t bd = k == 0 ? sbd[0] : (k == 1 ? sbd[1] : sbd[2]);
        const bool lf = (left >> i) & 1u;
        if (!lf && p < bd) ml |= 1u << i;
        if (lf && p >= bd) {
          const uint32_t T = k == 0 ? sT[0] : (k == 1 ? sT[1] : sT[2]);
          const uint32_t la = k == 0 ? sla[0] : (k == 1 ? sla[1] : sla[2]);
          const uint32_t lo = k == 0 ? slo[0] : (k == 1 ? slo[1] : slo[2]);
          S.bl[lo + T - 1u - (lp - la)] = (uint16_t)p;
        }
        lp += lf ? 1u : 0u;
      }
    }
  }
  __syncthreads();
  unsigned long long tq3 = GS_T();
  if (ml) {  // the swaps, by the misplaced-left side (pairs are disjoint); loads before stores
    uint32_t lp = pre;
    uint32_t qq[LS_ITEMS];
#pragma unroll
    for (int i = 0; i < LS_ITEMS; i++) {
      qq[i] = 0;
      if ((ml >> i) & 1u) {
        const uint32_t p = i0 + i;
        const uint32_t k = ((mseg[0] >> i) & 1u) ? 0u : (((mseg[1] >> i) & 1u) ? 1u : 2u);
        const uint32_t la = k == 0 ? sla[0] : (k == 1 ? sla[1] : sla[2]);
        const uint32_t lo = k == 0 ? slo[0] : (k == 1 ? slo[1] : slo[2]);
        qq[i] = S.bl[lo + (p - lo - 1u) - (lp - la)];  // partner: same rank from the right
      }
      lp += (left >> i) & 1u;
    }
    E vp[LS_ITEMS], vq[LS_ITEMS];
#pragma unroll
    for (int i = 0; i < LS_ITEMS; i++)
      if ((ml >> i) & 1u) {
        vp[i] = S.D()[i0 + i];
        vq[i] = S.D()[qq[i]];
      }
#pragma unroll
    for (int i = 0; i < LS_ITEMS; i++)
      if ((ml >> i) & 1u) {
        S.D()[i0 + i] = vq[i];
        S.D()[qq[i]] = vp[i];
      }
  }
  __syncthreads();
  if (threadIdx.x == 0 && mode == 0) {
    GS_STAT_ADD(12, tq1 - tq0);
    GS_STAT_ADD(13, tq2 - tq1);
    GS_STAT_ADD(14, tq3 - tq2);
    GS_STAT_ADD(15, GS_T() - tq3);
  }
  (void)tq1; (void)tq2; (void)tq3;
}

// ---- wave sorter: a segment of LEAF+1..WQ elements finished by one wave, one element per lane ---------
// Level-synchronous inside the wave: every lane knows its segment [s, e) (lane-relative) and depth,
// all segments of the subtree advance one quickSort node per iteration, and doPivot's steps are
// ballots (counts, ranks), shuffles (pivot-of-nine, probe, partner exchange) and two per-wave LDS
// slot lists (the k-th misplaced element of a segment). No workgroup barriers.
constexpr uint32_t WQ = 64;

__device__ __forceinline__ uint64_t lmask(uint32_t a, uint32_t b) {  // lanes [a, b), 0 <= a, b <= 64
  const uint64_t h = b >= 64 ? ~0ull : ((1ull << b) - 1ull);
  const uint64_t l = a >= 64 ? ~0ull : ((1ull << a) - 1ull);
  return h & ~l;
}

// one O(n) loop of doPivot for every active lane segment: range [s+1, z), mode 0 stays left on
// key >= pl, mode 1 on key > pl; returns the boundary s+1 + #left
template <int SH, class E>
__device__ __forceinline__ uint32_t wv_pass(E& v, uint32_t lane, bool act, uint32_t s, uint32_t e, uint32_t z,
                                            uint32_t pl, int mode, uint8_t* slL, uint8_t* slR) {
  const uint32_t a = s + 1;
  const bool inr = act && lane >= a && lane < z;
  const uint32_t key = KEY<SH>(v);
  const bool lf = inr && (mode == 0 ? key >= pl : key > pl);
  const uint64_t BL = __ballot(lf);
  const uint32_t bnd = a + ((act && z > a) ? (uint32_t)__popcll(BL & lmask(a, z)) : 0u);
  const bool ml = inr && !lf && lane < bnd, mr = inr && lf && lane >= bnd;
  const uint64_t BML = __ballot(ml), BMR = __ballot(mr);
  if (BML) {
    const uint32_t rl = (uint32_t)__popcll(BML & lmask(s, lane));
    const uint32_t rr = (uint32_t)__popcll(BMR & lmask(lane + 1, e));
    if (ml) slL[s + rl] = (uint8_t)lane;
    if (mr) slR[s + rr] = (uint8_t)lane;
    wave_sync();
    uint32_t partner = lane;
    if (ml) partner = slR[s + rl];
    if (mr) partner = slL[s + rr];
    const E pv = __shfl(v, (int)partner);
    if (ml || mr) v = pv;
    wave_sync();
  }
  return bnd;
}

template <int SH, int LEAF, class E, class L>
__device__ void wave_qs(L& S, uint32_t lo, uint32_t hi, int32_t dep0, uint8_t* slL, uint8_t* slR, E* slV) {
  const uint32_t lane = __lane_id(), n = hi - lo;
  E v = lane < n ? S.D()[lo + lane] : (E)0;
  uint32_t s = 0, e = lane < n ? n : 0;  // this lane's segment; e <= s: finished
  int32_t d = dep0;
  for (;;) {
    const uint32_t len = e > s ? e - s : 0u;
    const bool leaf = len >= 2 && len <= LEAF;
    const bool hp = len > LEAF && d <= 0;
    const bool act = len > LEAF && d > 0;
    if (__ballot(leaf)) {  // quickSort's tail: (LEAF 12) gap-6 shell pass (disjoint pairs), then
                           // insertionSort, which is the stable sort by Less
      const E up = __shfl(v, (int)(lane >= 6 ? lane - 6 : lane));
      const E dn = __shfl(v, (int)(lane + 6 < 64 ? lane + 6 : lane));
      if (LEAF == GO_LEAF12 && leaf) {
        if (lane >= s + 6) {
          if (LT<SH>(v, up)) v = up;
        } else if (lane + 6 < e) {
          if (LT<SH>(dn, v)) v = dn;
        }
      }
      const uint32_t k = KEY<SH>(v);
      uint32_t r = 0;
#pragma unroll
      for (uint32_t j = 0; j < 12; j++) {
        const uint32_t kx = KEY<SH>(__shfl(v, (int)min(s + j, 63u)));
        r += (s + j < e && (kx > k || (kx == k && s + j < lane))) ? 1u : 0u;
      }
      if (leaf) slV[s + r] = v;
      wave_sync();
      if (leaf) v = slV[lane];
      wave_sync();
    }
    if (__ballot(hp)) {  // depth budget exhausted: heapSort by the segment's first lane, in LDS
      if (lane < n) S.D()[lo + lane] = v;
      wave_sync();
      if (hp && lane == s) heap_sort<SH>(S.D(), lo + s, lo + e);
      wave_sync();
      if (lane < n) v = S.D()[lo + lane];
    }
    if (leaf || hp) s = e = lane;
    if (!__ballot(act)) break;
    // pivot choice (pivot-of-nine above 40 elements, then medianOfThree), moved into place
    const uint32_t m = (s + e) >> 1, t = len / 8;
    const bool nine = act && len > 40;
    uint32_t P[9];
    if (nine) {
      P[0] = s; P[1] = s + t; P[2] = s + 2 * t; P[3] = m - t; P[4] = m; P[5] = m + t;
      P[6] = e - 1 - 2 * t; P[7] = e - 1 - t; P[8] = e - 1;
    } else {
#pragma unroll
      for (int j = 0; j < 9; j++) P[j] = lane;
      if (act) {
        P[0] = s; P[1] = m; P[2] = e - 1;
      }
    }
    E x[9];
#pragma unroll
    for (int j = 0; j < 9; j++) x[j] = __shfl(v, (int)P[j]);
    if (nine) {
      mo3v<SH>(x[0], x[1], x[2]);
      mo3v<SH>(x[4], x[3], x[5]);
      mo3v<SH>(x[8], x[7], x[6]);
      mo3v<SH>(x[0], x[4], x[8]);
    } else if (act) {
      mo3v<SH>(x[0], x[1], x[2]);
    }
    if (act) {
#pragma unroll
      for (int j = 0; j < 9; j++)
        if (lane == P[j] && (nine || j < 3)) v = x[j];
    }
    const uint32_t pl = KEY<SH>(x[0]);
    // Hoare pass
    const uint32_t bnd = wv_pass<SH, E>(v, lane, act, s, e, e - 1, pl, 0, slL, slR);
    // dups probe on positions e-1, bnd, bnd-1, bnd-2, m (distinct whenever it runs) and pivot s
    uint32_t b = bnd, c = bnd;
    bool prot = act && e - c < 5;
    const bool probe = act && !prot && e - c < len / 4;
    const uint32_t q0 = probe ? e - 1 : lane, q1 = probe ? bnd : lane, q2 = probe ? bnd - 1 : lane,
                   q3 = probe ? bnd - 2 : lane, q4 = probe ? m : lane, qs = probe ? s : lane;
    E y0 = __shfl(v, (int)q0), y1 = __shfl(v, (int)q1), y2 = __shfl(v, (int)q2), y3 = __shfl(v, (int)q3),
      y4 = __shfl(v, (int)q4);
    const E pv = __shfl(v, (int)qs);
    if (probe) {
      auto get = [&](uint32_t p) -> E { return p == q0 ? y0 : p == q1 ? y1 : p == q2 ? y2 : p == q3 ? y3 : y4; };
      auto set = [&](uint32_t p, E w) {
        if (p == q0) y0 = w;
        if (p == q1) y1 = w;
        if (p == q2) y2 = w;
        if (p == q3) y3 = w;
        if (p == q4) y4 = w;
      };
      int dups = 0;
      if (!LT<SH>(pv, get(e - 1))) {  // data[hi-1] = pivot: swap(c, hi-1), c++
        const E w = get(c);
        set(c, get(e - 1));
        set(e - 1, w);
        c++;
        dups++;
      }
      if (!LT<SH>(get(b - 1), pv)) {  // data[b-1] = pivot
        b--;
        dups++;
      }
      if (!LT<SH>(get(m), pv)) {  // data[m] = pivot: swap(m, b-1), b--
        const E w = get(m);
        set(m, get(b - 1));
        set(b - 1, w);
        b--;
        dups++;
      }
      prot = dups > 1;
      if (lane == q0) v = y0;
      else if (lane == q1) v = y1;
      else if (lane == q2) v = y2;
      else if (lane == q3) v = y3;
      else if (lane == q4) v = y4;
    }
    if (__ballot(prot)) {  // the protect pass over [s+1, b)
      const uint32_t b2 = wv_pass<SH, E>(v, lane, prot, s, e, b, pl, 1, slL, slR);
      if (prot) b = b2;
    }
    // pivot into its final place b-1; children [s, b-1) and [c, e)
    const E xs = __shfl(v, (int)(act ? s : lane)), xb = __shfl(v, (int)(act ? b - 1 : lane));
    if (act) {
      if (lane == s) v = xb;
      if (lane == b - 1) v = xs;
      if (lane < b - 1) e = b - 1;
      else if (lane >= c) s = c;
      else s = e = lane;
      d--;
    }
  }
  if (lane < n) S.D()[lo + lane] = v;
}

template <class L>
__device__ __forceinline__ void ls_wave_push(L& S, uint32_t lo, uint32_t hi, int32_t dep) {
  const uint32_t i = atomicAdd(&S.nw, 1u);
  S.wl[i] = lo | (hi << 16);
  S.wd[i] = (int8_t)dep;
}

template <int SH, class E, int LEAF>
__global__ __launch_bounds__(LS_BLOCK) void k_ls_sort(const uint64_t* __restrict__ el, uint32_t* __restrict__ perm,
                                                      const Pack* __restrict__ packs, uint32_t npacks_host,
                                                      const uint32_t* npacks_dev, const Seg* __restrict__ segs,
                                                      uint32_t* bounce_cnt, Pack* bounce) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  LsLds<E, LEAF>& S = *reinterpret_cast<LsLds<E, LEAF>*>(smem);
  constexpr uint64_t LEN_LIMIT = SH >= 32 ? ~0ull : (1ull << (sizeof(E) * 8 - SH));
  // packs == nullptr: the items are single segments segs[range[0] .. range[1]) (children of the global
  // levels, npacks_dev points at that range)
  const uint32_t base = packs ? 0 : npacks_dev[0];
  const uint32_t npacks = packs ? (npacks_dev ? *npacks_dev : npacks_host) : npacks_dev[1] - npacks_dev[0];
  for (uint32_t pi = blockIdx.x; pi < npacks; pi += gridDim.x) {
    Pack pk;
    if (packs) {
      pk = packs[pi];
    } else {
      const Seg sg = segs[base + pi];
      pk = Pack{sg.lo, sg.hi, base + pi, base + pi + 1};
    }
    const uint32_t n = pk.phi - pk.plo;
    if (threadIdx.x == 0) {
      S.flag = 0;
      S.na = 0;
      S.nw = 0;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += LS_BLOCK) {
      const uint64_t len = el[pk.plo + i] >> 32;
      if (len >= LEN_LIMIT) S.flag = 1;
      S.D()[i] = (E)(((E)len << SH) | (E)i);
    }
    __syncthreads();
    if (S.flag) {  // a length does not fit this element format: the wide instantiation takes it
      if (threadIdx.x == 0) bounce[atomicAdd(bounce_cnt, 1u)] = pk;
      __syncthreads();
      continue;
    }
    // initial segments: terminal ones are finished right here, the others become active (in order)
    {
      const uint32_t ns = pk.send - pk.sbeg;
      uint32_t tot;
      // ordered placement: contiguous per-thread ranges of segments, counted then scanned
      const uint32_t per = (ns + LS_BLOCK - 1) / LS_BLOCK;
      const uint32_t k0 = threadIdx.x * per, k1 = min(ns, k0 + per);
      uint32_t cntA = 0;
      for (uint32_t k = k0; k < k1; k++) {
        const Seg sg = segs[pk.sbeg + k];
        if (sg.hi - sg.lo > WQ && sg.depth > 0) cntA++;
      }
      uint32_t o = block_excl_scan<LS_BLOCK>(cntA, S.red, &tot);
      for (uint32_t k = k0; k < k1; k++) {
        const Seg sg = segs[pk.sbeg + k];
        const uint32_t lo = sg.lo - pk.plo, hi = sg.hi - pk.plo;
        if (hi - lo > WQ && sg.depth > 0) {
          S.lo[0][o] = (uint16_t)lo;
          S.hi[0][o] = (uint16_t)hi;
          S.dep[0][o] = (int8_t)sg.depth;
          o++;
        } else if (hi - lo > LEAF && sg.depth > 0) {
          ls_wave_push(S, lo, hi, sg.depth);
        } else {
          seq_terminal<SH, LEAF>(S.D(), lo, hi, sg.depth);
        }
      }
      if (threadIdx.x == 0) S.na = tot;
      __syncthreads();
    }
    int cur = 0;
    unsigned long long nlev = 0;
    (void)nlev;
    unsigned long long tA = GS_T(), tB, tC, tD, tE, tF, tS = tA;
    (void)tB; (void)tC; (void)tD; (void)tE; (void)tF; (void)tS;
    if (threadIdx.x == 0) GS_STAT_ADD(0, 1);
    while (S.na > 0) {
      const uint32_t na = S.na;
      if (threadIdx.x == 0) {
        GS_STAT_ADD(1, 1);
        GS_STAT_MAX(10, na);
        nlev++;
      }
      tA = GS_T();
      // pivot choice, one thread per segment
      for (uint32_t s = threadIdx.x; s < na; s += LS_BLOCK) {
        const uint32_t lo = S.lo[cur][s], hi = S.hi[cur][s];
        S.m[s] = (uint16_t)seq_pivot<SH>(S.D(), lo, hi);
        S.pl[s] = KEY<SH>(S.D()[lo]);
        S.cnt[s] = 0;
      }
      if (threadIdx.x == 0) S.anyprot = 0;
      __syncthreads();
      tB = GS_T();
      ls_partition<SH, E>(S, cur, na, n, 0);
      tC = GS_T();
      // dups probe, one thread per segment
      for (uint32_t s = threadIdx.x; s < na; s += LS_BLOCK) {
        uint32_t b, c;
        S.prot[s] = seq_probe<SH>(S.D(), S.lo[cur][s], S.hi[cur][s], S.m[s], S.bnd[s], &b, &c);
        S.b[s] = (uint16_t)b;
        S.c[s] = (uint16_t)c;
        S.cnt[s] = 0;
        if (S.prot[s]) S.anyprot = 1;
      }
      __syncthreads();
      tD = GS_T();
      if (S.anyprot) ls_partition<SH, E>(S, cur, na, n, 1);
      tE = GS_T();
      // pivot into the middle; children: terminal ones finish now, the others stay active in order
      const uint32_t per = (na + LS_BLOCK - 1) / LS_BLOCK;
      const uint32_t s0 = threadIdx.x * per, s1 = min(na, s0 + per);
      uint32_t cntA = 0;
      for (uint32_t s = s0; s < s1; s++) {
        const uint32_t lo = S.lo[cur][s], hi = S.hi[cur][s];
        const uint32_t b = S.prot[s] ? S.bnd[s] : S.b[s];
        const uint32_t mlo = b - 1, mhi = S.c[s];
        const int32_t dep = S.dep[cur][s] - 1;
        swp(S.D(), lo, b - 1);
        S.b[s] = (uint16_t)mlo;  // reuse: child boundaries
        if (mlo - lo > WQ && dep > 0) cntA++;
        else if (mlo - lo > LEAF && dep > 0) ls_wave_push(S, lo, mlo, dep);
        else seq_terminal<SH, LEAF>(S.D(), lo, mlo, dep);
        if (hi - mhi > WQ && dep > 0) cntA++;
        else if (hi - mhi > LEAF && dep > 0) ls_wave_push(S, mhi, hi, dep);
        else seq_terminal<SH, LEAF>(S.D(), mhi, hi, dep);
      }
      uint32_t tot;
      uint32_t o = block_excl_scan<LS_BLOCK>(cntA, S.red, &tot);
      const int nx = cur ^ 1;
      for (uint32_t s = s0; s < s1; s++) {
        const uint32_t lo = S.lo[cur][s], hi = S.hi[cur][s];
        const uint32_t mlo = S.b[s], mhi = S.c[s];
        const int32_t dep = S.dep[cur][s] - 1;
        if (mlo - lo > WQ && dep > 0) {
          S.lo[nx][o] = (uint16_t)lo;
          S.hi[nx][o] = (uint16_t)mlo;
          S.dep[nx][o] = (int8_t)dep;
          o++;
        }
        if (hi - mhi > WQ && dep > 0) {
          S.lo[nx][o] = (uint16_t)mhi;
          S.hi[nx][o] = (uint16_t)hi;
          S.dep[nx][o] = (int8_t)dep;
          o++;
        }
      }
      __syncthreads();
      if (threadIdx.x == 0) S.na = tot;
      cur = nx;
      __syncthreads();
      tF = GS_T();
      if (threadIdx.x == 0) {
        GS_STAT_ADD(3, tB - tA);
        GS_STAT_ADD(4, tC - tB);
        GS_STAT_ADD(5, tD - tC);
        GS_STAT_ADD(6, tE - tD);
        GS_STAT_ADD(7, tF - tE);
      }
    }
    {  // the wave sorter's segments, one per wave at a time
      __syncthreads();
      const uint32_t nw = S.nw, w = threadIdx.x >> 6;
      uint8_t* scr = reinterpret_cast<uint8_t*>(S.bl) + w * (128 + 64 * sizeof(E));
      for (uint32_t it = w; it < nw; it += LS_BLOCK / 64) {
        const uint32_t x = S.wl[it];
        wave_qs<SH, LEAF, E>(S, x & 0xFFFFu, x >> 16, S.wd[it], scr, scr + 64, reinterpret_cast<E*>(scr + 128));
      }
      __syncthreads();
      if (threadIdx.x == 0) GS_STAT_ADD(11, nw);
    }
    if (threadIdx.x == 0) {
      GS_STAT_ADD(2, GS_T() - tS);
      GS_STAT_MAX(16, GS_T() - tS);  // slowest pack: cycles, its levels, its size
      GS_STAT_MAX(17, ((GS_T() - tS) << 24) | ((unsigned long long)nlev << 14) | n);
    }
    constexpr E MASK = (E)((1ull << SH) - 1);
    for (uint32_t i = threadIdx.x; i < n; i += LS_BLOCK) perm[pk.plo + i] = pk.plo + (uint32_t)(S.D()[i] & MASK);
    __syncthreads();
  }
}

// =====================================================================================================
// Global levels: segments larger than T_SEG, in place in el[] (HBM / L2).
// =====================================================================================================
// One ROUND advances every big segment by one pass of doPivot's O(n) loops, in three kernels:
//   k_gr_count  per 4096-element tile: #(stays left) in the pass range
//   k_gr_lists  per tile: the rank of every misplaced element straight from the prefix of "stays
//               left" counts (no second scan): with L(p) = #left in [a, p) and T = #left in [a, e),
//               the boundary is a + T, a misplaced-left element (not left, p < bnd) has rank
//               k = (p - a) - L(p) from the left, a misplaced-right one (left, p >= bnd) has rank
//               T - 1 - L(p) from the right, and the Hoare loop swaps equal ranks
//   k_gr_swap   the swaps; the last tile of a segment to finish (agent-scope release / acquire
//               through a per-segment arrival counter) runs the segment's O(1) tail: the dups probe,
//               then either re-admits the segment for its protect pass next round or swaps the
//               pivot into place and routes the children (next round / LDS sorter / heapSort).
// A round is three dependent launches; the protect pass costs its segment one extra round.
typedef __attribute__((address_space(1))) unsigned long long gu64;  // global (not flat) 8-byte word

struct GLvl {
  uint32_t pl, m, bnd, b, c, mode, ng, pad;  // mode 0: Hoare pass, 1: protect pass
};

struct GCtl {
  uint32_t nnext, nlds, nheap, round;  // nnext stays 0: [nnext, nlds) is the LDS children range
};

struct GPlan {
  uint32_t nseg, ntiles;
};

struct GLevel {
  Seg* segs;
  GLvl* lv;
  uint32_t* toff;
  uint32_t* done;  // tiles of the segment whose swaps have been published
  uint2* tseg;
  GPlan* plan;
};

__device__ __forceinline__ uint32_t gl_ntiles(const Seg& sg) { return (sg.hi - sg.lo + GL_TILE - 1) / GL_TILE; }

// one wave: reserve the segment's tiles in nx and publish its pass state
__device__ __forceinline__ void gl_enter(const Seg& sg, const GLvl& L, uint32_t idx, GLevel nx) {
  const uint32_t nt = gl_ntiles(sg);
  uint32_t t0 = 0;
  if (__lane_id() == 0) t0 = atomicAdd(&nx.plan->ntiles, nt);
  t0 = __shfl(t0, 0);
  for (uint32_t t = __lane_id(); t < nt; t += 64) nx.tseg[t0 + t] = make_uint2(idx, t);
  if (__lane_id() == 0) {
    nx.segs[idx] = sg;
    nx.toff[idx] = t0;
    nx.done[idx] = 0;
    nx.lv[idx] = L;
  }
}

// one wave: a new doPivot node enters the next round (pivot choice, Hoare pass)
__device__ __forceinline__ void gl_admit(uint64_t* el, const Seg& sg, GLevel nx) {
  uint32_t idx = 0;
  if (__lane_id() == 0) idx = atomicAdd(&nx.plan->nseg, 1u);
  idx = __shfl(idx, 0);
  const uint32_t m = wave_pivot<32>(el, sg.lo, sg.hi);
  wave_sync();
  GLvl L{};
  L.m = m;
  if (__lane_id() == 0) L.pl = KEY<32>(el[sg.lo]);
  gl_enter(sg, L, idx, nx);
}

// initial round: the big call groups; the call's epoch tags the host progress words
__global__ __launch_bounds__(64) void k_gl_init(uint64_t* el, const Seg* big, uint32_t nbig, GLevel nx, GCtl* ctl,
                                                uint32_t epoch) {
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl->round = epoch << 16;
  for (uint32_t i = blockIdx.x; i < nbig; i += gridDim.x) gl_admit(el, big[i], nx);
}

// the range and the "stays left" predicate of a pass
__device__ __forceinline__ bool gl_range(const Seg& sg, const GLvl& L, uint32_t* a, uint32_t* e) {
  *a = sg.lo + 1;
  *e = L.mode == 0 ? sg.hi - 1 : L.b;
  return *a < *e;
}
__device__ __forceinline__ bool gl_left(uint32_t k, const GLvl& L) { return L.mode == 0 ? k >= L.pl : k > L.pl; }

__device__ __forceinline__ void gr_count(const uint64_t* el, const GLevel& cur, uint32_t ntiles, uint32_t* tcnt,
                                         uint32_t* red) {
  for (uint32_t tb = blockIdx.x; tb < ntiles; tb += gridDim.x) {
    const uint2 st = cur.tseg[tb];
    const Seg sg = cur.segs[st.x];
    const GLvl L = cur.lv[st.x];
    uint32_t a, e, c = 0;
    if (gl_range(sg, L, &a, &e)) {
      const uint32_t t0 = sg.lo + st.y * GL_TILE;
#pragma unroll 4
      for (int i = 0; i < GL_ITEMS; i++) {
        const uint32_t p = t0 + i * GL_BLOCK + threadIdx.x;
        if (p >= a && p < e) c += gl_left(KEY<32>(el[p]), L) ? 1u : 0u;
      }
    }
    c = block_sum<GL_BLOCK>(c, red);
    if (threadIdx.x == 0) tcnt[tb] = c;
  }
}


__global__ __launch_bounds__(GL_BLOCK) void k_gr_count(const uint64_t* el, GLevel cur, GPlan* next_plan,
                                                       uint32_t* tcnt, GCtl* ctl, unsigned long long* host_word) {
  __shared__ uint32_t red[GL_BLOCK / 64 + 1];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *next_plan = GPlan{0, 0};  // read by the previous round only
    // progress word for the host: (epoch << 48 | round << 32) | segments in this round
    const uint32_t r = ++ctl->round;
    __hip_atomic_store(host_word, ((unsigned long long)r << 32) | cur.plan->nseg, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  gr_count(el, cur, cur.plan->ntiles, tcnt, red);
}

// Tile of 4096 elements staged in LDS with coalesced loads; thread t owns the run [16t, 16t+16).
__device__ __forceinline__ void gl_stage(const uint64_t* el, uint32_t t0, uint32_t hi, uint64_t* tile) {
  for (uint32_t i = threadIdx.x; i < GL_TILE; i += GL_BLOCK) {
    const uint32_t p = t0 + i;
    tile[i + (i >> 4)] = p < hi ? el[p] : 0;
  }
  __syncthreads();
}

__device__ __forceinline__ void gr_lists(const uint64_t* el, const GLevel& cur, uint32_t ntiles, const uint32_t* tcnt,
                                         uint32_t* A, uint32_t* B, uint64_t* VA, uint64_t* VB, uint32_t* red,
                                         uint32_t* tpre, uint64_t* tile) {
  for (uint32_t tb = blockIdx.x; tb < ntiles; tb += gridDim.x) {
    const uint2 st = cur.tseg[tb];
    const Seg sg = cur.segs[st.x];
    const GLvl L = cur.lv[st.x];
    uint32_t a, e;
    if (!gl_range(sg, L, &a, &e)) continue;  // uniform per block
    const uint32_t t0 = sg.lo + st.y * GL_TILE;
    if (t0 + GL_TILE <= a || t0 >= e) continue;  // tile outside the pass range (protect pass)
    if (threadIdx.x < 64) {  // #left in the earlier tiles of this segment, and in all of them
      const uint32_t first = cur.toff[st.x], nt = gl_ntiles(sg);
      uint32_t pre = 0, all = 0;
      for (uint32_t t = __lane_id(); t < nt; t += 64) {
        const uint32_t v = tcnt[first + t];
        all += v;
        pre += t < st.y ? v : 0u;
      }
      pre = wave_sum(pre);
      all = wave_sum(all);
      if (threadIdx.x == 0) {
        tpre[0] = pre;
        tpre[1] = all;
      }
    }
    gl_stage(el, t0, sg.hi, tile);
    const uint32_t T = tpre[1], bnd = a + T;
    const uint32_t r0 = threadIdx.x * GL_ITEMS;
    uint32_t lbits = 0, rbits = 0;  // bit i: in range / stays left
#pragma unroll
    for (int i = 0; i < GL_ITEMS; i++) {
      const uint32_t p = t0 + r0 + i;
      const bool in = p >= a && p < e;
      rbits |= (in ? 1u : 0u) << i;
      lbits |= ((in && gl_left(KEY<32>(tile[r0 + i + (r0 >> 4)]), L)) ? 1u : 0u) << i;
    }
    uint32_t tot;
    uint32_t lp = tpre[0] + block_excl_scan<GL_BLOCK>((uint32_t)__popc(lbits), red, &tot);  // L(first position)
    uint32_t nml = 0;
#pragma unroll
    for (int i = 0; i < GL_ITEMS; i++) {
      const uint32_t p = t0 + r0 + i;
      if (!((rbits >> i) & 1u)) continue;
      const bool left = (lbits >> i) & 1u;
      if (!left && p < bnd) {  // position and value, so the swap kernel only scatters
        A[sg.lo + (p - a) - lp] = p;
        VA[sg.lo + (p - a) - lp] = tile[r0 + i + (r0 >> 4)];
        nml++;
      } else if (left && p >= bnd) {
        B[sg.lo + T - 1 - lp] = p;
        VB[sg.lo + T - 1 - lp] = tile[r0 + i + (r0 >> 4)];
      }
      lp += left ? 1u : 0u;
    }
    nml = block_sum<GL_BLOCK>(nml, red);
    if (threadIdx.x == 0) {
      if (nml) atomicAdd(&cur.lv[st.x].ng, nml);
      if (t0 <= a && a < t0 + GL_TILE) cur.lv[st.x].bnd = bnd;
    }
  }
}


__global__ __launch_bounds__(GL_BLOCK) void k_gr_lists(const uint64_t* el, GLevel cur, const uint32_t* tcnt,
                                                       uint32_t* A, uint32_t* B, uint64_t* VA, uint64_t* VB) {
  __shared__ uint32_t red[GL_BLOCK / 64 + 1];
  __shared__ uint32_t tpre[2];
  __shared__ uint64_t tile[GL_TILE + GL_TILE / 16];
  gr_lists(el, cur, cur.plan->ntiles, tcnt, A, B, VA, VB, red, tpre, tile);
}

// ---- the O(1) tail of a segment, by one wave after all its swaps are visible ----------------------
// Every element the tail touches is loaded once into a lane-distributed cache (lane i holds the
// value at position pos_i; the lowest lane holding a position owns it), updated in registers and
// stored once: two dependent memory round trips (probe + pivot positions, then the children's
// pivot-of-nine positions) instead of one per step.
struct WCache {
  uint32_t pos;
  uint64_t val;
  bool dirty;
  __device__ __forceinline__ int owner(uint32_t p) const {
    const unsigned long long bal = __ballot(pos == p);
    return bal ? __ffsll((long long)bal) - 1 : 0;
  }
  __device__ __forceinline__ uint64_t get(uint32_t p) const { return __shfl(val, owner(p)); }
  __device__ __forceinline__ void set(uint32_t p, uint64_t v) {
    if ((int)__lane_id() == owner(p)) {
      val = v;
      dirty = true;
    }
  }
  __device__ __forceinline__ void swap(uint32_t i, uint32_t j) {
    const uint64_t a = get(i), b = get(j);
    set(i, b);
    set(j, a);
  }
};

// medianOfThree(data, m1, m0, m2) through the cache
__device__ __forceinline__ void wc_mo3(WCache& W, uint32_t m1, uint32_t m0, uint32_t m2) {
  if (LT<32>(W.get(m1), W.get(m0))) W.swap(m1, m0);
  if (LT<32>(W.get(m2), W.get(m1))) {
    W.swap(m2, m1);
    if (LT<32>(W.get(m1), W.get(m0))) W.swap(m1, m0);
  }
}

// doPivot's pivot-of-nine / medianOfThree positions of [lo, hi) (slot j < 9, 0xFFFFFFFF if unused)
__device__ __forceinline__ uint32_t pivot_pos(uint32_t lo, uint32_t hi, uint32_t j) {
  const uint32_t m = (uint32_t)(((uint64_t)lo + hi) >> 1);
  if (hi - lo > 40) {
    const uint32_t s = (hi - lo) / 8;
    const uint32_t P[9] = {lo, lo + s, lo + 2 * s, m - s, m, m + s, hi - 1 - 2 * s, hi - 1 - s, hi - 1};
    return P[j];
  }
  return j == 0 ? lo : (j == 1 ? m : (j == 2 ? hi - 1 : 0xFFFFFFFFu));
}

__device__ __forceinline__ void wc_pivot(WCache& W, uint32_t lo, uint32_t hi) {
  const uint32_t m = (uint32_t)(((uint64_t)lo + hi) >> 1);
  if (hi - lo > 40) {
    const uint32_t s = (hi - lo) / 8;
    wc_mo3(W, lo, lo + s, lo + 2 * s);
    wc_mo3(W, m, m - s, m + s);
    wc_mo3(W, hi - 1, hi - 1 - s, hi - 1 - 2 * s);
  }
  wc_mo3(W, lo, m, hi - 1);
}

__device__ void gl_tail(uint64_t* el, const Seg& sg, const GLvl& L, GLevel nx, GCtl* ctl, Seg* lds, Seg* heap) {
  const uint32_t lane = __lane_id(), lo = sg.lo, hi = sg.hi;
  // round trip 1: lo, the probe positions (hi-1, bnd, bnd-1, bnd-2, m), the final place of the
  // pivot (b-1 for b in bnd, bnd-1, bnd-2), or the protect pass's b-1
  WCache W{0xFFFFFFFFu, 0, false};
  {
    uint32_t p = 0xFFFFFFFFu;
    if (L.mode == 0) {
      const uint32_t P[7] = {lo, hi - 1, L.bnd, L.bnd - 1, L.bnd - 2, L.bnd - 3, L.m};
      if (lane < 7) p = P[lane];
    } else {
      if (lane == 0) p = lo;
      if (lane == 1) p = L.bnd - 1;
    }
    if (p != 0xFFFFFFFFu && p >= lo && p < hi) {
      W.pos = p;
      W.val = el[p];
    }
  }
  uint32_t b, c;
  bool protect = false;
  if (L.mode == 0) {  // doPivot's dups probe (sort.go), on the cache
    b = L.bnd;
    c = L.bnd;
    protect = hi - c < 5;
    if (!protect && hi - c < (hi - lo) / 4) {
      const uint64_t pv = W.get(lo);
      int dups = 0;
      if (!LT<32>(pv, W.get(hi - 1))) {  // data[hi-1] = pivot
        W.swap(c, hi - 1);
        c++;
        dups++;
      }
      if (!LT<32>(W.get(b - 1), pv)) {  // data[b-1] = pivot
        b--;
        dups++;
      }
      if (!LT<32>(W.get(L.m), pv)) {  // data[m] = pivot
        W.swap(L.m, b - 1);
        b--;
        dups++;
      }
      protect = dups > 1;
    }
  } else {
    b = L.bnd;
    c = L.c;
  }
  Seg ch[2];
  uint32_t nadm = 0, ntl = 0;
  bool adm[2] = {false, false};
  if (protect) {  // the protect pass over [lo+1, b) next round
    uint32_t idx = 0;
    if (lane == 0) idx = atomicAdd(&nx.plan->nseg, 1u);
    idx = __shfl(idx, 0);
    GLvl P = L;
    P.mode = 1;
    P.b = b;
    P.c = c;
    P.bnd = lo + 1;  // the boundary if the range [lo+1, b) is empty
    P.ng = 0;
    if (W.dirty) el[W.pos] = W.val;
    gl_enter(sg, P, idx, nx);
    return;
  }
  W.swap(lo, b - 1);  // pivot into its final place
  const int32_t dep = sg.depth - 1;
  ch[0] = Seg{lo, b - 1, dep, 0};
  ch[1] = Seg{c, hi, dep, 0};
  for (int k = 0; k < 2; k++) {
    const uint32_t len = ch[k].hi - ch[k].lo;
    if (len <= 1) continue;
    if (len <= g_t_child) {
      if (lane == 0) lds[atomicAdd(&ctl->nlds, 1u)] = ch[k];
    } else if (dep == 0) {
      if (lane == 0) heap[atomicAdd(&ctl->nheap, 1u)] = ch[k];
    } else {
      adm[k] = true;
      nadm++;
      ntl += gl_ntiles(ch[k]);
    }
  }
  if (nadm) {
    // round trip 2: the admitted children's pivot positions (lanes 8.. and 24..), beside the slot
    // reservations; positions already cached take the cached value
    uint32_t p = 0xFFFFFFFFu;
    if (lane >= 8 && lane < 17 && adm[0]) p = pivot_pos(ch[0].lo, ch[0].hi, lane - 8);
    if (lane >= 24 && lane < 33 && adm[1]) p = pivot_pos(ch[1].lo, ch[1].hi, lane - 24);
    const unsigned long long have = __ballot(W.pos != 0xFFFFFFFFu);
    int src = -1;
    for (unsigned long long h = have; h; h &= h - 1) {  // cached lanes, lowest first
      const int l = __ffsll((long long)h) - 1;
      if (src < 0 && p != 0xFFFFFFFFu && __shfl(W.pos, l) == p) src = l;
      else (void)__shfl(W.pos, l);
    }
    uint32_t r = 0;
    if (lane == 0) r = atomicAdd(&nx.plan->nseg, nadm);
    if (lane == 1) r = atomicAdd(&nx.plan->ntiles, ntl);
    const uint64_t cached = __shfl(W.val, src < 0 ? (int)lane : src);
    if (p != 0xFFFFFFFFu) {
      W.pos = p;
      W.val = src >= 0 ? cached : el[p];
    }
    const uint32_t idx0 = __shfl(r, 0), t00 = __shfl(r, 1);
    uint32_t idx = idx0, t0 = t00;
    for (int k = 0; k < 2; k++) {
      if (!adm[k]) continue;
      wc_pivot(W, ch[k].lo, ch[k].hi);
      const uint32_t nt = gl_ntiles(ch[k]);
      for (uint32_t t = lane; t < nt; t += 64) nx.tseg[t0 + t] = make_uint2(idx, t);
      const uint64_t piv = W.get(ch[k].lo);
      if (lane == 0) {
        GLvl C{};
        C.m = (uint32_t)(((uint64_t)ch[k].lo + ch[k].hi) >> 1);
        C.pl = KEY<32>(piv);
        nx.segs[idx] = ch[k];
        nx.toff[idx] = t0;
        nx.done[idx] = 0;
        nx.lv[idx] = C;
      }
      idx++;
      t0 += nt;
    }
  }
  if (W.dirty) el[W.pos] = W.val;
}

// tile t of a segment swaps the pairs k in [t*TILE/2, (t+1)*TILE/2) (ng <= len/2 <= ntile*TILE/2);
// the last tile of the segment to arrive runs its tail. The lists carry the values, so a swap is two
// scattered stores. WT: write-through stores (agent scope, sc1) need no L2 write-back before the
// arrival; otherwise plain stores and one release fence per workgroup.
template <bool WT>
__device__ __forceinline__ void gr_swap(uint64_t* el, const GLevel& cur, uint32_t ntiles, const GLevel& nx,
                                        const uint32_t* A, const uint32_t* B, const uint64_t* VA, const uint64_t* VB,
                                        GCtl* ctl, Seg* lds, Seg* heap, uint32_t* last) {
  for (uint32_t tb = blockIdx.x; tb < ntiles; tb += gridDim.x) {
    const uint2 st = cur.tseg[tb];
    const Seg sg = cur.segs[st.x];
    const uint32_t ng = cur.lv[st.x].ng;
    const uint32_t k0 = st.y * (GL_TILE / 2), k1 = min(ng, k0 + GL_TILE / 2);
    for (uint32_t k = k0 + threadIdx.x; k < k1; k += GL_BLOCK) {
      const uint32_t i = A[sg.lo + k], j = B[sg.lo + k];
      const uint64_t x = VA[sg.lo + k], y = VB[sg.lo + k];
      if (WT) {
        __hip_atomic_store((gu64*)&el[i], y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((gu64*)&el[j], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        el[i] = y;
        el[j] = x;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    if (threadIdx.x == 0) {
      if (!WT) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      const uint32_t old = __hip_atomic_fetch_add(&cur.done[st.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last = old + 1 == gl_ntiles(sg);
    }
    __syncthreads();
    if (*last && threadIdx.x < 64) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const GLvl L = cur.lv[st.x];
      gl_tail(el, sg, L, nx, ctl, lds, heap);
    }
    __syncthreads();
  }
}


template <bool WT>
__global__ __launch_bounds__(GL_BLOCK) void k_gr_swap(uint64_t* el, GLevel cur, GLevel nx, const uint32_t* A,
                                                      const uint32_t* B, const uint64_t* VA, const uint64_t* VB,
                                                      GCtl* ctl, Seg* lds, Seg* heap) {
  __shared__ uint32_t last;
  gr_swap<WT>(el, cur, cur.plan->ntiles, nx, A, B, VA, VB, ctl, lds, heap, &last);
}

// ---- persistent form: every round in ONE launch ------------------------------------------------
// The three phases of a round are separated by grid barriers instead of kernel boundaries. The grid
// never exceeds what the device holds at once (host: occupancy x CUs), so every workgroup is resident
// and the barrier cannot wait on an unscheduled one. A barrier is the swap kernel's own publication
// pattern: each wave drains its stores, one agent-scope release per workgroup, an arrival on one
// agent-scope counter, then an agent-scope acquire. Every workgroup leaves the loop in the same round:
// the next round's segment count is final before the barrier that ends a round, or at maxr.
__device__ __forceinline__ void gr_grid_barrier(uint32_t* bar, uint32_t target) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <bool WT>
__global__ __launch_bounds__(GL_BLOCK) void k_gr_persist(uint64_t* el, GLevel l0, GLevel l1, uint32_t* tcnt,
                                                         uint32_t* A, uint32_t* B, uint64_t* VA, uint64_t* VB,
                                                         GCtl* ctl, Seg* lds, Seg* heap, uint32_t* bar,
                                                         uint32_t maxr) {
  __shared__ uint32_t red[GL_BLOCK / 64 + 1];
  __shared__ uint32_t tpre[2];
  __shared__ uint64_t tile[GL_TILE + GL_TILE / 16];
  __shared__ uint32_t last;
  __shared__ uint32_t plan[2];
  uint32_t target = 0;
  for (uint32_t r = 0; r < maxr; r++) {
    const GLevel cur = (r & 1) ? l1 : l0, nx = (r & 1) ? l0 : l1;
    if (threadIdx.x == 0) {
      plan[0] = __hip_atomic_fetch_add(&cur.plan->nseg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      plan[1] = __hip_atomic_fetch_add(&cur.plan->ntiles, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const uint32_t nseg = plan[0], ntiles = plan[1];
    if (nseg == 0) break;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // nx is read by nobody before the swap phase's tails
      __hip_atomic_store(&nx.plan->nseg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&nx.plan->ntiles, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    gr_count(el, cur, ntiles, tcnt, red);
    gr_grid_barrier(bar, target += gridDim.x);
    gr_lists(el, cur, ntiles, tcnt, A, B, VA, VB, red, tpre, tile);
    gr_grid_barrier(bar, target += gridDim.x);
    gr_swap<WT>(el, cur, ntiles, nx, A, B, VA, VB, ctl, lds, heap, &last);
    gr_grid_barrier(bar, target += gridDim.x);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl->round = 0x10000u | (target / gridDim.x / 3);  // rounds run
}

__global__ void k_gs_heap(uint64_t* el, const Seg* segs, const uint32_t* nsegs) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < *nsegs; i += gridDim.x * blockDim.x)
    heap_sort<32>(el, segs[i].lo, segs[i].hi);
}

__global__ void k_gs_init(uint32_t* perm, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    perm[i] = (uint32_t)i;
}

// dynamic LDS segments (children of global levels): one pack per segment
__global__ void k_dyn_packs(const Seg* segs, const uint32_t* n, Pack* packs) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < *n; i += gridDim.x * blockDim.x)
    packs[i] = Pack{segs[i].lo, segs[i].hi, i, i + 1};
}

// ---- host driver -------------------------------------------------------------------------------------
template <int SH, class E, int LEAF>
static void launch_ls_leaf(const uint64_t* el, uint32_t* perm, const Pack* packs, uint32_t npacks_host,
                           const uint32_t* npacks_dev, unsigned grid, const Seg* segs, uint32_t* bounce_cnt,
                           Pack* bounce, hipStream_t s) {
  static std::atomic<bool> attr[64];  // per device
  int dev = 0;
  SYZ_HIP(hipGetDevice(&dev));
  if (!attr[dev & 63].load()) {
    SYZ_HIP(hipFuncSetAttribute((const void*)k_ls_sort<SH, E, LEAF>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sizeof(LsLds<E, LEAF>)));
    attr[dev & 63] = true;
  }
  if (grid == 0) return;
  k_ls_sort<SH, E, LEAF><<<grid, LS_BLOCK, sizeof(LsLds<E, LEAF>), s>>>(el, perm, packs, npacks_host, npacks_dev,
                                                                        segs, bounce_cnt, bounce);
  SYZ_LAUNCHED();
}

// the process's leaf form (syzgpu_set_go_sort_leaf), read once per sort
static std::atomic<int> g_go_leaf{GO_LEAF12};
int gosort_leaf() { return g_go_leaf.load(); }

template <int SH, class E>
static void launch_ls(const uint64_t* el, uint32_t* perm, const Pack* packs, uint32_t npacks_host,
                      const uint32_t* npacks_dev, unsigned grid, const Seg* segs, uint32_t* bounce_cnt, Pack* bounce,
                      hipStream_t s, int leaf) {
  if (leaf == GO_LEAF7)
    launch_ls_leaf<SH, E, GO_LEAF7>(el, perm, packs, npacks_host, npacks_dev, grid, segs, bounce_cnt, bounce, s);
  else
    launch_ls_leaf<SH, E, GO_LEAF12>(el, perm, packs, npacks_host, npacks_dev, grid, segs, bounce_cnt, bounce, s);
}

// The static part of a sort over fixed call-group boundaries: which groups start the global levels,
// and how the small ones are packed for the LDS sorter. Built once per corpus layout.
GosortPlan::~GosortPlan() {
  if (small) (void)hipFree(small);
  if (packs) (void)hipFree(packs);
  if (big) (void)hipFree(big);
}

void gosort_plan(GosortPlan& P, const std::vector<uint64_t>& hstart, uint32_t ngroups, hipStream_t s) {
  // a plan may be re-made for a new layout (a corpus that grew since the last minimize, the incremental
  // corpus index): its device arrays are grow-only (a hipFree would wait for the whole device, the
  // transpose included), overwritten on s after their last users there; the learned round count stays
  // as a hint
  P.big_max = 0;
  std::vector<Seg> big, small;
  std::vector<Pack> packs;
  gosort_segments(hstart, ngroups, small, packs, big);
  P.n = hstart[ngroups];
  P.nsmall = (uint32_t)small.size();
  P.npacks = (uint32_t)packs.size();
  P.nbig = (uint32_t)big.size();
  P.big_total = 0;
  for (const Seg& sg : big) {
    P.big_total += sg.hi - sg.lo;
    P.big_max = std::max<uint64_t>(P.big_max, sg.hi - sg.lo);
  }
  auto grow = [](auto*& p, size_t& cap, size_t need) {
    if (p && cap >= need) return;
    if (p) SYZ_HIP(hipFree(p));
    p = nullptr;
    cap = need + need / 4 + 16;
    SYZ_HIP(hipMalloc(&p, cap * sizeof(*p)));
  };
  grow(P.small, P.cap_small, small.size() + 1);
  grow(P.packs, P.cap_packs, packs.size() + 1);
  grow(P.big, P.cap_big, big.size() + 1);
  // on the caller's stream, never the legacy one: another thread's graph capture may be running; from
  // the lane's plan staging (pinned), so the host goes on without waiting for the copies: the staging is
  // rewritten only once the previous plan's copies are done (ev_plan)
  Context& c = ctx();
  if (!c.ev_plan) SYZ_HIP(hipEventCreateWithFlags(&c.ev_plan, hipEventDisableTiming));
  else SYZ_HIP(hipEventSynchronize(c.ev_plan));
  const size_t bs = small.size() * sizeof(Seg), bp = packs.size() * sizeof(Pack), bb = big.size() * sizeof(Seg);
  uint8_t* h = c.pinned_plan.get<uint8_t>(bs + bp + bb + 16);
  std::memcpy(h, small.data(), bs);
  std::memcpy(h + bs, packs.data(), bp);
  std::memcpy(h + bs + bp, big.data(), bb);
  if (bs) SYZ_HIP(hipMemcpyAsync(P.small, h, bs, hipMemcpyHostToDevice, s));
  if (bp) SYZ_HIP(hipMemcpyAsync(P.packs, h + bs, bp, hipMemcpyHostToDevice, s));
  if (bb) SYZ_HIP(hipMemcpyAsync(P.big, h + bs + bp, bb, hipMemcpyHostToDevice, s));
  SYZ_HIP(hipEventRecord(c.ev_plan, s));
}

void gosort_groups(uint64_t* el, uint32_t* perm, size_t n, const std::vector<uint64_t>& hstart, uint32_t ngroups,
                   hipStream_t s) {
  GosortPlan P;
  gosort_plan(P, hstart, ngroups, s);
  gosort_run(el, perm, n, P, s);
  SYZ_HIP(hipStreamSynchronize(s));  // P's device arrays are freed on return
}

// Sorts every call group's range (as planned in P) with Go's sort.Sort semantics. Result: the element
// at sorted position r is el[perm[r]]. Enqueues everything on s; the host only waits for the
// level-count events of the global levels.
void gosort_run(uint64_t* el, uint32_t* perm, size_t n, const GosortPlan& P, hipStream_t s,
                const std::function<void(hipStream_t)>& small_done, const std::function<void(hipStream_t)>& big_done) {
  Context& c = ctx();
  Scratch& sc = c.scratch;
  if (n >= 0xFFFFFFF0ull || n != P.n) fail(SYZGPU_EINVAL, "gosort: plan does not match the elements");
  const int leaf = gosort_leaf();
  const uint32_t tch = t_child_host();
  const size_t maxseg = n / (tch / 2) + (size_t)P.nbig * 2 + 16;
  const size_t maxlds = n / 2 + 16;
  const Seg* d_small = P.small;
  const Pack* d_packs = P.packs;
  Seg* dlds = sc.get<Seg>("gs_lds", maxlds);
  Pack* dpacks = sc.get<Pack>("gs_dpacks", maxlds);
  Seg* heap = sc.get<Seg>("gs_heap", maxseg);
  Pack* bounceS = sc.get<Pack>("gs_bounceS", (size_t)P.npacks + 1);
  Pack* bounceD = sc.get<Pack>("gs_bounceD", maxlds);
  uint32_t* A = sc.get<uint32_t>("gs_A", n + 1);
  uint32_t* B = sc.get<uint32_t>("gs_B", n + 1);
  uint64_t* VA = sc.get<uint64_t>("gs_VA", n + 1);
  uint64_t* VB = sc.get<uint64_t>("gs_VB", n + 1);
  // ctl[0]: next-level count (reset by each plan) and the accumulated LDS / heap children;
  // ctl[2]: bounce counters of the static (nnext) and dynamic (nlds) LDS launches; ctl[3]: scratch
  GCtl* ctl = sc.get<GCtl>("gs_ctl", 4);
  SYZ_HIP(hipMemsetAsync(ctl, 0, 4 * sizeof(GCtl), s));
  {
    ProfScope ps("gosort_init", s, (uint64_t)n * 4);
    k_gs_init<<<grid_for(n, 256, 4096), 256, 0, s>>>(perm, n);
    SYZ_LAUNCHED();
  }
  // the small call groups (packed) are independent of the big ones: sort them on the side stream
  // while the main stream runs the global levels
  // (the big groups' rounds on a stream of the greatest priority measured no faster beside the
  // transpose: r04_t1, 2.988 vs 2.983 ms)
  ensure_side(c);
  const bool fork = P.npacks && P.nbig && !dev_env("SYZGPU_GS_NOFORK");
  hipStream_t ss = fork ? c.side : s;  // the small groups' stream
  hipStream_t bs = s;                  // the big groups'
  if (fork) {
    SYZ_HIP(hipEventRecord(c.ev_fork, s));
    SYZ_HIP(hipStreamWaitEvent(c.side, c.ev_fork, 0));
  }
  if (P.npacks) {
    {
      ProfScope ps("gosort_lds_small", ss, (uint64_t)n * 12);
      launch_ls<LS_SH, uint32_t>(el, perm, d_packs, P.npacks, nullptr, std::min<uint32_t>(P.npacks, 65535), d_small,
                              &ctl[2].nnext, bounceS, ss, leaf);
    }
    // packs with a length that does not fit the u32 element (>= 2^19 PCs) were bounced: the u64
    // instantiation sorts them (a launch over an empty bounce list returns at once)
    // (skipped when no cover can bounce: even an empty launch of its 64 KB-LDS workgroups waits for whole
    // CUs while the transpose runs beside the sort)
    if (P.may_bounce)
      launch_ls<32, uint64_t>(el, perm, bounceS, 0, &ctl[2].nnext, 64, d_small, &ctl[3].nnext, bounceS, ss, leaf);
  }
  if (small_done) small_done(ss);
  if (fork) SYZ_HIP(hipEventRecord(c.ev_join, ss));
  // global levels: the host issues level after level without waiting; each level's segment count is
  // copied back asynchronously and the host stops issuing once a finished level reports zero
  // (levels issued after the last real one find nseg == 0 and return at once).
  if (P.nbig) {
    const uint32_t nbig = P.nbig;
    const size_t max_tiles = n / GL_TILE + maxseg + 1;
    uint32_t* tcnt = sc.get<uint32_t>("gs_tcnt", max_tiles);
    GLevel lvl[2];
    for (int p = 0; p < 2; p++) {
      const std::string k = std::to_string(p);
      lvl[p].segs = sc.get<Seg>("gs_seg" + k, maxseg);
      lvl[p].lv = sc.get<GLvl>("gs_lv" + k, maxseg);
      lvl[p].toff = sc.get<uint32_t>("gs_toff" + k, maxseg);
      lvl[p].done = sc.get<uint32_t>("gs_done" + k, maxseg);
      lvl[p].tseg = sc.get<uint2>("gs_tseg" + k, max_tiles);
      lvl[p].plan = sc.get<GPlan>("gs_plan" + k, 1);
    }
    if (!c.gr_host) {
      SYZ_HIP(hipHostMalloc((void**)&c.gr_host, 64, hipHostMallocMapped | hipHostMallocCoherent));
      SYZ_HIP(hipHostGetDevicePointer((void**)&c.gr_dev, c.gr_host, 0));
      *c.gr_host = 0;
    }
    // grids sized to what the big groups can ever need (their elements only shrink round by round):
    // idle workgroups of a grid-stride kernel still cost dispatch time on every launch
    const size_t segs_max = P.big_total / tch + P.nbig + 1;
    const unsigned tgrid = (unsigned)std::min<size_t>(P.big_total / GL_TILE + segs_max, 2048);
    ProfScope ps("gosort_level", bs, 0);
    const uint32_t epoch = (++c.gr_epoch & 0x7FFFu) | 0x8000u;
    SYZ_HIP(hipMemsetAsync(lvl[0].plan, 0, sizeof(GPlan), bs));
    k_gl_init<<<std::min<uint32_t>(nbig, 1024), 64, 0, bs>>>(el, P.big, nbig, lvl[0], ctl, epoch);
    SYZ_LAUNCHED();
    // Default: the rounds as captured graphs of 3 launches each. SYZGPU_GR_PERSIST=1: all rounds in one
    // persistent launch with grid barriers (k_gr_persist). Measured slower at config 4 (global rounds
    // 0.74 ms at 64-256 workgroups vs 0.45 ms as graphs): a barrier's per-workgroup L2 write-back and
    // invalidate costs more than the launch gap it replaces.
    const char* pe = getenv("SYZGPU_GR_PERSIST");
    const bool wt = !dev_env("SYZGPU_GR_FENCE");  // A/B switch: write-through swaps vs release fence
    if (pe && !strcmp(pe, "1")) {
      if (!c.gr_resident) {  // workgroups the device holds at once: the persistent grid never exceeds it
        int per_cu = 0, cus = 0;
        SYZ_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_gr_persist<true>, GL_BLOCK, 0));
        int per_cu2 = 0;
        SYZ_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu2, k_gr_persist<false>, GL_BLOCK, 0));
        SYZ_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device));
        c.gr_resident = (uint32_t)std::max(1, std::min(per_cu, per_cu2) * cus);
      }
      // few workgroups: every barrier costs each of them an L2 write-back and invalidate
      const char* pg = getenv("SYZGPU_GR_PGRID");
      const unsigned want = pg ? (unsigned)std::max(1, atoi(pg)) : 256u;
      const unsigned pgrid = std::min<unsigned>(std::min<unsigned>(tgrid, want), c.gr_resident);
      uint32_t* bar = sc.get<uint32_t>("gs_bar", 1);
      SYZ_HIP(hipMemsetAsync(bar, 0, 4, bs));
      constexpr uint32_t MAXR = 512;
      if (wt)
        k_gr_persist<true><<<pgrid, GL_BLOCK, 0, bs>>>(el, lvl[0], lvl[1], tcnt, A, B, VA, VB, ctl, dlds, heap, bar, MAXR);
      else
        k_gr_persist<false><<<pgrid, GL_BLOCK, 0, bs>>>(el, lvl[0], lvl[1], tcnt, A, B, VA, VB, ctl, dlds, heap, bar, MAXR);
      SYZ_LAUNCHED();
      if (dev_env("SYZGPU_GS_DEBUG")) {
        GCtl h;
        SYZ_HIP(hipMemcpyAsync(&h, ctl, sizeof(h), hipMemcpyDeviceToHost, bs));
        SYZ_HIP(hipStreamSynchronize(bs));
        fprintf(stderr, "gosort: persistent grid %u, %u rounds\n", pgrid, h.round & 0xFFFFu);
      }
    } else {
      // one round = 3 dependent kernels with fixed arguments per buffer parity; RPG rounds (parity 0,
      // 1, 0, 1) are captured once into a HIP graph and replayed
      constexpr uint32_t RPG = 4;
      auto enqueue_round = [&](hipStream_t q, int parity) {
        const GLevel cur = lvl[parity], nx = lvl[parity ^ 1];
        k_gr_count<<<tgrid, GL_BLOCK, 0, q>>>(el, cur, nx.plan, tcnt, ctl, c.gr_dev);
        SYZ_LAUNCHED();
        k_gr_lists<<<tgrid, GL_BLOCK, 0, q>>>(el, cur, tcnt, A, B, VA, VB);
        SYZ_LAUNCHED();
        if (wt)
          k_gr_swap<true><<<tgrid, GL_BLOCK, 0, q>>>(el, cur, nx, A, B, VA, VB, ctl, dlds, heap);
        else
          k_gr_swap<false><<<tgrid, GL_BLOCK, 0, q>>>(el, cur, nx, A, B, VA, VB, ctl, dlds, heap);
        SYZ_LAUNCHED();
      };
      const std::vector<const void*> key = {el,          tcnt,        A,           B,           ctl,         dlds,
                                            heap,        lvl[0].segs, lvl[0].lv,   lvl[0].toff, lvl[0].done, lvl[0].tseg,
                                            lvl[0].plan, lvl[1].segs, lvl[1].lv,   lvl[1].toff, lvl[1].done, lvl[1].tseg,
                                            lvl[1].plan, c.gr_dev,    (const void*)(uintptr_t)tgrid,
                                            VA,          VB,          (const void*)(uintptr_t)wt};
      if (c.gl_key != key) {
        for (auto& row : c.gl_exec)
          for (auto& g : row) {
            if (g) SYZ_HIP(hipGraphExecDestroy(g));
            g = nullptr;
          }
        c.gl_key = key;
      }
      // graph of k rounds starting at buffer parity p, captured on first use
      auto graph = [&](int p, uint32_t k) -> hipGraphExec_t {
        hipGraphExec_t& ex = c.gl_exec[p][k - 1];
        if (!ex) {
          if (!c.cap) SYZ_HIP(hipStreamCreateWithFlags(&c.cap, hipStreamNonBlocking));
          hipGraph_t g;
          SYZ_HIP(hipStreamBeginCapture(c.cap, hipStreamCaptureModeThreadLocal));
          for (uint32_t r = 0; r < k; r++) enqueue_round(c.cap, (int)((p + r) & 1));
          SYZ_HIP(hipStreamEndCapture(c.cap, &g));
          SYZ_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
          SYZ_HIP(hipGraphDestroy(g));
        }
        return ex;
      };
      // The host issues rounds without waiting for them. The first count kernel of every round writes
      // (epoch, round, segments) into host-mapped memory; the host stops once a round of this call
      // reports zero segments (rounds issued past it find nothing and return at once). With a hint
      // (the rounds the previous run of this plan needed), exactly hint + 1 rounds are issued up front
      // and the last one reports zero; otherwise rounds go out RPG at a time, at most AHEAD beyond the
      // last one seen running.
      constexpr uint32_t MAXR = 512, AHEAD = RPG + 2;
      volatile unsigned long long* hw = c.gr_host;
      uint32_t issued = 0, seen = 0;
      auto launch = [&](uint32_t k) {
        if (issued + k > MAXR) fail(SYZGPU_EINTERNAL, "gosort: round limit");
        SYZ_HIP(hipGraphLaunch(graph((int)(issued & 1), k), bs));
        issued += k;
      };
      bool done = false;
      uint32_t last_rounds = 0;
      auto poll = [&]() -> bool {  // true: a round of this call reported zero segments
        const unsigned long long w = *hw;
        if ((uint32_t)(w >> 48) != epoch) return false;
        const uint32_t r = (uint32_t)(w >> 32) & 0xFFFFu, ns = (uint32_t)w;
        if (r > seen) seen = r;
        if (ns == 0) {
          last_rounds = r - 1;
          return true;
        }
        return false;
      };
      const bool hinted = P.rounds_hint > 0;
      if (hinted)
        while (issued < P.rounds_hint + 1) launch(std::min<uint32_t>(RPG, P.rounds_hint + 1 - issued));
      else
        launch(RPG);
      while (!(done = poll())) {
        if (!hinted && issued - seen < AHEAD) {
          launch(RPG);
          continue;
        }
        if (hipStreamQuery(bs) == hipSuccess) {  // everything issued has run
          if ((done = poll())) break;
          if (seen < issued) fail(SYZGPU_EINTERNAL, "gosort: no progress word from the rounds");
          launch(RPG);
          continue;
        }
        __builtin_ia32_pause();
      }
      P.rounds_hint = last_rounds;
      if (dev_env("SYZGPU_GS_DEBUG")) {
        SYZ_HIP(hipStreamSynchronize(bs));
        fprintf(stderr, "gosort: %u rounds issued, %u with segments\n", issued, last_rounds);
      }
    }
    // children that reached the LDS size and depth-exhausted big ones: counts stay on the device
    k_gs_heap<<<64, 64, 0, bs>>>(el, heap, &ctl[0].nheap);
    SYZ_LAUNCHED();
    // the LDS-sized children of all levels, one workgroup each ([0, nlds) via &ctl[0].nnext == 0);
    // running them per level beside the levels was measured slower: they take the CUs the
    // latency-bound level kernels need
    {
      ProfScope ps2("gosort_lds", bs, (uint64_t)n * 12);
      launch_ls<LS_SH, uint32_t>(el, perm, nullptr, 0, &ctl[0].nnext, 1024, dlds, &ctl[2].nlds, bounceD, bs, leaf);
    }
    if (P.may_bounce)
      launch_ls<32, uint64_t>(el, perm, bounceD, 0, &ctl[2].nlds, 64, dlds, &ctl[3].nlds, bounceD, bs, leaf);
  }
  if (big_done) big_done(bs);
  if (fork) SYZ_HIP(hipStreamWaitEvent(s, c.ev_join, 0));
  (void)dpacks;
}

// (no device work and no lane: callable before syzgpu_init)
extern "C" int syzgpu_set_go_sort_leaf(int leaf) {
  if (leaf != GO_LEAF12 && leaf != GO_LEAF7) return SYZGPU_EINVAL;
  g_go_leaf.store(leaf);
  return SYZGPU_OK;
}
extern "C" int syzgpu_go_sort_leaf(void) { return g_go_leaf.load(); }

#ifdef SYZ_GS_STATS
extern "C" int syzgpu_debug_gosort_stats(unsigned long long* out, int reset) {
  hipDeviceSynchronize();
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gs_stats), sizeof(unsigned long long) * 24);
  if (reset) {
    unsigned long long z[24] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_gs_stats), z, sizeof(z));
  }
  return 0;
}
#endif

}  // namespace syz

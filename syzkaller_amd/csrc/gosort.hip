// The permutation Go's sort.Sort (Go 1.7 quickSort) produces for cover.Minimize's input array
// (cover/cover.go:106-113, minInputArray.Less = len(a[i].cov) > len(a[j].cov), :140-143),
// computed on the GPU for every call group at once.
//
// sort.Sort is unstable: among equal lengths the order depends on the exact sequence of swaps, and
// that order decides which inputs Minimize keeps. The simulation therefore performs
// the same swaps as the sequential algorithm, but each doPivot's O(n) loops run in parallel:
//   * the Hoare loop of doPivot pairs the k-th element > pivot from the left with the k-th element
//     <= pivot from the right, for every k below the number of misplaced elements, so both lists
//     are built with ordered compaction (ballot/prefix scans) and swapped pairwise;
//   * the "protect" duplicate pass is the same pairing with (== pivot) vs (< pivot);
//   * the O(1) parts (ninther / medianOfThree, the dups probe, the final pivot swap) run on one lane.
// Disjoint subranges are independent, so all recursion nodes of one depth run concurrently:
//   level kernel   one 1024-thread workgroup per segment larger than FIN_MAX (global memory),
//   finisher       one wave per segment <= FIN_MAX, loaded into LDS, recursed to completion there
//                  (including the gap-6 shell pass + insertion sort and the heapSort fallback),
//   heap kernel    the depth-exhausted heapSort fallback for large segments (never seen in practice).
// Elements are packed as (len << 32) | global member index; Less compares the high word only.
#include "pipeline.hpp"

namespace syz {

__device__ __forceinline__ uint32_t LEN(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ bool LESS(uint64_t x, uint64_t y) { return LEN(x) > LEN(y); }

template <class P>
__device__ __forceinline__ void swp(P d, uint32_t i, uint32_t j) {
  uint64_t t = d[i];
  d[i] = d[j];
  d[j] = t;
}

// medianOfThree(data, m1, m0, m2): moves the median of data[m0], data[m1], data[m2] into data[m1].
template <class P>
__device__ void mo3(P d, uint32_t m1, uint32_t m0, uint32_t m2) {
  if (LESS(d[m1], d[m0])) swp(d, m1, m0);
  if (LESS(d[m2], d[m1])) {
    swp(d, m2, m1);
    if (LESS(d[m1], d[m0])) swp(d, m1, m0);
  }
}

// Pivot selection of doPivot (ninther for hi-lo > 40, then medianOfThree(lo, m, hi-1)). Returns m.
template <class P>
__device__ uint32_t choose_pivot(P d, uint32_t lo, uint32_t hi) {
  const uint32_t m = (uint32_t)(((uint64_t)lo + hi) >> 1);
  if (hi - lo > 40) {
    const uint32_t s = (hi - lo) / 8;
    mo3(d, lo, lo + s, lo + 2 * s);
    mo3(d, m, m - s, m + s);
    mo3(d, hi - 1, hi - 1 - s, hi - 1 - 2 * s);
  }
  mo3(d, lo, m, hi - 1);
  return m;
}

// The dups probe of doPivot after the main partition (b == c == bnd on entry).
template <class P>
__device__ bool dups_probe(P d, uint32_t lo, uint32_t hi, uint32_t m, uint32_t* b, uint32_t* c) {
  bool protect = hi - *c < 5;
  if (!protect && hi - *c < (hi - lo) / 4) {
    int dups = 0;
    if (!LESS(d[lo], d[hi - 1])) {  // data[hi-1] = pivot
      swp(d, *c, hi - 1);
      (*c)++;
      dups++;
    }
    if (!LESS(d[*b - 1], d[lo])) {  // data[b-1] = pivot
      (*b)--;
      dups++;
    }
    if (!LESS(d[m], d[lo])) {  // data[m] = pivot
      swp(d, m, *b - 1);
      (*b)--;
      dups++;
    }
    protect = dups > 1;
  }
  return protect;
}

template <class P>
__device__ void sift_down(P d, uint32_t lo, uint32_t hi, uint32_t first) {
  uint32_t root = lo;
  for (;;) {
    uint32_t child = 2 * root + 1;
    if (child >= hi) break;
    if (child + 1 < hi && LESS(d[first + child], d[first + child + 1])) child++;
    if (!LESS(d[first + root], d[first + child])) return;
    swp(d, first + root, first + child);
    root = child;
  }
}

template <class P>
__device__ void heap_sort(P d, uint32_t a, uint32_t b) {
  const uint32_t first = a, hi = b - a;
  for (int64_t i = ((int64_t)hi - 1) / 2; i >= 0; i--) sift_down(d, (uint32_t)i, hi, first);
  for (int64_t i = (int64_t)hi - 1; i >= 0; i--) {
    swp(d, first, first + (uint32_t)i);
    sift_down(d, 0, (uint32_t)i, first);
  }
}

template <class P>
__device__ void shell_insertion(P d, uint32_t a, uint32_t b) {
  for (uint32_t i = a + 6; i < b; i++)
    if (LESS(d[i], d[i - 6])) swp(d, i, i - 6);
  for (uint32_t i = a + 1; i < b; i++)
    for (uint32_t j = i; j > a && LESS(d[j], d[j - 1]); j--) swp(d, j, j - 1);
}

__device__ __forceinline__ void route(uint32_t a, uint32_t b, int32_t depth, uint32_t fin_max, Seg* big, Seg* fin,
                                      Seg* heap, uint32_t* cnt) {
  if (b - a <= 1) return;
  Seg s{a, b, depth, 0};
  if (b - a <= fin_max) {
    fin[atomicAdd(&cnt[1], 1u)] = s;
  } else if (depth == 0) {
    heap[atomicAdd(&cnt[2], 1u)] = s;
  } else {
    big[atomicAdd(&cnt[0], 1u)] = s;
  }
}

// ---- level kernel: one workgroup per large segment --------------------------------------------
constexpr int QB = 1024;

// Ordered compaction of positions p in [beg, end) with pred(p) into out[0..): returns count.
template <class Pred>
__device__ uint32_t block_collect(uint32_t beg, uint32_t end, Pred pred, uint32_t* out, uint32_t* red) {
  uint32_t k = 0;
  for (uint32_t base = beg; base < end; base += QB) {
    const uint32_t p = base + threadIdx.x;
    const uint32_t f = (p < end && pred(p)) ? 1u : 0u;
    uint32_t tot;
    const uint32_t r = block_excl_scan<QB>(f, red, &tot);
    if (f) out[k + r] = p;
    k += tot;
  }
  return k;
}

__global__ __launch_bounds__(QB) void k_qs_level(uint64_t* __restrict__ el, uint32_t* __restrict__ tmpA,
                                                 uint32_t* __restrict__ tmpB, const Seg* segs, uint32_t nsegs,
                                                 Seg* big, Seg* fin, Seg* heap, uint32_t* cnt, uint32_t fin_max) {
  __shared__ uint32_t red[QB / 64 + 1];
  __shared__ uint32_t sh[8];
  for (uint32_t si = blockIdx.x; si < nsegs; si += gridDim.x) {
    const Seg sg = segs[si];
    const uint32_t lo = sg.lo, hi = sg.hi;
    if (threadIdx.x == 0) {
      sh[1] = choose_pivot(el, lo, hi);
      sh[0] = LEN(el[lo]);
    }
    __syncthreads();
    const uint32_t plen = sh[0], m = sh[1];
    // main partition region [lo+1, hi-1): L = !Less(pivot, x) = len >= plen goes left
    // (Go's initial a-scan is not needed: every element left of it is < pivot in sort order, so it
    //  is never paired and the protect pass below may start at lo+1.)
    uint32_t lc = 0;
    for (uint32_t p = lo + 1 + threadIdx.x; p < hi - 1; p += QB) lc += LEN(el[p]) >= plen;
    const uint32_t Lcnt = block_sum<QB>(lc, red);
    uint32_t bnd = lo + 1 + Lcnt;
    uint32_t* A = tmpA + lo;
    uint32_t* B = tmpB + lo;
    const uint32_t nG = block_collect(lo + 1, bnd, [&](uint32_t p) { return LEN(el[p]) < plen; }, A, red);
    const uint32_t nL = block_collect(bnd, hi - 1, [&](uint32_t p) { return LEN(el[p]) >= plen; }, B, red);
    __syncthreads();
    (void)nL;  // == nG
    for (uint32_t k = threadIdx.x; k < nG; k += QB) swp(el, A[k], B[nG - 1 - k]);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t b = bnd, c = bnd;
      const bool protect = dups_probe(el, lo, hi, m, &b, &c);
      sh[2] = b;
      sh[3] = c;
      sh[4] = protect;
    }
    __syncthreads();
    uint32_t b = sh[2];
    const uint32_t c = sh[3];
    if (sh[4]) {
      // protect pass over [lo+1, b): X = len > plen stays left, E = len <= plen goes right
      uint32_t xc = 0;
      for (uint32_t p = lo + 1 + threadIdx.x; p < b; p += QB) xc += LEN(el[p]) > plen;
      const uint32_t b2 = lo + 1 + block_sum<QB>(xc, red);
      const uint32_t nE = block_collect(lo + 1, b2, [&](uint32_t p) { return LEN(el[p]) <= plen; }, A, red);
      const uint32_t nX = block_collect(b2, b, [&](uint32_t p) { return LEN(el[p]) > plen; }, B, red);
      __syncthreads();
      (void)nX;
      for (uint32_t k = threadIdx.x; k < nE; k += QB) swp(el, A[k], B[nE - 1 - k]);
      __syncthreads();
      b = b2;
    }
    if (threadIdx.x == 0) {
      swp(el, lo, b - 1);
      route(lo, b - 1, sg.depth - 1, fin_max, big, fin, heap, cnt);
      route(c, hi, sg.depth - 1, fin_max, big, fin, heap, cnt);
    }
    __syncthreads();
  }
}

__global__ void k_qs_heap(uint64_t* el, const Seg* segs, uint32_t nsegs) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsegs; i += gridDim.x * blockDim.x)
    heap_sort(el, segs[i].lo, segs[i].hi);
}

// ---- finisher: one wave per segment <= FIN_MAX, in LDS ----------------------------------------
constexpr int FIN_WAVES = 4;
constexpr int FIN_STACK = 64;

template <class Pred>
__device__ uint32_t wave_collect(uint32_t beg, uint32_t end, Pred pred, uint16_t* out) {
  uint32_t k = 0;
  for (uint32_t base = beg; base < end; base += 64) {
    const uint32_t p = base + __lane_id();
    const bool f = p < end && pred(p);
    const uint64_t mask = __ballot(f);
    if (f) out[k + __popcll(mask & lanemask_lt())] = (uint16_t)p;
    k += __popcll(mask);
  }
  return k;
}

__global__ __launch_bounds__(64 * FIN_WAVES) void k_qs_finish(uint64_t* __restrict__ el, const Seg* segs,
                                                              uint32_t nsegs) {
  __shared__ uint64_t sel[FIN_WAVES][FIN_MAX];
  __shared__ uint16_t sA[FIN_WAVES][FIN_MAX / 2];
  __shared__ uint16_t sB[FIN_WAVES][FIN_MAX / 2];
  __shared__ uint32_t stk[FIN_WAVES][FIN_STACK][3];
  __shared__ uint32_t bc[FIN_WAVES][4];
  const int w = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  uint64_t* d = sel[w];
  uint16_t* A = sA[w];
  uint16_t* B = sB[w];
  for (uint32_t si = blockIdx.x * FIN_WAVES + w; si < nsegs; si += gridDim.x * FIN_WAVES) {
    const Seg sg = segs[si];
    const uint32_t n = sg.hi - sg.lo;
    for (uint32_t i = lane; i < n; i += 64) d[i] = el[sg.lo + i];
    int sp = 0;
    if (lane == 0) {
      stk[w][0][0] = 0;
      stk[w][0][1] = n;
      stk[w][0][2] = (uint32_t)sg.depth;
    }
    sp = 1;
    wave_sync();
    while (sp > 0) {
      sp--;
      const uint32_t lo = stk[w][sp][0], hi = stk[w][sp][1];
      const int32_t depth = (int32_t)stk[w][sp][2];
      wave_sync();
      if (hi - lo <= 12) {
        if (lane == 0 && hi - lo > 1) shell_insertion(d, lo, hi);
        wave_sync();
        continue;
      }
      if (depth == 0) {
        if (lane == 0) heap_sort(d, lo, hi);
        wave_sync();
        continue;
      }
      if (lane == 0) {
        bc[w][1] = choose_pivot(d, lo, hi);
        bc[w][0] = LEN(d[lo]);
      }
      wave_sync();
      const uint32_t plen = bc[w][0], m = bc[w][1];
      uint32_t lc = 0;
      for (uint32_t p = lo + 1 + lane; p < hi - 1; p += 64) lc += LEN(d[p]) >= plen;
      const uint32_t bnd = lo + 1 + wave_sum(lc);
      const uint32_t nG = wave_collect(lo + 1, bnd, [&](uint32_t p) { return LEN(d[p]) < plen; }, A);
      (void)wave_collect(bnd, hi - 1, [&](uint32_t p) { return LEN(d[p]) >= plen; }, B);
      wave_sync();
      for (uint32_t k = lane; k < nG; k += 64) swp(d, A[k], B[nG - 1 - k]);
      wave_sync();
      if (lane == 0) {
        uint32_t b = bnd, c = bnd;
        bc[w][3] = dups_probe(d, lo, hi, m, &b, &c);
        bc[w][1] = b;
        bc[w][2] = c;
      }
      wave_sync();
      uint32_t b = bc[w][1];
      const uint32_t c = bc[w][2];
      if (bc[w][3]) {
        uint32_t xc = 0;
        for (uint32_t p = lo + 1 + lane; p < b; p += 64) xc += LEN(d[p]) > plen;
        const uint32_t b2 = lo + 1 + wave_sum(xc);
        const uint32_t nE = wave_collect(lo + 1, b2, [&](uint32_t p) { return LEN(d[p]) <= plen; }, A);
        (void)wave_collect(b2, b, [&](uint32_t p) { return LEN(d[p]) > plen; }, B);
        wave_sync();
        for (uint32_t k = lane; k < nE; k += 64) swp(d, A[k], B[nE - 1 - k]);
        wave_sync();
        b = b2;
      }
      if (lane == 0) {
        swp(d, lo, b - 1);
        stk[w][sp][0] = lo;
        stk[w][sp][1] = b - 1;
        stk[w][sp][2] = (uint32_t)(depth - 1);
        stk[w][sp + 1][0] = c;
        stk[w][sp + 1][1] = hi;
        stk[w][sp + 1][2] = (uint32_t)(depth - 1);
      }
      sp += 2;
      wave_sync();
    }
    for (uint32_t i = lane; i < n; i += 64) el[sg.lo + i] = d[i];
    wave_sync();
  }
}

__global__ void k_qs_roots(const uint64_t* gstart, uint32_t ngroups, uint32_t fin_max, Seg* big, Seg* fin,
                           Seg* heap, uint32_t* cnt) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += gridDim.x * blockDim.x) {
    const uint32_t lo = (uint32_t)gstart[g], hi = (uint32_t)gstart[g + 1];
    uint32_t depth = 0;
    for (uint32_t i = hi - lo; i > 0; i >>= 1) depth++;
    route(lo, hi, (int32_t)(2 * depth), fin_max, big, fin, heap, cnt);
  }
}

// Sorts every group's [gstart[g], gstart[g+1]) range of el with Go's sort.Sort semantics.
void gosort_groups(uint64_t* el, size_t n, const uint64_t* gstart_dev, uint32_t ngroups, hipStream_t s) {
  Context& c = ctx();
  const size_t maxseg = n / 2 + ngroups + 16;
  Seg* bigA = c.scratch.get<Seg>("qs_bigA", maxseg);
  Seg* bigB = c.scratch.get<Seg>("qs_bigB", maxseg);
  Seg* fin = c.scratch.get<Seg>("qs_fin", maxseg);
  Seg* heap = c.scratch.get<Seg>("qs_heap", maxseg);
  uint32_t* tmpA = c.scratch.get<uint32_t>("qs_tmpA", n + 1);
  uint32_t* tmpB = c.scratch.get<uint32_t>("qs_tmpB", n + 1);
  uint32_t* cnt = c.scratch.get<uint32_t>("qs_cnt", 8);
  uint32_t* hcnt = c.pinned.get<uint32_t>(8);
  SYZ_HIP(hipMemsetAsync(cnt, 0, 8 * sizeof(uint32_t), s));
  {
    ProfScope ps("gosort_roots", s, 0);
    k_qs_roots<<<grid_for(ngroups, 256, 1024), 256, 0, s>>>(gstart_dev, ngroups, FIN_MAX, bigA, fin, heap, cnt);
    SYZ_LAUNCHED();
  }
  SYZ_HIP(hipMemcpyAsync(hcnt, cnt, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  uint32_t nbig = hcnt[0];
  int level = 0;
  while (nbig > 0) {
    SYZ_HIP(hipMemsetAsync(cnt, 0, sizeof(uint32_t), s));  // next big count; fin/heap keep appending
    {
      ProfScope ps("gosort_level", s, 0);
      k_qs_level<<<(unsigned)std::min<uint32_t>(nbig, 4096), QB, 0, s>>>(el, tmpA, tmpB, bigA, nbig, bigB, fin,
                                                                          heap, cnt, FIN_MAX);
      SYZ_LAUNCHED();
    }
    SYZ_HIP(hipMemcpyAsync(hcnt, cnt, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    nbig = hcnt[0];
    std::swap(bigA, bigB);
    if (++level > 4096) fail(SYZGPU_EINTERNAL, "gosort: level limit");
  }
  const uint32_t nfin = hcnt[1], nheap = hcnt[2];
  if (nheap) {
    k_qs_heap<<<grid_for(nheap, 64, 4096), 64, 0, s>>>(el, heap, nheap);
    SYZ_LAUNCHED();
  }
  if (nfin) {
    ProfScope ps("gosort_finish", s, 0);
    k_qs_finish<<<(unsigned)std::min<uint32_t>((nfin + FIN_WAVES - 1) / FIN_WAVES, 8192), 64 * FIN_WAVES, 0, s>>>(
        el, fin, nfin);
    SYZ_LAUNCHED();
  }
}

}  // namespace syz

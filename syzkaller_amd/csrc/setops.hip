// Coverage set algebra on sorted uint32 PC lists — cover/cover.go:28-102.
//
// foreach (cover.go:81-102) walks two sorted lists with two pointers that both advance on equal
// values. On sorted inputs that is a multiset merge: for a value v occurring ca times in a and cb
// times in b, the first min(ca, cb) copies are paired. So each element's fate is a local function of
// (its rank inside its run of equal values, the count of v in the other list):
//   Difference            keep a[x] iff rank_a >= cb
//   Intersection          keep a[x] iff rank_a <  cb
//   Union                 keep every a[x]; keep b[y] iff rank_b >= ca
//   SymmetricDifference   keep a[x] iff rank_a >= cb; keep b[y] iff rank_b >= ca
// and 0xFFFFFFFF (the sentinel, cover.go:17) is never emitted. Outputs are placed by prefix sums
// of the keep flags — one lane per element (a wave per pair), no sequential merge.
//
// Canonicalize (cover.go:28-40): per-cover sort in LDS (bitonic, up to 16384 PCs = the kcov limit,
// executor.cc:48) or a global bitonic network beyond, then unique with last = sentinel.
#include <algorithm>

#include "pipeline.hpp"

namespace syz {

// ---- batched set operations -------------------------------------------------------------------


// Work unit: a segment of <= SO_SEG consecutive elements of one pair's list (a pair of n elements has
// ceil(n / SO_SEG) segments; segoff = their exclusive scan over the pairs), one wave per segment
// (grid-stride): the pair is found once per segment, so an element costs only its searches inside
// the other list, whose few lines the wave's lanes share through L1; long lists still spread over
// many waves.
constexpr uint64_t SO_SEG = 1024;

__global__ void k_setop_nseg(const uint64_t* off, uint32_t npairs, uint32_t* nseg) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += gridDim.x * blockDim.x)
    nseg[p] = (uint32_t)((off[p + 1] - off[p] + SO_SEG - 1) / SO_SEG);
}

// segment sid -> (pair, element range)
__device__ __forceinline__ uint32_t seg_pair(const uint64_t* segoff, uint32_t npairs, uint64_t sid, const uint64_t* off,
                                             uint64_t* x0, uint64_t* x1) {
  const uint32_t p = (uint32_t)upper_bound_dev<uint64_t>(segoff, 0, npairs + 1, sid) - 1;
  *x0 = off[p] + (sid - segoff[p]) * SO_SEG;
  *x1 = min(off[p + 1], *x0 + SO_SEG);
  return p;
}

// side 0 classifies a-elements against b, side 1 b-elements against a.
__global__ __launch_bounds__(256) void k_setop_classify(int op, int side, const uint32_t* a, const uint64_t* aoff,
                                                        const uint32_t* b, const uint64_t* boff, uint32_t npairs,
                                                        const uint64_t* segoff, uint8_t* keep, int* err) {
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6, nseg = segoff[npairs];
  for (uint64_t sid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; sid < nseg; sid += waves) {
    uint64_t x0, x1;
    const uint32_t p = seg_pair(segoff, npairs, sid, aoff, &x0, &x1);
    const uint64_t beg = aoff[p], end = aoff[p + 1], b0 = boff[p], b1 = boff[p + 1];
    for (uint64_t x = x0 + __lane_id(); x < x1; x += 64) {
      const uint32_t v = a[x];
      if (x + 1 < end && a[x + 1] < v) atomicOr(err, 1);  // unsorted input
      uint8_t k = 0;
      if (v != SENT) {
        uint64_t rank = 0;
        if (x > beg && a[x - 1] == v) rank = x - lower_bound_dev<uint32_t>(a, beg, x, v);
        const uint64_t lb = lower_bound_dev<uint32_t>(b, b0, b1, v);
        uint64_t cnt = 0;
        if (lb < b1 && b[lb] == v) cnt = upper_bound_dev<uint32_t>(b, lb, b1, v) - lb;
        if (side == 0) {
          switch (op) {
            case SYZGPU_DIFFERENCE:
            case SYZGPU_SYMMETRIC_DIFFERENCE: k = rank >= cnt; break;
            case SYZGPU_UNION: k = 1; break;
            default: k = rank < cnt; break;
          }
        } else {
          k = (op == SYZGPU_UNION || op == SYZGPU_SYMMETRIC_DIFFERENCE) ? (rank >= cnt) : 0;
        }
      }
      keep[x] = k;
    }
  }
}

__global__ void k_setop_pairlen(const uint64_t* aoff, const uint64_t* boff, const uint64_t* ka, const uint64_t* kb,
                                uint32_t npairs, uint64_t* plen) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += gridDim.x * blockDim.x)
    plen[p] = (ka[aoff[p + 1]] - ka[aoff[p]]) + (kb[boff[p + 1]] - kb[boff[p]]);
}

// Scatter kept elements of one side. For side 0 (a): pos = KA(x) + KB(lb_b(v)); side 1 (b):
// pos = KB(y) + KA(ub_a(w)) — equal values from a precede those from b (they are identical). One wave
// per pair, as k_setop_classify.
__global__ __launch_bounds__(256) void k_setop_scatter(int side, const uint32_t* a, const uint64_t* aoff,
                                                       const uint32_t* b, const uint64_t* boff, uint32_t npairs,
                                                       const uint64_t* segoff, const uint8_t* keep, const uint64_t* ka,
                                                       const uint64_t* kb, const uint64_t* outoff, uint32_t* out) {
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6, nseg = segoff[npairs];
  for (uint64_t sid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; sid < nseg; sid += waves) {
    uint64_t x0, x1;
    const uint32_t p = seg_pair(segoff, npairs, sid, aoff, &x0, &x1);
    const uint64_t beg = aoff[p], b0 = boff[p], b1 = boff[p + 1];
    const uint64_t base = outoff[p] - ka[beg] - kb[b0];
    for (uint64_t x = x0 + __lane_id(); x < x1; x += 64) {
      if (!keep[x]) continue;
      const uint32_t v = a[x];
      const uint64_t other = side == 0 ? lower_bound_dev<uint32_t>(b, b0, b1, v) : upper_bound_dev<uint32_t>(b, b0, b1, v);
      out[base + ka[x] + kb[other]] = v;
    }
  }
}

// ---- merge-path tiles (strictly increasing lists, the kcov case) --------------------------------
// For strictly increasing lists foreach's walk (cover.go:81-102) is the stable merge (a first on ties)
// in which an element is PAIRED iff its merged neighbour holds the same value: a[i] with the b at the
// walk's b pointer when a[i] is taken, b[j] with the a taken just before it. So every pair's merged
// sequence is cut into tiles of SO_T merged elements at merge-path diagonals; a tile's two sub-lists
// (+ one halo element each) are staged in LDS with coalesced loads, each thread merges SO_VT elements
// from its own diagonal, and the pass either counts the op's outputs per tile (count) or, after a scan
// of the counts, stages them in LDS and stores the tile's run coalesced (emit). A pair with a repeated
// value (allowed by Go, never produced by the executor's sort + unique) sends the batch to the
// per-element rank path above; a descending neighbour is the Go panic (EINVAL).
#ifndef SYZ_SO_BLOCK
#define SYZ_SO_BLOCK 128
#endif
#ifndef SYZ_SO_VT
#define SYZ_SO_VT 8
#endif
constexpr int SO_BLOCK = SYZ_SO_BLOCK;
constexpr int SO_VT = SYZ_SO_VT;
constexpr uint32_t SO_T = SO_BLOCK * SO_VT;  // merged elements per tile
constexpr int SO_LOG_T = SO_T == 512 ? 9 : SO_T == 1024 ? 10 : SO_T == 2048 ? 11 : SO_T == 4096 ? 12 : -1;
static_assert(SO_LOG_T > 0 && SO_T == 1u << SO_LOG_T, "tile size");

__global__ void k_so_ntiles(const uint64_t* aoff, const uint64_t* boff, uint32_t npairs, uint32_t* nt) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += gridDim.x * blockDim.x) {
    const uint64_t m = (aoff[p + 1] - aoff[p]) + (boff[p + 1] - boff[p]);
    nt[p] = (uint32_t)((m + SO_T - 1) / SO_T);
  }
}

// tpair[t] = the pair of tile t
__global__ void k_so_tpair(const uint64_t* tstart, uint32_t npairs, uint32_t* tpair) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += gridDim.x * blockDim.x)
    for (uint64_t t = tstart[p]; t < tstart[p + 1]; t++) tpair[t] = p;
}

// merge path: the number of a-elements among the first d merged ones (a first on ties)
template <class RA, class RB>
__device__ __forceinline__ uint32_t merge_path(RA A, uint32_t la, RB B, uint32_t lb, uint32_t d) {
  uint32_t lo = d > lb ? d - lb : 0u, hi = d < la ? d : la;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (A(mid) <= B(d - mid - 1))
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// the same search with three probes a step (a quarter of the range left each time): half the chain of
// dependent loads of merge_path when the lists are in HBM (the probes' loads are in flight together)
template <class RA, class RB>
__device__ __forceinline__ uint32_t merge_path4(RA A, uint32_t la, RB B, uint32_t lb, uint32_t d) {
  uint32_t lo = d > lb ? d - lb : 0u, hi = d < la ? d : la;
  while (hi - lo >= 4) {  // every probe i in [lo, hi): A(i) and B(d - i - 1) exist
    const uint32_t n = hi - lo, m1 = lo + n / 4, m2 = lo + n / 2, m3 = lo + 3 * (n / 4);
    const uint32_t a1 = A(m1), b1 = B(d - m1 - 1), a2 = A(m2), b2 = B(d - m2 - 1), a3 = A(m3), b3 = B(d - m3 - 1);
    if (!(a1 <= b1)) {
      hi = m1;
    } else if (!(a2 <= b2)) {
      lo = m1 + 1;
      hi = m2;
    } else if (!(a3 <= b3)) {
      lo = m2 + 1;
      hi = m3;
    } else {
      lo = m3 + 1;
    }
  }
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (A(mid) <= B(d - mid - 1))
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// A tile's sub-lists a[a0, a0 + na) and b[b0, b0 + nb) (n = na | nb << 16) and its halo values: aprev, the a
// taken just before the tile (a[a0 - 1]; without one, b[b0] - 1, which pairs with no b of the tile but a
// sentinel); anext / bnext, the a / b taken after it (0xFFFFFFFF past the pair's end: the sentinel is never
// an output). With them a tile's merge is closed: an exhausted list reads its halo, which orders after
// everything the other list still has in the tile (the merge-path property), and a pairing across a tile
// edge is a compare against a halo. Built once per batch (which also checks the list order across tile
// edges), so a tile walk's only dependent read is this 32-byte record.
struct SoDesc {
  uint64_t a0, b0;
  uint32_t n, aprev, anext, bnext;
};

// one thread per tile: its pair and merge-path diagonals (a one-tile pair needs no search)
__global__ void k_so_tdesc(const uint32_t* __restrict__ a, const uint64_t* __restrict__ aoff,
                           const uint32_t* __restrict__ b, const uint64_t* __restrict__ boff,
                           const uint64_t* __restrict__ tstart, const uint32_t* __restrict__ tpair, uint32_t npairs,
                           SoDesc* __restrict__ desc, int* flags, int* err) {
  const uint64_t ntiles = tstart[npairs];
  // (block-uniform loop: the lanes of a wave exchange their diagonals)
  for (uint64_t tb = blockIdx.x * (uint64_t)blockDim.x; tb < ntiles; tb += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t t = tb + threadIdx.x;
    const bool ok = t < ntiles;
    const uint32_t p = ok ? tpair[t] : 0u;
    const uint64_t a0 = ok ? aoff[p] : 0, b0 = ok ? boff[p] : 0;
    const uint32_t la = ok ? (uint32_t)(aoff[p + 1] - a0) : 0u, lb = ok ? (uint32_t)(boff[p + 1] - b0) : 0u;
    const uint32_t d0 = ok ? (uint32_t)(t - tstart[p]) * SO_T : 0u, d1 = min(d0 + SO_T, la + lb);
    auto ga = [&](uint32_t i) { return a[a0 + i]; };
    auto gb = [&](uint32_t j) { return b[b0 + j]; };
    const uint32_t i1 = d1 == la + lb ? la : merge_path4(ga, la, gb, lb, d1);
    // a tile's start diagonal is the end of the tile before it: the lane before's, when it holds it
    const uint32_t i1p = (uint32_t)__shfl_up((int)i1, 1, 64), pp = (uint32_t)__shfl_up((int)p, 1, 64);
    const bool nb = __lane_id() > 0 && pp == p;
    const uint32_t i0 = d0 == 0 ? 0u : nb ? i1p : merge_path4(ga, la, gb, lb, d0);
    if (!ok) continue;
    const uint32_t j0 = d0 - i0, j1 = d1 - i1;
    // the order of the neighbours this tile's end separates
    int f = 0, e = 0;
    if (i1 > 0 && i1 < la) {
      const uint32_t x = a[a0 + i1 - 1], y = a[a0 + i1];
      f |= x == y;
      e |= y < x;
    }
    if (j1 > 0 && j1 < lb) {
      const uint32_t x = b[b0 + j1 - 1], y = b[b0 + j1];
      f |= x == y;
      e |= y < x;
    }
    if (f) atomicOr(flags, 1);
    if (e) atomicOr(err, 1);
    SoDesc d;
    d.a0 = a0 + i0;
    d.b0 = b0 + j0;
    d.n = (i1 - i0) | (j1 - j0) << 16;
    d.aprev = i0 > 0 ? a[a0 + i0 - 1] : j0 < j1 ? b[b0 + j0] - 1u : 0u;
    d.anext = i1 < la ? a[a0 + i1] : 0xFFFFFFFFu;
    d.bnext = j1 < lb ? b[b0 + j1] : 0xFFFFFFFFu;
    desc[t] = d;
  }
}

constexpr int SO_RSRC_FLAGS = 0x00020000;

// SO_COUNT: tcnt[tile] = outputs of the tile; flags bit 0 = a repeated value, err = descending
// SO_EMIT: the tile's outputs at out[tout[tile]..] (after a scan of the counts)
// SO_GAP: both in one pass, the outputs at out[a0 + b0..] (the tile's merged start: a gapped image of the
// result in a scratch of na + nb words, which k_so_compact closes up after the scan)
// A grid of a few workgroups per CU walks the tiles (one workgroup per tile made the launch's dispatch
// the bound: ~1M short workgroups per batch). The walk is software-pipelined: while tile k merges out of
// LDS, tile k+1's elements and tile k+2's record are in flight into registers. Every global access is a
// buffer op whose descriptor range is the tile's own (out-of-range loads return 0, stores are dropped),
// so the loop has no data-dependent branches around memory and the only wait before staging a tile is
// for its own loads (issued a merge earlier), not for the stores behind them.
constexpr int SO_COUNT = 0, SO_EMIT = 1, SO_GAP = 2;
template <int MODE>
__global__ __launch_bounds__(SO_BLOCK) void k_so_tile(int op, const uint32_t* __restrict__ a,
                                                      const uint32_t* __restrict__ b,
                                                      const SoDesc* __restrict__ desc,
                                                      const uint64_t* __restrict__ ntiles_dev, uint32_t* tcnt,
                                                      const uint64_t* __restrict__ tout, uint32_t* out, int* flags,
                                                      int* err) {
  constexpr bool EMIT = MODE != SO_COUNT, CHECK = MODE != SO_EMIT, DIRECT = MODE == SO_EMIT;
  // (+ SO_VT + 1: a walk that runs past a list's end reads on, ignored, instead of clamping its index)
  __shared__ __attribute__((aligned(16))) uint32_t As[SO_T + SO_VT + 4], Bs[SO_T + SO_VT + 4];
  __shared__ uint32_t st[EMIT ? SO_T + 1 : 1];
  __shared__ uint32_t red[SO_BLOCK / 64 + 1];
  // the op's outputs (cover.go:81-102): a paired / a unpaired / b unpaired (a paired b is never one)
  const bool eap = op == SYZGPU_INTERSECTION || op == SYZGPU_UNION;
  const bool eau = op != SYZGPU_INTERSECTION;
  const bool ebu = op == SYZGPU_UNION || op == SYZGPU_SYMMETRIC_DIFFERENCE;
  const uint64_t ntiles = *ntiles_dev;
  uint64_t tile = blockIdx.x;
  if (tile >= ntiles) return;
  const uint32_t lane = __lane_id();
  // a tile's record (lanes 0..7, one word each) and, for EMIT, its output offset (lanes 0..1)
  auto rec_load = [&](uint64_t t) {
    const bool ok = t < ntiles;
    const auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(desc + (ok ? t : 0)), 0, ok ? 32 : 0, SO_RSRC_FLAGS);
    return __builtin_amdgcn_raw_buffer_load_b32(r, (lane & 7) * 4, 0, 0);
  };
  auto tout_load = [&](uint64_t t) {
    const bool ok = DIRECT && t < ntiles;
    const auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(tout + (ok ? t : 0)), 0, ok ? 8 : 0, SO_RSRC_FLAGS);
    return __builtin_amdgcn_raw_buffer_load_b32(r, (lane & 1) * 4, 0, 0);
  };
  uint32_t ra[SO_VT], rb[SO_VT];
  auto fetch = [&](uint64_t a0, uint32_t na, uint64_t b0, uint32_t nb) {
    const auto rsa = __builtin_amdgcn_make_buffer_rsrc((void*)(a + a0), 0, na * 4, SO_RSRC_FLAGS);
    const auto rsb = __builtin_amdgcn_make_buffer_rsrc((void*)(b + b0), 0, nb * 4, SO_RSRC_FLAGS);
#pragma unroll
    for (int r = 0; r < SO_VT; r++) {
      ra[r] = __builtin_amdgcn_raw_buffer_load_b32(rsa, (threadIdx.x + r * SO_BLOCK) * 4, 0, 0);
      rb[r] = __builtin_amdgcn_raw_buffer_load_b32(rsb, (threadIdx.x + r * SO_BLOCK) * 4, 0, 0);
    }
  };
  auto field = [](uint32_t w, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)w, k); };
  auto a0_of = [&](uint32_t w) { return (uint64_t)field(w, 0) | (uint64_t)field(w, 1) << 32; };
  auto b0_of = [&](uint32_t w) { return (uint64_t)field(w, 2) | (uint64_t)field(w, 3) << 32; };
  // prologue: tile k's record (waited for), its elements, tile k+1's record and tile k's output offset
  uint32_t dw = rec_load(tile);
  uint32_t na = field(dw, 4) & 0xFFFFu, nb = field(dw, 4) >> 16;
  uint32_t hp = field(dw, 5), ha = field(dw, 6), hb = field(dw, 7);
  uint64_t gbase = a0_of(dw) + b0_of(dw);  // SO_GAP's output offset of the tile in flight
  fetch(a0_of(dw), na, b0_of(dw), nb);
  dw = rec_load(tile + gridDim.x);
  uint32_t tw = tout_load(tile);
  {
    // as many (empty-range, dropped) stores as an iteration ends with, so the loop head's wait for the
    // loads above is the same counted vmcnt on entry as on the back edge (else the merge makes it vmcnt(0),
    // a wait for the previous tile's stores)
    const auto rz = __builtin_amdgcn_make_buffer_rsrc((void*)(EMIT ? out : tcnt), 0, 0, SO_RSRC_FLAGS);
#pragma unroll
    for (int r = 0; r < (EMIT ? SO_VT : 0) + (CHECK ? 1 : 0); r++)
      __builtin_amdgcn_raw_buffer_store_b32(0u, rz, (threadIdx.x + r * SO_BLOCK) * 4, 0, 0);
  }
  int f = 0, e = 0;  // a repeated value / a descending neighbour, over all of this thread's tiles
  for (;;) {
#pragma unroll
    for (int r = 0; r < SO_VT; r++) {
      As[threadIdx.x + r * SO_BLOCK] = ra[r];
      Bs[threadIdx.x + r * SO_BLOCK] = rb[r];
    }
    const uint64_t obase = DIRECT ? (uint64_t)field(tw, 0) | (uint64_t)field(tw, 1) << 32 : gbase;
    const uint32_t cna = na, cnb = nb, chp = hp, cha = ha, chb = hb;
    const uint64_t next = tile + gridDim.x;
    __syncthreads();
    // tile k+1: its elements in flight during this merge (a past-the-end tile loads nothing)
    {
      const bool ok = next < ntiles;
      na = ok ? field(dw, 4) & 0xFFFFu : 0;
      nb = ok ? field(dw, 4) >> 16 : 0;
      hp = field(dw, 5);
      ha = field(dw, 6);
      hb = field(dw, 7);
      fetch(ok ? a0_of(dw) : 0, na, ok ? b0_of(dw) : 0, nb);
      gbase = ok ? a0_of(dw) + b0_of(dw) : 0;
      dw = rec_load(next + gridDim.x);
      tw = tout_load(next);
    }
    // this thread's merged range [t * VT, (t + 1) * VT) of the tile, from the merge path at its start by
    // a fixed number of halvings
    const uint32_t m = cna + cnb, dt0 = min((uint32_t)threadIdx.x * SO_VT, m);
    uint32_t lo = dt0 > cnb ? dt0 - cnb : 0u, hi = min(dt0, cna);
#pragma unroll
    for (int it = 0; it < SO_LOG_T + 1; it++) {
      const uint32_t mid = (lo + hi) >> 1;
      const bool le = As[mid & (SO_T - 1)] <= Bs[(dt0 - mid - 1) & (SO_T - 1)];
      const bool live = lo < hi;
      lo = (live & le) ? mid + 1 : lo;
      hi = (live & !le) ? mid : hi;
    }
    uint32_t i = lo, j = dt0 - lo;
    const uint32_t pv = As[i > 0 ? i - 1 : 0];
    uint32_t pa = i > 0 ? pv : chp;  // the a taken just before
    uint32_t outv[SO_VT];
    uint32_t c = 0, em = 0;  // em bit r: merged element dt0 + r is an output
#pragma unroll
    for (int r = 0; r < SO_VT; r++) {
      const uint32_t av = As[i], bv = Bs[j];
      const uint32_t ae = i < cna ? av : cha, be = j < cnb ? bv : chb;  // an exhausted list reads its halo
      const bool take_a = ae <= be;
      const uint32_t v = take_a ? ae : be;
      // a: paired with the b at the walk's pointer; b: with the a taken just before it
      const bool paired = (take_a ? be : pa) == v;
      const bool out_a = paired ? eap : eau;
      const bool emit = (dt0 + r < m) & (v != SENT) & (take_a ? out_a : (!paired & ebu));
      outv[r] = v;
      em |= emit ? 1u << r : 0u;
      c += emit ? 1u : 0u;
      pa = take_a ? ae : pa;
      i += take_a ? 1u : 0u;
      j += take_a ? 0u : 1u;
    }
    uint32_t tot;
    const uint32_t pre = block_excl_scan<SO_BLOCK>(c, red, &tot);
    tot = __builtin_amdgcn_readfirstlane(tot);  // (uniform: a store range from a VGPR is a waterfall loop)
    if (CHECK) {
      const auto rc = __builtin_amdgcn_make_buffer_rsrc((void*)(tcnt + tile), 0, 4, SO_RSRC_FLAGS);
      __builtin_amdgcn_raw_buffer_store_b32(tot, rc, threadIdx.x * 4, 0, 0);  // thread 0's store is the one in range
    }
    if (EMIT) {
#pragma unroll
      for (int r = 0; r < SO_VT; r++)
        st[(em >> r & 1) ? pre + __popc(em & ((1u << r) - 1)) : SO_T] = outv[r];  // st[SO_T]: a dump slot
      __syncthreads();
      const auto ro = __builtin_amdgcn_make_buffer_rsrc((void*)(out + obase), 0, tot * 4, SO_RSRC_FLAGS);
#pragma unroll
      for (int r = 0; r < SO_VT; r++) {
        const uint32_t k = threadIdx.x + r * SO_BLOCK;
        __builtin_amdgcn_raw_buffer_store_b32(st[k], ro, k * 4, 0, 0);
      }
    }
    // order checks inside the tile (its edges are the record builder's), after the merge so that their
    // reads are not hoisted into it (register pressure); like the merge, branch-free
    if (CHECK) {  // (the emit pass runs only on checked input)
      const uint32_t k0 = threadIdx.x * SO_VT;  // this thread's VT neighbours of each list, read as b128s
#pragma unroll
      for (int side = 0; side < 2; side++) {
        const uint32_t* S = side ? Bs : As;
        const uint32_t n = side ? cnb : cna;
#pragma unroll
        for (int q = 0; q < SO_VT; q += 4) {  // a b128 and the element after it at a time (few live VGPRs)
          const uint4 x = *reinterpret_cast<const uint4*>(S + k0 + q);
          const uint32_t v[5] = {x.x, x.y, x.z, x.w, S[(k0 + q + 4) & (SO_T - 1)]};
#pragma unroll
          for (int u = 0; u < 4; u++) {
            const bool ok = k0 + q + u + 1 < n;
            f |= ok & (v[u] == v[u + 1]);  // (bitwise: && would become branches)
            e |= ok & (v[u + 1] < v[u]);
          }
        }
      }
    }
    __syncthreads();  // the tile's LDS is free for the next one
    if (next >= ntiles) break;
    tile = next;
  }
  if (__ballot(f)) {
    if (lane == 0) atomicOr(flags, 1);
  }
  if (__ballot(e)) {
    if (lane == 0) atomicOr(err, 1);
  }
}

// SO_GAP's gapped image closed up: tile t's tcnt[t] outputs from gap[a0 + b0..] to out[tout[t]..]. Each
// WAVE walks its own tiles (no LDS, no barrier: more tiles in flight per CU for a walk that is all
// latency), two tiles deep (see step below).
constexpr int SC_VT = SO_T / 64;
#ifndef SYZ_SC_DEPTH
#define SYZ_SC_DEPTH 2
#endif
constexpr int SC_DEPTH = SYZ_SC_DEPTH;  // tiles in flight per compaction wave
__global__ __launch_bounds__(SO_BLOCK) void k_so_compact(const SoDesc* __restrict__ desc,
                                                         const uint32_t* __restrict__ tcnt,
                                                         const uint64_t* __restrict__ tout,
                                                         const uint64_t* __restrict__ ntiles_dev,
                                                         const uint32_t* __restrict__ gap, uint32_t* out,
                                                         uint64_t out_cap) {
  const uint64_t ntiles = *ntiles_dev;
  const uint64_t stride = (uint64_t)gridDim.x * (SO_BLOCK / 64);
  uint64_t tile = (uint64_t)blockIdx.x * (SO_BLOCK / 64) + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (tile >= ntiles) return;
  const uint32_t lane = __lane_id();
  // a tile's offsets, one word a lane: 0..3 the record's a0/b0, 4 its count, 5..6 its output offset
  auto meta_load = [&](uint64_t t) {
    const bool ok = t < ntiles;
    const uint64_t tt = ok ? t : 0;
    const auto rd = __builtin_amdgcn_make_buffer_rsrc((void*)(desc + tt), 0, ok ? 16 : 0, SO_RSRC_FLAGS);
    const auto rc = __builtin_amdgcn_make_buffer_rsrc((void*)(tcnt + tt), 0, ok ? 4 : 0, SO_RSRC_FLAGS);
    const auto ro = __builtin_amdgcn_make_buffer_rsrc((void*)(tout + tt), 0, ok ? 8 : 0, SO_RSRC_FLAGS);
    const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(rd, (lane & 3) * 4, 0, 0);
    const uint32_t y = __builtin_amdgcn_raw_buffer_load_b32(rc, 0, 0, 0);
    const uint32_t z = __builtin_amdgcn_raw_buffer_load_b32(ro, (lane & 1) * 4, 0, 0);
    return lane < 4 ? x : lane == 4 ? y : z;  // (lanes 5, 6: z's words 1, 0; fixed below)
  };
  auto field = [](uint32_t w, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)w, k); };
  auto src_of = [&](uint32_t w) {
    return ((uint64_t)field(w, 0) | (uint64_t)field(w, 1) << 32) + ((uint64_t)field(w, 2) | (uint64_t)field(w, 3) << 32);
  };
  auto dst_of = [&](uint32_t w) { return (uint64_t)field(w, 6) | (uint64_t)field(w, 5) << 32; };  // lane 6: word 0
  auto fetch = [&](uint32_t w, bool ok, uint32_t* v) {
    const uint32_t n = ok ? field(w, 4) : 0;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(gap + (ok ? src_of(w) : 0)), 0, n * 4, SO_RSRC_FLAGS);
#pragma unroll
    for (int r = 0; r < SC_VT; r++)
      if (r * 64 < (int)n) v[r] = __builtin_amdgcn_raw_buffer_load_b32(rs, (lane + r * 64) * 4, 0, 0);
  };
  // SC_DEPTH tiles' words and SC_DEPTH more tiles' offsets in flight per wave: tile k is stored from
  // D[k % SC_DEPTH] while tile k + SC_DEPTH's words load into it (its offsets were read SC_DEPTH steps ago)
  // and tile k + 2 SC_DEPTH's offsets into M[k % SC_DEPTH]
  uint32_t D[SC_DEPTH][SC_VT], M[SC_DEPTH], nn[SC_DEPTH];
  uint64_t dd[SC_DEPTH];
#pragma unroll
  for (int q = 0; q < SC_DEPTH; q++) {
    const bool ok = tile + q * stride < ntiles;
    const uint32_t m = meta_load(tile + q * stride);
    nn[q] = ok ? field(m, 4) : 0;
    dd[q] = ok ? dst_of(m) : 0;
    fetch(m, ok, D[q]);
  }
#pragma unroll
  for (int q = 0; q < SC_DEPTH; q++) M[q] = meta_load(tile + (SC_DEPTH + q) * stride);
  {
    const auto rz = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, 0, SO_RSRC_FLAGS);  // (see k_so_tile)
#pragma unroll
    for (int r = 0; r < SC_VT; r++)
      __builtin_amdgcn_raw_buffer_store_b32(0u, rz, (lane + r * 64) * 4, 0, 0);
  }
  auto step = [&](uint32_t* Dq, uint32_t& Mq, uint32_t& n, uint64_t& d) {
    // (launched before the host has checked the total against out_cap: stores past it are dropped)
    const uint32_t nc = d < out_cap ? (uint32_t)min<uint64_t>(n, out_cap - d) : 0u;
    const auto rd = __builtin_amdgcn_make_buffer_rsrc((void*)(out + d), 0, nc * 4, SO_RSRC_FLAGS);
#pragma unroll
    for (int r = 0; r < SC_VT; r++)  // (wave-uniform: a tile's empty slots issue nothing)
      if (r * 64 < (int)n) __builtin_amdgcn_raw_buffer_store_b32(Dq[r], rd, (lane + r * 64) * 4, 0, 0);
    const bool ok = tile + SC_DEPTH * stride < ntiles;
    n = ok ? field(Mq, 4) : 0;
    d = ok ? dst_of(Mq) : 0;
    fetch(Mq, ok, Dq);
    Mq = meta_load(tile + 2 * SC_DEPTH * stride);
    tile += stride;
    return tile < ntiles;
  };
  for (;;) {
    bool more = true;
#pragma unroll
    for (int q = 0; q < SC_DEPTH; q++)
      if (more) more = step(D[q], M[q], nn[q], dd[q]);
    if (!more) break;
  }
}

// workgroups of a tile walk: enough to fill the CUs several times over (env SYZGPU_SO_GRID for A/B)
static unsigned so_grid(uint64_t tiles) {
  static const unsigned cap = dev_env("SYZGPU_SO_GRID") ? (unsigned)atoi(dev_env("SYZGPU_SO_GRID")) : 16384u;
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(tiles, cap));
}

// out_off[p] = tout[tstart[p]] (a pair without tiles: the next one's start)
__global__ void k_so_pairoff(const uint64_t* tstart, const uint64_t* tout, uint32_t npairs, uint64_t* out_off) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p <= npairs; p += gridDim.x * blockDim.x)
    out_off[p] = tout[tstart[p]];
}

static uint64_t setop_batch_rank(int op, const uint32_t* a, const uint64_t* aoff, uint64_t na, const uint32_t* b,
                                 const uint64_t* boff, uint64_t nb, uint32_t npairs, uint32_t* out, uint64_t out_cap,
                                 uint64_t* out_off_dev, hipStream_t s);

// Device-side batched set op. All pointers device; out_off_dev gets npairs+1 offsets.
// Returns total output length (host), throws on unsorted input / capacity.
uint64_t setop_batch_dev(int op, const uint32_t* a, const uint64_t* aoff, uint64_t na, const uint32_t* b,
                         const uint64_t* boff, uint64_t nb, uint32_t npairs, uint32_t* out, uint64_t out_cap,
                         uint64_t* out_off_dev, hipStream_t s) {
  Context& c = ctx();
  if (dev_env("SYZGPU_SETOP_RANK") && atoi(dev_env("SYZGPU_SETOP_RANK")))
    return setop_batch_rank(op, a, aoff, na, b, boff, nb, npairs, out, out_cap, out_off_dev, s);
  const uint64_t tbound = npairs + (na + nb) / SO_T + 1;
  uint32_t* ntile = c.scratch.get<uint32_t>("so_ntile", npairs + 1);
  uint64_t* tstart = c.scratch.get<uint64_t>("so_tstart", npairs + 2);
  uint32_t* tcnt = c.scratch.get<uint32_t>("so_tcnt", tbound + 1);
  uint64_t* tout = c.scratch.get<uint64_t>("so_tout", tbound + 2);
  int* fl = c.scratch.get<int>("so_fl", 2);
  SYZ_HIP(hipMemsetAsync(fl, 0, 2 * sizeof(int), s));
  uint32_t* tpair = c.scratch.get<uint32_t>("so_tpair", tbound + 1);
  SoDesc* desc = c.scratch.get<SoDesc>("so_desc", tbound + 1);
  k_so_ntiles<<<grid_for(npairs, 256, 4096), 256, 0, s>>>(aoff, boff, npairs, ntile);
  SYZ_LAUNCHED();
  exclusive_scan_u32(ntile, tstart, npairs, s);
  k_so_tpair<<<grid_for(npairs, 256, 4096), 256, 0, s>>>(tstart, npairs, tpair);
  SYZ_LAUNCHED();
  k_so_tdesc<<<grid_for(tbound, 256, 8192), 256, 0, s>>>(a, aoff, b, boff, tstart, tpair, npairs, desc, fl, fl + 1);
  SYZ_LAUNCHED();
  // one merge pass into a gapped image + a compaction (default), or count + scan + a second merge
  // (SYZGPU_SO_TWOPASS=1, for A/B: the merge is VALU-bound, so running it once is what pays)
  static const bool twopass = dev_env("SYZGPU_SO_TWOPASS") && atoi(dev_env("SYZGPU_SO_TWOPASS"));
  uint32_t* gap = twopass ? nullptr : c.scratch.get<uint32_t>("so_gap", na + nb + 1);
  if (twopass) {
    ProfScope ps("setop_count", s, 4 * (na + nb) + 16 * (uint64_t)npairs);
    k_so_tile<SO_COUNT><<<so_grid(tbound), SO_BLOCK, 0, s>>>(op, a, b, desc, tstart + npairs, tcnt, nullptr, nullptr,
                                                              fl, fl + 1);
    SYZ_LAUNCHED();
  } else {
    SYZ_HIP(hipMemsetAsync(tcnt, 0, (tbound + 1) * 4, s));  // the scan runs over the bound
    ProfScope ps("setop_merge", s, 4 * (na + nb) + 16 * (uint64_t)npairs);
    k_so_tile<SO_GAP><<<so_grid(tbound), SO_BLOCK, 0, s>>>(op, a, b, desc, tstart + npairs, tcnt, nullptr, gap, fl,
                                                            fl + 1);
    SYZ_LAUNCHED();
  }
  int* herr = c.pinned.get<int>(4);
  uint64_t* htot = reinterpret_cast<uint64_t*>(herr + 2);
  if (twopass) {
    uint64_t* hnt = c.pinned.get<uint64_t>(2);
    SYZ_HIP(hipMemcpyAsync(hnt, tstart + npairs, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    const uint64_t ntiles = *hnt;
    exclusive_scan_u32(tcnt, tout, ntiles, s);
    k_so_pairoff<<<grid_for(npairs + 1, 256, 4096), 256, 0, s>>>(tstart, tout, npairs, out_off_dev);
    SYZ_LAUNCHED();
    SYZ_HIP(hipMemcpyAsync(herr, fl, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(htot, tout + ntiles, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (herr[1]) fail(SYZGPU_EINVAL, "set operation input is not sorted ascending");
    if (herr[0])  // a repeated value: the multiset rank path
      return setop_batch_rank(op, a, aoff, na, b, boff, nb, npairs, out, out_cap, out_off_dev, s);
    const uint64_t total = *htot;
    if (total > out_cap) fail(SYZGPU_ECAPACITY, "set operation output capacity too small");
    if (ntiles) {
      ProfScope ps("setop_emit", s, 4 * (na + nb) + 4 * total + 8 * (uint64_t)npairs);
      k_so_tile<SO_EMIT><<<so_grid(ntiles), SO_BLOCK, 0, s>>>(op, a, b, desc, tstart + npairs, nullptr, tout, out,
                                                               nullptr, nullptr);
      SYZ_LAUNCHED();
    }
    return total;
  }
  // one pass: the scan over the tile bound (the counts past the last tile were zeroed before the
  // merge), the pair offsets and the compaction (its stores clamped to out_cap) go out without a wait;
  // one read-back of the flags and the total at the end
  exclusive_scan_u32(tcnt, tout, tbound, s);
  k_so_pairoff<<<grid_for(npairs + 1, 256, 4096), 256, 0, s>>>(tstart, tout, npairs, out_off_dev);
  SYZ_LAUNCHED();
  {
    ProfScope ps("setop_compact", s, 0);  // (its bytes, 8 per output, are not known at launch)
    k_so_compact<<<so_grid((tbound + SO_BLOCK / 64 - 1) / (SO_BLOCK / 64)), SO_BLOCK, 0, s>>>(desc, tcnt, tout,
                                                                                           tstart + npairs, gap, out,
                                                                                           out_cap);
    SYZ_LAUNCHED();
  }
  SYZ_HIP(hipMemcpyAsync(herr, fl, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(htot, tout + tbound, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (herr[1]) fail(SYZGPU_EINVAL, "set operation input is not sorted ascending");
  if (herr[0])  // a repeated value: the multiset rank path (rewrites out and the offsets)
    return setop_batch_rank(op, a, aoff, na, b, boff, nb, npairs, out, out_cap, out_off_dev, s);
  const uint64_t total = *htot;
  if (total > out_cap) fail(SYZGPU_ECAPACITY, "set operation output capacity too small");
  return total;
}

// The per-element multiset rank path (any sorted input, repeated values included).
static uint64_t setop_batch_rank(int op, const uint32_t* a, const uint64_t* aoff, uint64_t na, const uint32_t* b,
                         const uint64_t* boff, uint64_t nb, uint32_t npairs, uint32_t* out, uint64_t out_cap,
                         uint64_t* out_off_dev, hipStream_t s) {
  Context& c = ctx();
  uint8_t* keepa = c.scratch.get<uint8_t>("so_keepa", na + 1);
  uint8_t* keepb = c.scratch.get<uint8_t>("so_keepb", nb + 1);
  uint64_t* ka = c.scratch.get<uint64_t>("so_ka", na + 1);
  uint64_t* kb = c.scratch.get<uint64_t>("so_kb", nb + 1);
  uint64_t* plen = c.scratch.get<uint64_t>("so_plen", npairs + 1);
  int* err = c.scratch.get<int>("so_err", 1);
  uint32_t* nsa = c.scratch.get<uint32_t>("so_nsa", npairs + 1);
  uint32_t* nsb = c.scratch.get<uint32_t>("so_nsb", npairs + 1);
  uint64_t* sga = c.scratch.get<uint64_t>("so_sga", npairs + 1);
  uint64_t* sgb = c.scratch.get<uint64_t>("so_sgb", npairs + 1);
  SYZ_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  k_setop_nseg<<<grid_for(npairs, 256, 4096), 256, 0, s>>>(aoff, npairs, nsa);
  SYZ_LAUNCHED();
  k_setop_nseg<<<grid_for(npairs, 256, 4096), 256, 0, s>>>(boff, npairs, nsb);
  SYZ_LAUNCHED();
  exclusive_scan_u32(nsa, sga, npairs, s);
  exclusive_scan_u32(nsb, sgb, npairs, s);
  const uint64_t sega = npairs + na / SO_SEG + 1, segb = npairs + nb / SO_SEG + 1;  // segment bounds
  if (na) {
    k_setop_classify<<<grid_for(sega * 64, 256, 65536), 256, 0, s>>>(op, 0, a, aoff, b, boff, npairs, sga, keepa, err);
    SYZ_LAUNCHED();
  }
  if (nb) {
    k_setop_classify<<<grid_for(segb * 64, 256, 65536), 256, 0, s>>>(op, 1, b, boff, a, aoff, npairs, sgb, keepb, err);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u8(keepa, ka, na, s);
  exclusive_scan_u8(keepb, kb, nb, s);
  k_setop_pairlen<<<grid_for(npairs, 256, 4096), 256, 0, s>>>(aoff, boff, ka, kb, npairs, plen);
  SYZ_LAUNCHED();
  exclusive_scan_u64(plen, out_off_dev, npairs, s);
  int* herr = c.pinned.get<int>(4);
  uint64_t* htot = reinterpret_cast<uint64_t*>(herr + 2);
  SYZ_HIP(hipMemcpyAsync(herr, err, sizeof(int), hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(htot, out_off_dev + npairs, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (*herr) fail(SYZGPU_EINVAL, "set operation input is not sorted ascending");
  const uint64_t total = *htot;
  if (total > out_cap) fail(SYZGPU_ECAPACITY, "set operation output capacity too small");
  if (na) {
    k_setop_scatter<<<grid_for(sega * 64, 256, 65536), 256, 0, s>>>(0, a, aoff, b, boff, npairs, sga, keepa, ka, kb,
                                                                    out_off_dev, out);
    SYZ_LAUNCHED();
  }
  if (nb) {
    k_setop_scatter<<<grid_for(segb * 64, 256, 65536), 256, 0, s>>>(1, b, boff, a, aoff, npairs, sgb, keepb, kb, ka,
                                                                    out_off_dev, out);
    SYZ_LAUNCHED();
  }
  return total;
}

// ---- Canonicalize -------------------------------------------------------------------------------

constexpr int CANON_LDS = 16384;  // PCs sorted in LDS per cover (kCoverSize = 16<<10)
constexpr int CANON_BLOCK = 1024;

// One workgroup per cover of length <= CANON_LDS: bitonic sort in LDS (padded with the sentinel,
// which sorts last and is cut off), then unique with last = sentinel, written back in place.
__global__ __launch_bounds__(CANON_BLOCK) void k_canon_lds(uint32_t* pcs, const uint64_t* off,
                                                           const uint32_t* list, uint32_t nlist,
                                                           uint64_t* out_len) {
  __shared__ uint32_t s[CANON_LDS];
  __shared__ uint32_t red[CANON_BLOCK / 64 + 1];
  for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
    const uint32_t seg = list[li];
    const uint64_t beg = off[seg];
    const uint32_t n = (uint32_t)(off[seg + 1] - beg);
    uint32_t P = 1;
    while (P < n) P <<= 1;
    for (uint32_t i = threadIdx.x; i < P; i += CANON_BLOCK) s[i] = i < n ? pcs[beg + i] : SENT;
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t i = threadIdx.x; i < P; i += CANON_BLOCK) {
          const uint32_t ij = i ^ j;
          if (ij > i) {
            const uint32_t x = s[i], y = s[ij];
            const bool up = (i & k) == 0;
            if ((x > y) == up) {
              s[i] = y;
              s[ij] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    // unique: keep[i] = s[i] != (i ? s[i-1] : SENT); chunked ordered compaction
    uint32_t outp = 0;
    for (uint32_t base = 0; base < n; base += CANON_BLOCK) {
      const uint32_t i = base + threadIdx.x;
      uint32_t v = 0, k = 0;
      if (i < n) {
        v = s[i];
        const uint32_t prev = i ? s[i - 1] : SENT;
        k = v != prev;
      }
      uint32_t tot;
      const uint32_t r = block_excl_scan<CANON_BLOCK>(k, red, &tot);
      if (k) pcs[beg + outp + r] = v;
      outp += tot;
    }
    if (threadIdx.x == 0) out_len[seg] = outp;
    __syncthreads();
  }
}

// Large covers: global bitonic network over a padded copy, one (k, j) step per launch.
__global__ void k_canon_pad(const uint32_t* src, uint64_t n, uint32_t* dst, uint64_t P) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = i < n ? src[i] : SENT;
}
__global__ void k_bitonic_step(uint32_t* s, uint64_t P, uint64_t k, uint64_t j) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t ij = i ^ j;
    if (ij > i) {
      const uint32_t x = s[i], y = s[ij];
      const bool up = (i & k) == 0;
      if ((x > y) == up) {
        s[i] = y;
        s[ij] = x;
      }
    }
  }
}
__global__ void k_unique_flags(const uint32_t* s, uint64_t n, uint8_t* keep) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    keep[i] = s[i] != (i ? s[i - 1] : SENT);
}
__global__ void k_unique_scatter(const uint32_t* s, uint64_t n, const uint8_t* keep, const uint64_t* pos,
                                 uint32_t* dst) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (keep[i]) dst[pos[i]] = s[i];
}
__global__ void k_store_len(const uint64_t* pos, uint64_t n, uint64_t* out_len, uint32_t seg) {
  out_len[seg] = pos[n];
}

// ---- Canonicalize on a device-resident CSR (no host copy of the offsets) --------------------------
// Covers are classed on the device by length (k_canon_class): <= 1024 PCs take one wave each, in
// registers (k_canon_net), <= 16384 (kCoverSize) a workgroup of register-sorted 1024-slot chunks merged
// through LDS (k_canon_mrg), <= 32768 (raw kcov output with repeats) a 1024-thread LDS bitonic sort with
// 128 KB of LDS (k_canon_cls); longer ones go through the global network one by one.
// After the sort: unique with last = sentinel and the in-place store of the kept prefix
// (cover.go:28-40), the new length to out_len.
template <uint32_t PMAX, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_canon_cls(uint32_t* pcs, const uint64_t* off, const uint32_t* list,
                                                     const uint32_t* nlist_dev, uint64_t* out_len) {
  __shared__ uint32_t sh[PMAX];
  __shared__ uint32_t red[BLOCK / 64 + 1];
  const uint32_t nlist = *nlist_dev;
  for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
    const uint32_t seg = list[li];
    const uint64_t beg = off[seg];
    const uint32_t n = (uint32_t)(off[seg + 1] - beg);
    uint32_t P = 64;
    while (P < n) P <<= 1;
    for (uint32_t i = threadIdx.x; i < P; i += BLOCK) sh[i] = i < n ? pcs[beg + i] : SENT;
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        // one compare-exchange per pair (i, i ^ j), i with bit j clear: P / 2 of them
        for (uint32_t t = threadIdx.x; t < P / 2; t += BLOCK) {
          const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
          const uint32_t ij = i | j;
          const uint32_t x = sh[i], y = sh[ij];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            sh[i] = y;
            sh[ij] = x;
          }
        }
        __syncthreads();
      }
    }
    uint32_t outp = 0;
    for (uint32_t base = 0; base < n; base += BLOCK) {
      const uint32_t i = base + threadIdx.x;
      uint32_t v = 0, kk = 0;
      if (i < n) {
        v = sh[i];
        kk = v != (i ? sh[i - 1] : SENT);
      }
      uint32_t tot;
      const uint32_t r = block_excl_scan<BLOCK>(kk, red, &tot);
      if (kk) pcs[beg + outp + r] = v;
      outp += tot;
    }
    if (threadIdx.x == 0) out_len[seg] = outp;
    __syncthreads();
  }
}

// One WAVE per cover of <= 64 R PCs, the cover in registers in BLOCKED order (lane l holds elements
// l R .. l R + R - 1): a bitonic network over 64 R slots (the class's covers are longer than 32 R, so at
// most half of it is padding), fully unrolled so every compare-exchange's direction is a compile-time
// or per-lane constant. Distances below R are register pairs (min/max), the others lane exchanges by
// DPP (xor 1, 2), ds_swizzle (xor 4..16) or v_permlane32_swap (xor 32): no LDS traffic, no barriers,
// no exec-mask loops. Then unique (cover.go:28-40: a PC is kept iff it differs from the one before,
// the first against the sentinel) and the kept PCs stored in place after a wave scan of the per-lane
// counts. Four independent waves per workgroup walk the class list.
template <int M>
__device__ __forceinline__ uint32_t xor_lane(uint32_t x) {
  if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
  else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // 2,3,0,1
  else if constexpr (M == 3) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x1B, 0xF, 0xF, false);  // 3,2,1,0
  else if constexpr (M == 7) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  else if constexpr (M == 15) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);  // row_mirror
  else if constexpr (M < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (M << 10));  // 4, 8, 16, 31
  else {  // 32, 63: the halves swapped (whichever way the two results come back, their xor with x is the
          // other half's value), then for 63 the mirror inside each half
    const auto h = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    const uint32_t y = h[0] ^ h[1] ^ x;
    if constexpr (M == 63) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)y, 0x1F | (31 << 10));
    else return y;
  }
}

// The bitonic network in its direction-free form: the first stage of merge K pairs element e with
// e ^ (K - 1) (the mirror), the later ones with e ^ J, and every comparator keeps the minimum at the
// lower index. Pairs inside a lane's R registers are plain min/max; across lanes each lane keeps the
// min or the max by one lane bit. Compile-time recursion (not unrolled loops), so every exchange is
// resolved at compile time however long the network is.
template <int R, int J>
__device__ __forceinline__ void cn_half(uint32_t (&x)[R], unsigned lane) {
  if constexpr (J > 0) {
    if constexpr (J < R) {  // register pairs (r, r | J)
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (r & J) continue;
        const uint32_t lo = min(x[r], x[r | J]), hi = max(x[r], x[r | J]);
        x[r] = lo;
        x[r | J] = hi;
      }
    } else {  // lane pairs (l, l ^ J / R)
      const bool keepmin = ((uint32_t)lane & (uint32_t)(J / R)) == 0;
#pragma unroll
      for (int r = 0; r < R; r++) {
        const uint32_t y = xor_lane<J / R>(x[r]);
        x[r] = keepmin ? min(x[r], y) : max(x[r], y);
      }
    }
    cn_half<R, J / 2>(x, lane);
  }
}

template <int R, int K>
__device__ __forceinline__ void cn_merges(uint32_t (&x)[R], unsigned lane) {
  if constexpr (K <= 64 * R) {
    if constexpr (K <= R) {  // the mirror inside a lane: (r, r ^ (K - 1)) for r with bit K / 2 clear
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (r & (K >> 1)) continue;
        const int q = r ^ (K - 1);
        const uint32_t lo = min(x[r], x[q]), hi = max(x[r], x[q]);
        x[r] = lo;
        x[q] = hi;
      }
    } else {  // the mirror across lanes: lane ^ (K / R - 1), register R - 1 - r
      const bool keepmin = ((uint32_t)lane & (uint32_t)(K / (2 * R))) == 0;
      uint32_t y[R];
#pragma unroll
      for (int r = 0; r < R; r++) y[r] = xor_lane<K / R - 1>(x[R - 1 - r]);
#pragma unroll
      for (int r = 0; r < R; r++) x[r] = keepmin ? min(x[r], y[r]) : max(x[r], y[r]);
    }
    cn_half<R, K / 4>(x, lane);
    cn_merges<R, 2 * K>(x, lane);
  }
}

template <int R>
__device__ __forceinline__ void canon_net(uint32_t (&x)[R], unsigned lane) {
  cn_merges<R, 2>(x, lane);
}

template <int R>
__global__ __launch_bounds__(256) void k_canon_net(uint32_t* pcs, const uint64_t* off, const uint32_t* list,
                                                   const uint32_t* nlist_dev, uint64_t* out_len) {
  const uint32_t nlist = *nlist_dev;
  const unsigned lane = __lane_id();
  const uint32_t waves = gridDim.x * (blockDim.x >> 6);
  for (uint32_t li = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); li < nlist; li += waves) {
    const uint32_t seg = list[li];
    const uint64_t beg = off[seg];
    const uint32_t n = (uint32_t)(off[seg + 1] - beg);
    uint32_t x[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint32_t e = lane * R + r;
      x[r] = e < n ? pcs[beg + e] : SENT;
    }
    canon_net<R>(x, lane);
    const uint32_t pl = (uint32_t)__builtin_amdgcn_mov_dpp((int)x[R - 1], 0x138, 0xF, 0xF, false);  // lane - 1's last
    uint32_t km = 0;  // bit r: element lane R + r is kept
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint32_t prev = r ? x[r > 0 ? r - 1 : 0] : (lane ? pl : SENT);
      km |= (lane * R + r < n && x[r] != prev) ? 1u << r : 0u;
    }
    const uint32_t cnt = (uint32_t)__popc(km);
    const uint32_t incl = wave_incl_scan(cnt);
    uint32_t* dst = pcs + beg + (incl - cnt);
    uint32_t q = 0;
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (km >> r & 1u) dst[q] = x[r];
      q += km >> r & 1u;
    }
    if (lane == 63) out_len[seg] = incl;
  }
}

// One WORKGROUP of P / 1024 waves per cover of P / 2 < n <= P PCs (P = 2048 .. 16384): each wave
// sorts a 1024-slot chunk in registers (canon_net<16>), then log2(P / 1024) rounds of pairwise merges
// through LDS (ping-pong buffers; each thread finds its 16 outputs' start by a merge-path search and
// merges them), the last round's outputs straight into unique and the in-place store. Against the
// all-LDS bitonic network (log2(P) (log2(P) + 1) / 2 barrier-separated stages) this is 55 register
// stages and 2-4 merge rounds.
template <int P>
__global__ __launch_bounds__(P / 16) void k_canon_mrg(uint32_t* pcs, const uint64_t* off, const uint32_t* list,
                                                     const uint32_t* nlist_dev, uint64_t* out_len) {
  constexpr int BLOCK = P / 16, WAVES = BLOCK / 64;
  __shared__ __attribute__((aligned(16))) uint32_t buf[2][P];
  __shared__ uint32_t wl[WAVES];
  __shared__ uint32_t red[WAVES + 1];
  const uint32_t nlist = *nlist_dev;
  const unsigned lane = __lane_id();
  const uint32_t wv = threadIdx.x >> 6, o = threadIdx.x * 16;
  for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
    const uint32_t seg = list[li];
    const uint64_t beg = off[seg];
    const uint32_t n = (uint32_t)(off[seg + 1] - beg);
    uint32_t x[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const uint32_t e = wv * 1024 + lane * 16 + r;
      x[r] = e < n ? pcs[beg + e] : SENT;
    }
    canon_net<16>(x, lane);
    int cur = 0;
#pragma unroll
    for (int r = 0; r < 16; r += 4)
      *reinterpret_cast<uint4*>(&buf[0][o + r]) = make_uint4(x[r], x[r + 1], x[r + 2], x[r + 3]);
    __syncthreads();
#pragma unroll
    for (int sl = 1024; sl < P; sl <<= 1) {
      const uint32_t* src = buf[cur];
      const uint32_t pb = o & ~(2u * sl - 1), d = o - pb;
      const uint32_t* A = src + pb;
      const uint32_t* B = src + pb + sl;
      uint32_t lo = d > (uint32_t)sl ? d - sl : 0u, hi = min(d, (uint32_t)sl);
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (A[mid] <= B[d - mid - 1])
          lo = mid + 1;
        else
          hi = mid;
      }
      uint32_t i = lo, j = d - lo;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const uint32_t a = A[min(i, (uint32_t)sl - 1)], b = B[min(j, (uint32_t)sl - 1)];
        const bool ta = (j >= (uint32_t)sl) | ((i < (uint32_t)sl) & (a <= b));
        x[r] = ta ? a : b;
        i += ta ? 1u : 0u;
        j += ta ? 0u : 1u;
      }
      if (2 * sl < P) {  // not the last round: to the other buffer
        uint32_t* dst = buf[cur ^ 1];
#pragma unroll
        for (int r = 0; r < 16; r += 4)
          *reinterpret_cast<uint4*>(&dst[o + r]) = make_uint4(x[r], x[r + 1], x[r + 2], x[r + 3]);
        __syncthreads();
        cur ^= 1;
      }
    }
    // x = merged elements o .. o + 15; unique against the element before (a lane's / a wave's neighbour)
    if (lane == 63) wl[wv] = x[15];
    __syncthreads();
    const uint32_t pl = (uint32_t)__builtin_amdgcn_mov_dpp((int)x[15], 0x138, 0xF, 0xF, false);
    uint32_t km = 0;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const uint32_t prev = r ? x[r > 0 ? r - 1 : 0] : lane ? pl : wv ? wl[wv > 0 ? wv - 1 : 0] : SENT;
      km |= (o + r < n && x[r] != prev) ? 1u << r : 0u;
    }
    uint32_t tot;
    const uint32_t pre = block_excl_scan<BLOCK>((uint32_t)__popc(km), red, &tot);
    uint32_t* dstg = pcs + beg + pre;
    uint32_t q = 0;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      if (km >> r & 1u) dstg[q] = x[r];
      q += km >> r & 1u;
    }
    if (threadIdx.x == 0) out_len[seg] = tot;
    __syncthreads();  // wl / buffers reused by the next cover
  }
}

// cls lists: [0..4] <= 64 << c (one wave each, k_canon_net<1 << c>), [5..8] <= 2048 << (c - 5)
// (k_canon_mrg), [9] <= 32768 (k_canon_cls), [10] longer
constexpr int CANON_NCLS = 11;
constexpr int CANON_LDS2 = 32768;  // a 1024-thread workgroup with 128 KB of LDS (raw kcov covers with repeats)
// A workgroup classes CANON_CHUNK covers: wave-aggregated LDS counts, one global reservation per class
// per workgroup (global atomics per wave on nine counters were the kernel's bound), then the list entries.
constexpr int CANON_CHUNK = 4096;
__device__ __forceinline__ int canon_class_of(uint64_t n) {
  return n <= 64 ? 0 : n <= 128 ? 1 : n <= 256 ? 2 : n <= 512 ? 3 : n <= 1024 ? 4 : n <= 2048 ? 5
       : n <= 4096 ? 6 : n <= 8192 ? 7 : n <= 16384 ? 8 : n <= (uint64_t)CANON_LDS2 ? 9 : 10;
}
// The first CANON_PRE = 8 PCs of every cover, eight covers per wave (lane 8 c + e reads PC e of cover
// c: one coalesced load for eight covers): cand[i] = 1 when they increase strictly (a candidate for the
// canonical-cover check, k_canon_sorted), so a raw cover costs the check one 4-byte read per PC of its
// prefix.
constexpr int CANON_PRE = 8;  // lanes per cover: 64 / CANON_PRE covers per load
static_assert(CANON_PRE == 8, "k_canon_prefix's lane groups");
__global__ __launch_bounds__(256) void k_canon_prefix(const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off,
                                                      size_t ncov, uint8_t* __restrict__ cand) {
  const unsigned lane = __lane_id();
  const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
  for (size_t c0 = ((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8; c0 < ncov; c0 += nw * 8) {
    const size_t i = c0 + (lane >> 3);
    const uint32_t e = lane & 7;
    uint64_t b = 0, n = 0;
    if (i < ncov) {
      b = off[i];
      n = off[i + 1] - b;
    }
    const uint32_t x = e < n ? pcs[b + e] : 0u;
    const uint32_t prev = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x138, 0xF, 0xF, false);  // lane - 1
    const bool bad = e > 0 && e < n && prev >= x;
    const uint64_t m = __ballot(bad);
    if (e == 0 && i < ncov) cand[i] = ((m >> (lane & ~7u)) & 0xFFu) == 0;
  }
}

// Classes by length; a cover flagged in cand (its prefix increases) is left to the canonical-cover check
// (k_canon_runs), which lists it in its class only if it fails.
__global__ __launch_bounds__(256) void k_canon_class(const uint64_t* off, size_t ncov, uint32_t* lists, size_t cap,
                                                     uint32_t* cnt, const uint8_t* cand = nullptr) {
  constexpr int NC = CANON_NCLS;
  __shared__ uint32_t lc[NC], lb[NC];
  const unsigned lane = __lane_id();
  for (size_t c0 = (size_t)blockIdx.x * CANON_CHUNK; c0 < ncov; c0 += (size_t)gridDim.x * CANON_CHUNK) {
    if (threadIdx.x < NC) lc[threadIdx.x] = 0;
    __syncthreads();
    constexpr int PER = CANON_CHUNK / 256;
    int cls[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const size_t i = c0 + (size_t)q * blockDim.x + threadIdx.x;
      cls[q] = (i >= ncov || (cand && cand[i])) ? -1 : canon_class_of(off[i + 1] - off[i]);
    }
    for (int pass = 0; pass < 2; pass++) {  // 0: counts; 1: entries at the reserved bases
#pragma unroll
      for (int q = 0; q < PER; q++) {
        const size_t i = c0 + (size_t)q * blockDim.x + threadIdx.x;
        const int c = cls[q];
#pragma unroll
        for (int k = 0; k < NC; k++) {
          const uint64_t m = __ballot(c == k);
          if (!m) continue;
          const unsigned leader = (unsigned)__ffsll((unsigned long long)m) - 1;
          uint32_t base = 0;
          if (lane == leader) base = atomicAdd(&lc[k], (uint32_t)__popcll(m));
          if (pass) {
            base = (uint32_t)__shfl((int)base, (int)leader, 64);
            if (c == k) lists[k * cap + lb[k] + base + (uint32_t)__popcll(m & lanemask_lt())] = (uint32_t)i;
          }
        }
      }
      __syncthreads();
      if (pass == 0 && threadIdx.x < NC) {
        lb[threadIdx.x] = lc[threadIdx.x] ? atomicAdd(&cnt[threadIdx.x], lc[threadIdx.x]) : 0u;
        lc[threadIdx.x] = 0;
      }
      __syncthreads();
    }
  }
}

// Already-canonical covers (the executor's dedup on, executor.cc:565-585 -> fuzzer.go:355): k_canon_prefix
// flags the covers whose first CANON_PRE PCs increase (candidates); here one wave takes 64 consecutive
// covers and streams each maximal run of consecutive candidates as ONE contiguous range of PCs
// (CANON_SCAN_U x 64 PCs a step, lane i of load k at PC 64 k + i), checking every PC against the one
// before it. A break inside the run is either a cover start (the next cover's first PC) or a violation:
// the wave resolves it by a ballot over its covers' start offsets (one per lane) and flags the cover;
// the rest of a flagged cover's breaks in that load are skipped, and a run whose covers are all flagged
// stops streaming (a raw cover with an increasing prefix: one step). A
// strictly increasing cover is its own Canonicalize (sorted, no repeat; a 0xFFFFFFFF can only be its
// last PC, kept unless it is the only one): its length goes to out_len and no network touches it. A
// flagged candidate joins its length class. With every cover a candidate (the sorted batch) the pass is
// one coalesced stream over the PCs.
#ifndef SYZ_CANON_SCAN_U
#define SYZ_CANON_SCAN_U 8
#endif
constexpr int CANON_SCAN_U = SYZ_CANON_SCAN_U;
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
}
__global__ __launch_bounds__(256) void k_canon_runs(const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off,
                                                    size_t ncov, const uint8_t* __restrict__ cand,
                                                    uint32_t* __restrict__ lists, size_t cap, uint32_t* cnt,
                                                    uint64_t* __restrict__ out_len) {
  const unsigned lane = __lane_id();
  const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
  for (size_t c0 = ((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; c0 < ncov; c0 += nw * 64) {
    const size_t c = c0 + lane;
    const bool has = c < ncov;
    const uint64_t ob = off[has ? c : ncov], oe = has ? off[c + 1] : ob;
    const bool ca = has && cand[c];
    uint64_t cm = __ballot(ca);
    uint64_t badm = 0;  // (wave-uniform) covers found not increasing
    while (cm) {
      const int s = __ffsll((unsigned long long)cm) - 1;
      const uint64_t inv = ~cm & (~0ull << s);  // lanes at or after s that are not candidates
      const int e = inv ? __ffsll((unsigned long long)inv) - 1 : 64;
      cm = e >= 64 ? 0 : (cm & (~0ull << e));
      const uint64_t runm = (e >= 64 ? ~0ull : ((1ull << e) - 1)) & (~0ull << s);
      const uint64_t jb = readlane64(ob, s), je = readlane64(oe, e - 1);
      const bool inrun = (int)lane >= s && (int)lane < e;
      const uint32_t* x = pcs;
      uint32_t last = 0;
      for (uint64_t j0 = jb; j0 < je && (badm & runm) != runm; j0 += 64 * CANON_SCAN_U) {
        uint32_t v[CANON_SCAN_U];
#pragma unroll
        for (int k = 0; k < CANON_SCAN_U; k++) {
          const uint64_t j = j0 + 64 * k + lane;
          v[k] = j < je ? x[j] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int k = 0; k < CANON_SCAN_U; k++) {
          const uint64_t j = j0 + 64 * k + lane;
          uint32_t prev = (uint32_t)__builtin_amdgcn_mov_dpp((int)v[k], 0x138, 0xF, 0xF, false);  // lane - 1
          if (lane == 0) prev = k == 0 ? last : (uint32_t)__builtin_amdgcn_readlane((int)v[k - 1], 63);
          uint64_t vm = __ballot(j < je && j > jb && prev >= v[k]);
          while (vm) {  // a cover start or a violation: the cover holding PC jj
            const int bl = __ffsll((unsigned long long)vm) - 1;
            vm &= vm - 1;
            const uint64_t jj = j0 + 64 * k + bl;
            const int L = s + __popcll(__ballot(inrun && ob <= jj)) - 1;
            if (readlane64(ob, L) != jj) {
              badm |= 1ull << L;
              // every cover of the run out of order (a raw cover with an increasing prefix): done
              if ((badm & runm) == runm) break;
              const uint64_t eL = readlane64(oe, L), p0 = j0 + 64 * k;  // cover L's other breaks here
              const uint64_t eb = eL > p0 ? eL - p0 : 0;
              vm &= eb >= 64 ? 0ull : ~((1ull << eb) - 1);
            }
          }
        }
        last = (uint32_t)__builtin_amdgcn_readlane((int)v[CANON_SCAN_U - 1], 63);
      }
    }
    if (ca) {
      const uint64_t n = oe - ob;
      if (!((badm >> lane) & 1ull)) {
        out_len[c] = (n == 1 && pcs[ob] == 0xFFFFFFFFu) ? 0 : n;
      } else {  // not canonical after all: the network of its length class
        const int k = canon_class_of(n);
        lists[(size_t)k * cap + atomicAdd(&cnt[k], 1u)] = (uint32_t)c;
      }
    }
  }
}

// the bounds [off[seg], off[seg + 1]) of the listed covers
static __global__ void k_canon_bigoff(const uint32_t* segs, uint32_t nseg, const uint64_t* off, uint64_t* out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nseg; i += gridDim.x * blockDim.x) {
    out[2 * i] = off[segs[i]];
    out[2 * i + 1] = off[segs[i] + 1];
  }
}

void canonicalize_batch_dev2(uint32_t* pcs, const uint64_t* off, size_t ncov, uint64_t* out_len, hipStream_t s) {
  Context& c = ctx();
  if (ncov == 0) return;
  if (ncov >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "too many covers");
  uint32_t* lists = c.scratch.get<uint32_t>("cd_lists", CANON_NCLS * ncov);
  uint32_t* cnt = c.scratch.get<uint32_t>("cd_cnt", CANON_NCLS);
  SYZ_HIP(hipMemsetAsync(cnt, 0, CANON_NCLS * 4, s));
  // classes by length; covers with an increasing prefix are checked whole first: canonical ones are
  // done (no network), the others join their class before the class kernels run
  uint8_t* cand = c.scratch.get<uint8_t>("cd_cand", ncov + 1);
  {
    ProfScope ps("canon_classes", s, 0);
    k_canon_prefix<<<(unsigned)std::min<size_t>((ncov + 31) / 32, 8192), 256, 0, s>>>(pcs, off, ncov, cand);
    SYZ_LAUNCHED();
    k_canon_class<<<(unsigned)std::min<size_t>((ncov + CANON_CHUNK - 1) / CANON_CHUNK, 2048), 256, 0, s>>>(
        off, ncov, lists, ncov, cnt, cand);
    SYZ_LAUNCHED();
  }
  {
    ProfScope ps("canon_check", s, 0);
    k_canon_runs<<<(unsigned)std::min<size_t>((ncov + 255) / 256, 8192), 256, 0, s>>>(pcs, off, ncov, cand, lists,
                                                                                      ncov, cnt, out_len);
    SYZ_LAUNCHED();
  }
  if (!c.ncu) SYZ_HIP(hipDeviceGetAttribute(&c.ncu, hipDeviceAttributeMultiprocessorCount, c.device));
  const unsigned ncu = (unsigned)std::max(1, c.ncu);
  // the long classes (few covers, long per-cover chains: the 32768 class is one workgroup's bitonic
  // network) on the side stream, started first, beside the short classes' persistent walks
  ensure_side(c);
  ProfScope psn("canon_nets", s, 0);
  SYZ_HIP(hipEventRecord(c.ev_fork, s));
  SYZ_HIP(hipStreamWaitEvent(c.side, c.ev_fork, 0));
  k_canon_cls<CANON_LDS2, CANON_BLOCK><<<ncu, CANON_BLOCK, 0, c.side>>>(pcs, off, lists + 9 * ncov, cnt + 9, out_len);
  SYZ_LAUNCHED();
  k_canon_mrg<16384><<<ncu, 1024, 0, c.side>>>(pcs, off, lists + 8 * ncov, cnt + 8, out_len);
  SYZ_LAUNCHED();
  k_canon_mrg<8192><<<ncu * 2, 512, 0, c.side>>>(pcs, off, lists + 7 * ncov, cnt + 7, out_len);
  SYZ_LAUNCHED();
  SYZ_HIP(hipEventRecord(c.ev_join, c.side));
  k_canon_mrg<4096><<<ncu * 4, 256, 0, s>>>(pcs, off, lists + 6 * ncov, cnt + 6, out_len);
  SYZ_LAUNCHED();
  k_canon_mrg<2048><<<ncu * 8, 128, 0, s>>>(pcs, off, lists + 5 * ncov, cnt + 5, out_len);
  SYZ_LAUNCHED();
  k_canon_net<16><<<ncu * 8, 256, 0, s>>>(pcs, off, lists + 4 * ncov, cnt + 4, out_len);
  SYZ_LAUNCHED();
  k_canon_net<8><<<ncu * 8, 256, 0, s>>>(pcs, off, lists + 3 * ncov, cnt + 3, out_len);
  SYZ_LAUNCHED();
  k_canon_net<4><<<ncu * 8, 256, 0, s>>>(pcs, off, lists + 2 * ncov, cnt + 2, out_len);
  SYZ_LAUNCHED();
  k_canon_net<2><<<ncu * 8, 256, 0, s>>>(pcs, off, lists + ncov, cnt + 1, out_len);
  SYZ_LAUNCHED();
  k_canon_net<1><<<ncu * 8, 256, 0, s>>>(pcs, off, lists, cnt, out_len);
  SYZ_LAUNCHED();
  SYZ_HIP(hipStreamWaitEvent(s, c.ev_join, 0));
  psn.end();
  // longer covers: their list back to the host, then the global network one by one
  uint32_t* h = c.pinned.get<uint32_t>(CANON_NCLS);
  SYZ_HIP(hipMemcpyAsync(h, cnt, CANON_NCLS * 4, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint32_t nbig = h[CANON_NCLS - 1];
  if (!nbig) return;
  // every long cover's bounds in one copy (one host wait for the whole batch, not one per cover)
  uint64_t* dbo = c.scratch.get<uint64_t>("canon_bigoff", 2 * (size_t)nbig);
  k_canon_bigoff<<<grid_for(nbig, 256, 1024), 256, 0, s>>>(lists + (CANON_NCLS - 1) * ncov, nbig, off, dbo);
  SYZ_LAUNCHED();
  std::vector<uint32_t> big(nbig);
  std::vector<uint64_t> hbo(2 * (size_t)nbig);
  SYZ_HIP(hipMemcpyAsync(big.data(), lists + (CANON_NCLS - 1) * ncov, nbig * 4, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hbo.data(), dbo, 16 * (size_t)nbig, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  uint64_t nmax = 0;
  for (uint32_t i = 0; i < nbig; i++) nmax = std::max(nmax, hbo[2 * i + 1] - hbo[2 * i]);
  uint64_t Pmax = 1;
  while (Pmax < nmax) Pmax <<= 1;
  uint32_t* tmp = c.scratch.get<uint32_t>("canon_big", Pmax);
  uint8_t* keep = c.scratch.get<uint8_t>("canon_keep", nmax);
  uint64_t* pos = c.scratch.get<uint64_t>("canon_pos", nmax + 1);
  for (uint32_t i = 0; i < nbig; i++) {
    const uint32_t seg = big[i];
    const uint64_t hoff[2] = {hbo[2 * i], hbo[2 * i + 1]};
    const uint64_t n = hoff[1] - hoff[0];
    uint64_t P = 1;
    while (P < n) P <<= 1;
    const unsigned g = grid_for(P, 256, 65536);
    k_canon_pad<<<g, 256, 0, s>>>(pcs + hoff[0], n, tmp, P);
    SYZ_LAUNCHED();
    for (uint64_t k = 2; k <= P; k <<= 1)
      for (uint64_t j = k >> 1; j > 0; j >>= 1) {
        k_bitonic_step<<<g, 256, 0, s>>>(tmp, P, k, j);
        SYZ_LAUNCHED();
      }
    k_unique_flags<<<grid_for(n, 256, 65536), 256, 0, s>>>(tmp, n, keep);
    SYZ_LAUNCHED();
    exclusive_scan_u8(keep, pos, n, s);
    k_unique_scatter<<<grid_for(n, 256, 65536), 256, 0, s>>>(tmp, n, keep, pos, pcs + hoff[0]);
    SYZ_LAUNCHED();
    k_store_len<<<1, 1, 0, s>>>(pos, n, out_len, seg);
    SYZ_LAUNCHED();
  }
}

// Canonicalize every cover of a device CSR in place. host_off is the host copy of off.
void canonicalize_batch_dev(uint32_t* pcs, const uint64_t* off, const uint64_t* host_off, size_t ncov,
                            uint64_t* out_len, hipStream_t s) {
  Context& c = ctx();
  std::vector<uint32_t> small, big;
  for (size_t i = 0; i < ncov; i++) {
    uint64_t n = host_off[i + 1] - host_off[i];
    if (n <= (uint64_t)CANON_LDS)
      small.push_back((uint32_t)i);
    else
      big.push_back((uint32_t)i);
  }
  if (!small.empty()) {
    uint32_t* dlist = c.scratch.get<uint32_t>("canon_list", small.size());
    SYZ_HIP(hipMemcpyAsync(dlist, small.data(), small.size() * 4, hipMemcpyHostToDevice, s));
    unsigned grid = (unsigned)std::min<size_t>(small.size(), 4096);
    k_canon_lds<<<grid, CANON_BLOCK, 0, s>>>(pcs, off, dlist, (uint32_t)small.size(), out_len);
    SYZ_LAUNCHED();
    SYZ_HIP(hipStreamSynchronize(s));  // dlist reused below / by the next call
  }
  for (uint32_t seg : big) {
    const uint64_t n = host_off[seg + 1] - host_off[seg];
    uint64_t P = 1;
    while (P < n) P <<= 1;
    uint32_t* tmp = c.scratch.get<uint32_t>("canon_big", P);
    uint8_t* keep = c.scratch.get<uint8_t>("canon_keep", n);
    uint64_t* pos = c.scratch.get<uint64_t>("canon_pos", n + 1);
    const unsigned g = grid_for(P, 256, 65536);
    k_canon_pad<<<g, 256, 0, s>>>(pcs + host_off[seg], n, tmp, P);
    SYZ_LAUNCHED();
    for (uint64_t k = 2; k <= P; k <<= 1)
      for (uint64_t j = k >> 1; j > 0; j >>= 1) {
        k_bitonic_step<<<g, 256, 0, s>>>(tmp, P, k, j);
        SYZ_LAUNCHED();
      }
    k_unique_flags<<<grid_for(n, 256, 65536), 256, 0, s>>>(tmp, n, keep);
    SYZ_LAUNCHED();
    exclusive_scan_u8(keep, pos, n, s);
    k_unique_scatter<<<grid_for(n, 256, 65536), 256, 0, s>>>(tmp, n, keep, pos, pcs + host_off[seg]);
    SYZ_LAUNCHED();
    k_store_len<<<1, 1, 0, s>>>(pos, n, out_len, seg);
    SYZ_LAUNCHED();
  }
}

}  // namespace syz

using namespace syz;

namespace {

int pair_op(int op, const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, size_t cap,
            size_t* out_n) {
  SYZ_API_BODY({
    hipStream_t s = C_.stream;
    if ((na && !a) || (nb && !b) || !out_n) fail(SYZGPU_EINVAL, "null pointer");
    uint32_t* da = C_.scratch.get<uint32_t>("po_a", na + 1);
    uint32_t* db = C_.scratch.get<uint32_t>("po_b", nb + 1);
    uint64_t* doff = C_.scratch.get<uint64_t>("po_off", 4);
    uint32_t* dout = C_.scratch.get<uint32_t>("po_out", na + nb + 1);
    uint64_t* doo = C_.scratch.get<uint64_t>("po_oo", 2);
    uint64_t hoff[4] = {0, (uint64_t)na, 0, (uint64_t)nb};
    if (na) SYZ_HIP(hipMemcpyAsync(da, a, na * 4, hipMemcpyHostToDevice, s));
    if (nb) SYZ_HIP(hipMemcpyAsync(db, b, nb * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(doff, hoff, sizeof(hoff), hipMemcpyHostToDevice, s));
    uint64_t tot = setop_batch_dev(op, da, doff, na, db, doff + 2, nb, 1, dout, na + nb, doo, s);
    if (tot > cap) fail(SYZGPU_ECAPACITY, "output capacity too small");
    if (tot) SYZ_HIP(hipMemcpyAsync(out, dout, tot * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    *out_n = tot;
  })
}

}  // namespace

extern "C" {

int syzgpu_difference(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, size_t cap,
                      size_t* out_n) {
  return pair_op(SYZGPU_DIFFERENCE, a, na, b, nb, out, cap, out_n);
}
int syzgpu_symmetric_difference(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out,
                                size_t cap, size_t* out_n) {
  return pair_op(SYZGPU_SYMMETRIC_DIFFERENCE, a, na, b, nb, out, cap, out_n);
}
int syzgpu_union(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, size_t cap,
                 size_t* out_n) {
  return pair_op(SYZGPU_UNION, a, na, b, nb, out, cap, out_n);
}
int syzgpu_intersection(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, size_t cap,
                        size_t* out_n) {
  return pair_op(SYZGPU_INTERSECTION, a, na, b, nb, out, cap, out_n);
}

int syzgpu_setop_batch(int op, const uint32_t* a, const uint64_t* a_off, const uint32_t* b, const uint64_t* b_off,
                       size_t npairs, uint32_t* out, size_t out_cap, uint64_t* out_off) {
  SYZ_API_BODY({
    if (op < 0 || op > 3) fail(SYZGPU_EINVAL, "bad set operation");
    if (!a_off || !b_off || !out_off) fail(SYZGPU_EINVAL, "null pointer");
    if (npairs == 0) {
      out_off[0] = 0;
      return SYZGPU_OK;
    }
    hipStream_t s = C_.stream;
    const uint64_t na = a_off[npairs], nb = b_off[npairs];
    if (a_off[0] != 0 || b_off[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
    uint32_t* da = C_.scratch.get<uint32_t>("sb_a", na + 1);
    uint32_t* db = C_.scratch.get<uint32_t>("sb_b", nb + 1);
    uint64_t* dao = C_.scratch.get<uint64_t>("sb_ao", npairs + 1);
    uint64_t* dbo = C_.scratch.get<uint64_t>("sb_bo", npairs + 1);
    uint64_t* doo = C_.scratch.get<uint64_t>("sb_oo", npairs + 1);
    uint64_t cap_needed = 0;
    switch (op) {
      case SYZGPU_DIFFERENCE: cap_needed = na; break;
      case SYZGPU_INTERSECTION: cap_needed = std::min(na, nb); break;
      default: cap_needed = na + nb;
    }
    uint32_t* dout = C_.scratch.get<uint32_t>("sb_out", cap_needed + 1);
    if (na) SYZ_HIP(hipMemcpyAsync(da, a, na * 4, hipMemcpyHostToDevice, s));
    if (nb) SYZ_HIP(hipMemcpyAsync(db, b, nb * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(dao, a_off, (npairs + 1) * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(dbo, b_off, (npairs + 1) * 8, hipMemcpyHostToDevice, s));
    uint64_t tot = setop_batch_dev(op, da, dao, na, db, dbo, nb, (uint32_t)npairs, dout, cap_needed, doo, s);
    if (tot > out_cap) fail(SYZGPU_ECAPACITY, "output capacity too small");
    if (tot) SYZ_HIP(hipMemcpyAsync(out, dout, tot * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(out_off, doo, (npairs + 1) * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_setop_batch_dev(int op, const uint32_t* a, const uint64_t* a_off, uint64_t na, const uint32_t* b,
                           const uint64_t* b_off, uint64_t nb, size_t npairs, uint32_t* out, size_t out_cap,
                           uint64_t* out_off, void* stream, uint64_t* total) {
  SYZ_API_BODY({
    if (op < 0 || op > 3) fail(SYZGPU_EINVAL, "bad set operation");
    if (!a_off || !b_off || !out_off || (na && !a) || (nb && !b)) fail(SYZGPU_EINVAL, "null pointer");
    if (npairs >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "too many pairs");
    hipStream_t s = (hipStream_t)stream;
    uint64_t tot = 0;
    if (npairs == 0) {
      SYZ_HIP(hipMemsetAsync(out_off, 0, 8, s));
      SYZ_HIP(hipStreamSynchronize(s));
    } else {
      tot = setop_batch_dev(op, a, a_off, na, b, b_off, nb, (uint32_t)npairs, out, out_cap, out_off, s);
      SYZ_HIP(hipStreamSynchronize(s));
    }
    if (total) *total = tot;
  })
}

int syzgpu_canonicalize_batch(uint32_t* pcs, const uint64_t* off, size_t ncov, uint64_t* out_len) {
  SYZ_API_BODY({
    if (!off || !out_len) fail(SYZGPU_EINVAL, "null pointer");
    if (ncov == 0) return SYZGPU_OK;
    hipStream_t s = C_.stream;
    const uint64_t n = off[ncov];
    uint32_t* dp = C_.scratch.get<uint32_t>("cb_pcs", n + 1);
    uint64_t* doff = C_.scratch.get<uint64_t>("cb_off", ncov + 1);
    uint64_t* dlen = C_.scratch.get<uint64_t>("cb_len", ncov + 1);
    if (n) SYZ_HIP(hipMemcpyAsync(dp, pcs, n * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(doff, off, (ncov + 1) * 8, hipMemcpyHostToDevice, s));
    canonicalize_batch_dev(dp, doff, off, ncov, dlen, s);
    if (n) SYZ_HIP(hipMemcpyAsync(pcs, dp, n * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(out_len, dlen, ncov * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_canonicalize_batch_dev(uint32_t* pcs, const uint64_t* off, size_t ncov, uint64_t* out_len, void* stream) {
  SYZ_API_BODY({
    if (!off || !out_len || (ncov && !pcs)) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = (hipStream_t)stream;
    canonicalize_batch_dev2(pcs, off, ncov, out_len, s);
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_canonicalize(uint32_t* cov, size_t n, size_t* out_n) {
  if (!out_n || (n && !cov)) return SYZGPU_EINVAL;
  if (n == 0) {
    *out_n = 0;
    return SYZGPU_OK;
  }
  uint64_t off[2] = {0, (uint64_t)n};
  uint64_t len = 0;
  int rc = syzgpu_canonicalize_batch(cov, off, 1, &len);
  if (rc == SYZGPU_OK) *out_n = (size_t)len;
  return rc;
}

}  // extern "C"

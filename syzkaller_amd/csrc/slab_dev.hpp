// Slab form of the raw Minimize pipeline's transpose (P) and window walk (M): the covers are read from
// HBM once.
//
// A SLAB is up to SL_TILES = 256 tiles of one call group's members (a tile = <= 64 consecutive PCs of
// one member's sorted cover), i.e. <= 16K PCs, cut from the group's member sequence (partition order)
// in blocks of at most SL_MEMB (and 2^(32 - S)) members so a member's tag fits the element. One
// workgroup per slab, ONE pass (the whole slab is staged in LDS):
//   * member table in LDS (in the staging buffer's space), each lane resolves one tile of its wave
//     (address, count, tag) by a search; the wave's 32 tiles are loaded with wave-uniform (scalar)
//     addresses, all of them in flight;
//   * window histogram by LDS atomics, an exclusive scan -> padded window starts inside the slab;
//   * one returning LDS atomic per element for its place in the staging buffer, the padding slots
//     filled, and the slab leaves as one contiguous run of 16-byte stores;
//   * the window starts go out WINDOW-MAJOR per call group: D[dbase + w * stride + j] = element offset
//     (from the group's first element) of window w of the group's slab j, so M reads, for its window,
//     two contiguous rows (starts, and the next window's starts = ends).
// Round 4's form (512-tile slabs through a 16K-element buffer in up to three passes, each pass walking
// every tile again) took 1.27 ms against this form's 1.13 ms at config 4 (serialized).
// M (for_slab_window) then walks one run per slab: a window's runs are ~SL_TILES * 64 / W elements long.
#pragma once
#include <atomic>

#include "panels_dev.hpp"
#include "scan.hpp"

namespace syz {

// Diagnostic build only (-DSYZ_SMIN_STATS, tools/smin_stats.py): where a direct-window M workgroup's cycles
// go. [0] workgroups [1] cycles [2] table init [3] walk [4] emit [5] batches [6] element windows
// [7] wave-0 steps [8] batch set-up cycles (scan, run maps) [9] step-loop cycles [10] vectors [11] runs
// P's phases in the same build: g_sl_stats [0] slabs [1] cycles [2] member table + tile resolution
// [3] tile loads waited + histogram [4] scan + D rows [5] placement [6] padding [7] stores
#ifdef SYZ_SMIN_STATS
static __device__ unsigned long long g_sm_stats[16];
static __device__ unsigned long long g_sl_stats[8];
#define SL_STAT_ADD(i, v) \
  do {                    \
    if (threadIdx.x == 0) atomicAdd(&g_sl_stats[i], (unsigned long long)(v)); \
  } while (0)
#define SM_STAT_ADD(i, v) \
  do {                    \
    if (threadIdx.x == 0) atomicAdd(&g_sm_stats[i], (unsigned long long)(v)); \
  } while (0)
#define SM_T() __builtin_amdgcn_s_memtime()
#else
#define SM_STAT_ADD(i, v)
#define SL_STAT_ADD(i, v)
#define SM_T() 0ull
#endif

// (SL_BLOCK, SL_TPW, SL_TILES, SL_MEMB: plan_host.hpp)
static_assert(SL_TPW <= 64, "a wave's tile table is one register per lane");
constexpr uint32_t SL_NONE = 0xFFFFFFFFu;  // a padding slot: no element (no member has the all-ones tag)

// the value of lane - 1 (DPP wave_shr:1, a VALU op: shuffles through LDS would keep 64 tiles' results
// in flight in registers)
__device__ __forceinline__ uint32_t lane_prev(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x138, 0xF, 0xF, false);
}

// Once-read streams with the non-temporal cache policy, so they do not push the data that is re-read
// (the Go sort's keys, M's rank array and D rows) out of L2: P's cover loads and element stores
// (SYZ_SL_NTL / SYZ_SL_NTS, on: `k_slab` 1.03 -> 1.00 ms alone, step 2.54-2.55 -> 2.52 ms); M's element
// loads (SYZ_M_NT, off: M direct 0.96 -> 1.01 ms, step 2.61 ms), profiles/r06_ab/r06_nt_pm.log
#ifndef SYZ_SL_NTL
#define SYZ_SL_NTL 1
#endif
#ifndef SYZ_SL_NTS
#define SYZ_SL_NTS 1
#endif
#ifndef SYZ_M_NT
#define SYZ_M_NT 0
#endif
typedef unsigned syz_v4u __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint32_t ld_once(const uint32_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ uint4 ld_once4(const uint4* p) {
  if constexpr (NT) {
    const syz_v4u v = __builtin_nontemporal_load(reinterpret_cast<const syz_v4u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void st_once4(uint4* p, uint4 x) {
  if constexpr (NT) {
    syz_v4u v = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(v, reinterpret_cast<syz_v4u*>(p));
  } else {
    *p = x;
  }
}

// ---- slab planning on the device ------------------------------------------------------------------
// tiles per member, and the member lengths with them (one scan gives mpos and tpos)
struct TilesFn {
  const uint32_t* mlen;
  __device__ void operator()(size_t m, uint64_t* v) const { v[0] = (mlen[m] + 63) >> 6; }
};
struct LenTilesFn {
  const uint32_t* mlen;
  __device__ void operator()(size_t m, uint64_t* v) const {
    const uint32_t l = mlen[m];
    v[0] = l;
    v[1] = (l + 63) >> 6;
  }
};

// slabs per block of memb members (the scan's input: cstart = its prefix)
struct BlockSlabsFn {
  const uint32_t* bgroup;
  const uint32_t* gblock;
  const uint64_t* gstart;
  const SGroup* sg;
  const uint64_t* tpos;
  __device__ void operator()(size_t b, uint64_t* v) const {
    const uint32_t g = bgroup[b];
    const uint32_t mb_ = sg[g].memb;
    // (clamped: a plan run speculatively on another layout may hold more blocks than the group needs)
    const uint64_t mb = min<uint64_t>(gstart[g] + (uint64_t)(b - gblock[g]) * mb_, gstart[g + 1]);
    const uint64_t me = min<uint64_t>(mb + mb_, gstart[g + 1]);
    v[0] = (tpos[me] - tpos[mb] + SL_TILES - 1) / SL_TILES;
  }
};

// slab c of block b (cstart[b] <= c < cstart[b + 1])
__device__ __forceinline__ PSlab slab_at(uint64_t c, uint32_t b, const uint32_t* bgroup, const uint32_t* gblock,
                                         const uint64_t* gstart, const SGroup* sg, const uint64_t* tpos,
                                         const uint64_t* mpos, const uint64_t* cstart) {
  const uint32_t g = bgroup[b];
  const uint32_t mb_ = sg[g].memb;
  const uint64_t mb = min<uint64_t>(gstart[g] + (uint64_t)(b - gblock[g]) * mb_, gstart[g + 1]);
  const uint64_t me = min<uint64_t>(mb + mb_, gstart[g + 1]);
  const uint64_t T0 = tpos[mb] + (c - cstart[b]) * SL_TILES;
  const uint64_t T1 = min<uint64_t>(T0 + SL_TILES, tpos[me]);
  // the member holding tile T0: the first m with tpos[m + 1] > T0; the one holding T1 - 1 likewise
  const uint64_t m0 = upper_bound_dev<uint64_t>(tpos, mb + 1, me + 1, T0) - 1;
  const uint64_t m1 = upper_bound_dev<uint64_t>(tpos, m0 + 1, me + 1, T1 - 1) - 1;
  const uint64_t pcpos = mpos[m0] + 64 * (T0 - tpos[m0]);  // the slab's first PC in the slices' order
  PSlab s;
  // PCs before it + the padding slots of every slab before it (at most slab_pad(W) each), 4-aligned
  const SGroup gp = sg[g];
  s.elem = (pcpos + gp.xbase + (c - cstart[gblock[g]]) * slab_pad(gp.W) + 3) & ~3ull;
  s.t0 = T0;
  s.m0 = (uint32_t)m0;
  s.nmem = (uint32_t)(m1 - m0 + 1);
  s.nt = (uint32_t)(T1 - T0);
  s.g = g;
  s.j = (uint32_t)(c - cstart[gblock[g]]);
  s.pad = 0;
  return s;
}

// one thread per slab (grid over a bound; cstart[B] = the slabs there are); the first G + 1 threads
// also write gslab[g] = the group's first slab (gslab[G] = all of them) and gebase[g] = its first element
[[maybe_unused]] static __global__ void k_sl_slabs(const uint32_t* bgroup, uint32_t B, const uint32_t* gblock, const uint64_t* gstart,
                                  const SGroup* sg, const uint64_t* tpos, const uint64_t* mpos, const uint64_t* cstart,
                                  uint64_t bound, PSlab* slabs, uint32_t G, uint32_t* gslab, uint64_t* gebase) {
  const uint64_t ns = cstart[B];
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g = i0; g <= G; g += step) {
    const uint32_t b = gblock[g];
    const uint64_t c = cstart[b];
    gslab[g] = (uint32_t)c;
    if (g < G) gebase[g] = c < cstart[gblock[g + 1]] && c < bound ? slab_at(c, b, bgroup, gblock, gstart, sg, tpos, mpos,
                                                                           cstart).elem : 0;
  }
  for (uint64_t c = i0; c < min(ns, bound); c += step) {
    const uint32_t b = (uint32_t)upper_bound_dev<uint64_t>(cstart, 0, B + 1, c) - 1;  // cstart[b] <= c < cstart[b+1]
    slabs[c] = slab_at(c, b, bgroup, gblock, gstart, sg, tpos, mpos, cstart);
  }
}

// ---- P: one slab per workgroup, one pass ------------------------------------------------------------
// (see the file comment). The whole slab (<= 64 SL_TILES elements + 3 W padding slots) is staged in LDS
// (dynamic: slab_lds_bytes(Wmax) for the widest call of the launch), so every element is placed once:
// histogram by LDS atomics, a scan to the padded window starts (D rows), one returning atomic per
// element for its place, the padding slots filled, and the slab leaves as one run of 16-byte stores.
// err bit 1: a PC outside [lo, lo + W << S) (an unsorted cover: the job is redone on exact bounds).
// NOV: the new-coverage check's second source (members with an entry id >= ns.n1 are maxCover tables),
// every list checked strictly increasing as it is read (err 1 for a table, 4 for a cover: lane
// neighbours, and a tile's first PC against the member's PC before it); wtot (optional): per (call,
// window) element totals, added up over the slabs.
__host__ __device__ constexpr uint32_t slab_obuf_words(uint32_t Wmax) { return (64 * SL_TILES + 3 * Wmax + 4 + 3) & ~3u; }
__host__ __device__ constexpr uint32_t slab_hist_words(uint32_t Wmax) { return (Wmax + 1 + 64 + 3) & ~3u; }
__host__ __device__ constexpr size_t slab_lds_bytes(uint32_t Wmax) {
  return 4ull * (slab_obuf_words(Wmax) + 2 * slab_hist_words(Wmax) + 16);
}
static_assert(5 * SL_MEMB + SL_MEMB / 4 <= 64 * SL_TILES, "the member table lives in the staging buffer's space");

#ifndef SYZ_SL_RUNS
#define SYZ_SL_RUNS 1
#endif
constexpr bool SL_RUNS = SYZ_SL_RUNS != 0;
#ifndef SYZ_SL_SPW
#define SYZ_SL_SPW 1  // slabs per P workgroup (c, c + grid, ...): fewer workgroups to dispatch
#endif
#ifndef SYZ_SL_PERSIST
#define SYZ_SL_PERSIST 0  // P as a grid of resident workgroups (two per CU) walking the slabs
#endif
#ifndef SYZ_SL_XCDK
// > 0: P's slabs in XCD chunks of this many, chunk k on XCD k mod 8 (blocks b and b + 8 share an XCD):
// consecutive slabs' D words share lines, which then fill in one L2. 16: step 2.487-2.493 against
// 2.521-2.532 ms; 64: 2.491-2.559 ms (profiles/r06_ab/r06_xcd_slab_chunks_pm.log). (All slabs of a launch
// on one XCD each, consecutive, was slower: 2.62 vs 2.54 ms, r06_xcd_slabs_pm.log.)
#define SYZ_SL_XCDK 16
#endif
#ifndef SYZ_SL_NOD
#define SYZ_SL_NOD 0  // timing experiment only (results wrong when 1): P without its D-row stores
#endif
// A wave's lanes with window w, ok: the maximal runs of consecutive ok lanes with one window. head: the
// lane starts a run (len: its length); hd: the head of the lane's run.
struct WinRun {
  bool head;
  uint32_t len, hd;
};
__device__ __forceinline__ WinRun win_run(uint32_t w, bool ok, unsigned lane) {
  const uint32_t wp = lane_prev(w);
  const bool head = ok && (lane == 0 || wp != w);
  const uint64_t hm = __ballot(head), okm = __ballot(ok);
  const uint64_t upto = (2ull << lane) - 1;  // lanes <= this one (lane 63: all)
  const uint64_t ends = (hm | ~okm) & ~upto;  // run boundaries after this lane
  const uint64_t mine = hm & upto;
  WinRun r;
  r.head = head;
  r.len = (ends ? (uint32_t)__builtin_ctzll(ends) : 64u) - lane;
  r.hd = mine ? 63u - (uint32_t)__builtin_clzll(mine) : lane;
  return r;
}

template <int BLOCK, int TPW, bool NOV = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_slab(
    const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off, const uint32_t* __restrict__ members,
    const uint32_t* __restrict__ mlen, const uint64_t* __restrict__ tpos, const uint32_t* __restrict__ sbeg,
    const PSlab* __restrict__ slabs, const uint64_t* nslab, const SGroup* __restrict__ sg,
    const uint64_t* __restrict__ gebase, uint32_t lo, uint32_t* __restrict__ elems, uint32_t* __restrict__ D,
    int* err, uint32_t Wmax, uint64_t ecap, uint32_t* wtot = nullptr, NovSrc ns = NovSrc{}, int cls = 0,
    const int* gate = nullptr) {
  constexpr int WAVES = BLOCK / 64;
  static_assert((uint32_t)TPW * WAVES == SL_TILES, "slab tiles");
  extern __shared__ __align__(16) uint32_t slds[];
  uint32_t* obuf = slds;                                  // the slab's elements, window-major
  uint32_t* hist = obuf + slab_obuf_words(Wmax);          // counts, then cursors; + a dummy slot per lane
  uint32_t* pst = hist + slab_hist_words(Wmax);           // padded window starts
  uint32_t* red = pst + slab_hist_words(Wmax);            // block scan
  // the member table, in the staging buffer's space (dead once the tiles are resolved)
  int32_t* mrel = reinterpret_cast<int32_t*>(obuf);       // member i's tile 0 as a slab tile index (< 0: began earlier)
  uint32_t* mtp = obuf + SL_MEMB;                         // the search keys: mrel clipped to [0, nt]
  uint32_t* mlo = obuf + 2 * SL_MEMB;
  uint32_t* mhi = obuf + 3 * SL_MEMB;
  uint32_t* mln = obuf + 4 * SL_MEMB;
  uint8_t* mtab = reinterpret_cast<uint8_t*>(obuf + 5 * SL_MEMB);  // NOV: member i is a table
  // a step speculated on a plan that does not fit the layout read back (panels.hip k_gpack)
  if (gate && *gate) return;
  const uint64_t nsl = *nslab;
  // one slab per workgroup, or (SYZ_SL_PERSIST) a grid of resident workgroups walking the slabs
#if SYZ_SL_PERSIST
  for (uint64_t c = blockIdx.x; c < nsl; c += gridDim.x) {
#else
  // SYZ_SL_SPW slabs per workgroup, as straight-line copies of the body (a loop spills, r06)
#pragma unroll
  for (uint32_t q_ = 0; q_ < SYZ_SL_SPW; q_++) {
    uint64_t c = (uint64_t)blockIdx.x + (uint64_t)q_ * gridDim.x;
    if (SYZ_SL_XCDK) {  // chunks of SYZ_SL_XCDK consecutive slabs on one XCD, chunk k on XCD k mod 8
      const uint32_t x = blockIdx.x & 7u, r = blockIdx.x >> 3;
      c = ((uint64_t)(r / SYZ_SL_XCDK) * 8u + x) * SYZ_SL_XCDK + r % SYZ_SL_XCDK;
    }
    if (c >= nsl) return;
    if (q_) __syncthreads();  // the staging buffer is free for the next slab
#endif
  [&]() {  // (a `return` below ends this slab)
  const int wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  const PSlab sl = slabs[c];
  const SGroup gp = sg[sl.g];
  // cls 1 / 2: only the slabs of small / big call groups (SGroup.pad bit 0)
  if (cls && (gp.pad & 1u) != (uint32_t)(cls - 1)) return;
  const uint32_t S = gp.S, W = gp.W, nt = sl.nt, nmem = sl.nmem;
  // a plan that does not fit this layout (run speculatively before the layout was read back): the
  // slab's D column, staging or elements (checked at the store) would fall outside their buffers;
  // flagged (err 64) and redone
  if (sl.j >= gp.stride || W > Wmax) {
    if (threadIdx.x == 0) atomicOr(err, 64);
    return;
  }
  [[maybe_unused]] const uint64_t q0 = SM_T();
  for (uint32_t i = threadIdx.x; i < nmem; i += BLOCK) {
    const uint64_t m = (uint64_t)sl.m0 + i;
    const int64_t r = (int64_t)tpos[m] - (int64_t)sl.t0;
    mrel[i] = (int32_t)r;
    mtp[i] = (uint32_t)min<int64_t>(max<int64_t>(r, 0), (int64_t)nt);
    const uint32_t e = members[m];
    const uint32_t* src;
    if constexpr (NOV) {
      src = e >= ns.n1 ? ns.mc + ns.mc_off[e - ns.n1] : pcs + off[e];
      mtab[i] = e >= ns.n1;
    } else {
      src = pcs + off[e] + (sbeg ? sbeg[m] : 0u);
    }
    const uint64_t a = (uint64_t)(uintptr_t)src;
    mlo[i] = (uint32_t)a;
    mhi[i] = (uint32_t)(a >> 32);
    mln[i] = mlen[m];
  }
  for (uint32_t i = threadIdx.x; i < W + 1 + 64; i += BLOCK) hist[i] = 0;
  __syncthreads();
  // lane k of this wave: tile t = wv + WAVES k (its member by a search of the tile prefix)
  uint32_t alo, ahi, cz;
  uint32_t pprev = 0;  // NOV: the PC before the lane's tile in its member (a tile other than the first)
  {
    const uint32_t t = wv + WAVES * lane;
    const uint32_t tt = t < nt ? t : 0u;
    uint32_t a = 0, b = nmem;  // largest i with mtp[i] <= tt
    while (b - a > 1) {
      const uint32_t mid = (a + b) >> 1;
      if (mtp[mid] <= tt)
        a = mid;
      else
        b = mid;
    }
    const uint32_t ti = (uint32_t)((int32_t)tt - mrel[a]);  // tile inside the member
    const uint64_t addr = (((uint64_t)mhi[a] << 32) | mlo[a]) + 256ull * ti;
    alo = (uint32_t)addr;
    ahi = (uint32_t)(addr >> 32);
    const uint32_t cnt = (t < nt && lane < (unsigned)TPW) ? min(64u, mln[a] - 64 * ti) : 0u;
    // count | (not the member's first tile) << 7 | (a table) << 8 | member tag << 9
    uint32_t fl = 0;
    if constexpr (NOV) {
      fl = (ti > 0 ? 0x80u : 0u) | (mtab[a] ? 0x100u : 0u);
      // loaded here, beside the tiles' loads, so the order check below waits for none of them one by one
      if (ti > 0 && cnt) pprev = reinterpret_cast<const uint32_t*>((uintptr_t)addr)[-1];
    }
    cz = cnt | fl | (a << 9);
  }
  [[maybe_unused]] const uint64_t q1 = SM_T();
  // every tile's PCs into registers, all loads in flight (a tile's address is wave-uniform)
  uint32_t v[TPW];
#pragma unroll
  for (int k = 0; k < TPW; k++) {
    const uint32_t z = (uint32_t)__builtin_amdgcn_readlane((int)cz, k);
    const uint64_t base = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)ahi, k) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)alo, k);
    const uint32_t cnt = z & 0x7Fu;
    v[k] = ld_once<SYZ_SL_NTL != 0>(reinterpret_cast<const uint32_t*>((uintptr_t)base) + (lane < cnt ? lane : 0u));
    if ((k & 7) == 7) __builtin_amdgcn_sched_barrier(0);
  }
  int bad = 0;  // err bits this lane saw
  if constexpr (NOV) {
    // strictly increasing: lane neighbours inside a tile; a tile's first PC against the PC before it
#pragma unroll
    for (int k = 0; k < TPW; k++) {
      const uint32_t z = (uint32_t)__builtin_amdgcn_readlane((int)cz, k);
      const uint32_t cnt = z & 0x7Fu;
      const int eb = (z & 0x100u) ? 1 : 4;
      const uint32_t pv = lane_prev(v[k]);
      if (lane > 0 && lane < cnt && pv >= v[k]) bad |= eb;
      if ((z & 0x80u) && lane == 0 && cnt && (uint32_t)__builtin_amdgcn_readlane((int)pprev, k) >= v[k]) bad |= eb;
    }
  }
  // from here on v holds the PC's offset from lo: window = v >> S, offset in it = v & omask
  // window histogram. A tile's PCs are sorted, so its lanes' windows come in runs: one LDS atomic per
  // run (its head lane adds the run's length), not one per element (SYZ_SL_RUNS=0: per element, lanes
  // outside the tile counting into a dummy slot of their own)
  const uint32_t DUMMY = W + 1 + lane;
#pragma unroll
  for (int k = 0; k < TPW; k++) {
    const uint32_t z = (uint32_t)__builtin_amdgcn_readlane((int)cz, k);
    const uint32_t cnt = z & 0x7Fu;
    v[k] -= lo;
    const uint32_t w = v[k] >> S;
    const bool in = lane < cnt;
    // outside the windows: an unsorted cover (Minimize: redone on exact bounds; NOV: out of order)
    bad |= (in && w >= W) ? (NOV ? ((z & 0x100u) ? 1 : 4) : 1) : 0;
    if (SL_RUNS) {
      const WinRun r = win_run(w, in && w < W, lane);
      if (r.head) atomicAdd(&hist[w], r.len);
    } else {
      atomicAdd(&hist[in && w < W ? w : DUMMY], 1u);
    }
    if ((k & 7) == 7) __builtin_amdgcn_sched_barrier(0);
  }
  {
    const uint64_t bm = __ballot(bad != 0);
    if (bm) {
      int all = bad;
#pragma unroll
      for (int dd = 32; dd >= 1; dd >>= 1) all |= __shfl_xor(all, dd, 64);
      if (lane == (unsigned)(__ffsll((unsigned long long)bm) - 1)) atomicOr(err, all);
    }
  }
  __syncthreads();
  [[maybe_unused]] const uint64_t q2 = SM_T();
  if (wtot && gp.wbase != SG_NO_WTOT)
    for (uint32_t i = threadIdx.x; i < W; i += BLOCK)
      if (hist[i]) atomicAdd(&wtot[gp.wbase + i], hist[i]);
  // padded window starts -> cursors (hist), pst, D rows
  uint32_t total;
  {
    uint32_t run = 0;
    const uint64_t dcol = gp.dbase + sl.j;
    const uint32_t erel = (uint32_t)(sl.elem - gebase[sl.g]);
    for (uint32_t b0 = 0; b0 <= W; b0 += BLOCK) {
      const uint32_t i = b0 + threadIdx.x;
      const uint32_t x = i < W ? (hist[i] + 3u) & ~3u : 0u;  // runs padded to 16 bytes (M's vectors)
      uint32_t tot;
      const uint32_t pre = block_excl_scan<BLOCK>(x, red, &tot) + run;
      if (i <= W) {
        hist[i] = pre;
        pst[i] = pre;
        if (!SYZ_SL_NOD) D[dcol + (uint64_t)i * gp.stride] = erel + pre;
      }
      run += tot;
    }
    total = run;
  }
  __syncthreads();
  [[maybe_unused]] const uint64_t q3 = SM_T();
  // each element's place from its window's cursor (lanes outside the tile or the windows issue nothing)
  const uint32_t omask = (1u << S) - 1;
  {
    constexpr int PB = 8;
#pragma unroll
    for (int k0 = 0; k0 < TPW; k0 += PB) {
      uint32_t pos[PB], el[PB];
      bool ok[PB];
#pragma unroll
      for (int q = 0; q < PB; q++) {
        const int kk = k0 + q;
        const uint32_t z = (uint32_t)__builtin_amdgcn_readlane((int)cz, kk);
        const uint32_t d = v[kk], w = d >> S;
        ok[q] = lane < (z & 0x7Fu) && w < W;
        el[q] = (d & omask) | ((z >> 9) << S);
        pos[q] = 0;
        if (SL_RUNS) {  // the run's head takes the run's places; its lanes follow it
          const WinRun r = win_run(w, ok[q], lane);
          const uint32_t b = r.head ? atomicAdd(&hist[w], r.len) : 0u;
          pos[q] = (uint32_t)__shfl((int)b, (int)r.hd, 64) + (lane - r.hd);
        } else if (ok[q]) {
          pos[q] = atomicAdd(&hist[w], 1u);
        }
      }
#pragma unroll
      for (int q = 0; q < PB; q++)
        if (ok[q]) obuf[pos[q]] = el[q];
    }
  }
  __syncthreads();
  [[maybe_unused]] const uint64_t q4 = SM_T();
  // the padding slots of each run hold the no-element value: [cursor, next padded start)
  for (uint32_t i = threadIdx.x; i < W; i += BLOCK)
    for (uint32_t e = hist[i]; e < pst[i + 1]; e++) obuf[e] = SL_NONE;
  __syncthreads();
  [[maybe_unused]] const uint64_t q5 = SM_T();
  // the slab leaves as one run of 16-byte stores (sl.elem and total are multiples of 4)
  if (sl.elem + total > ecap) {
    if (threadIdx.x == 0) atomicOr(err, 64);
    return;
  }
  {
    uint4* g4 = reinterpret_cast<uint4*>(elems + sl.elem);
    const uint4* o4 = reinterpret_cast<const uint4*>(obuf);
    for (uint32_t q = threadIdx.x; q < total / 4; q += BLOCK) st_once4<SYZ_SL_NTS != 0>(g4 + q, o4[q]);
  }
  [[maybe_unused]] const uint64_t q6 = SM_T();
  SL_STAT_ADD(0, 1);
  SL_STAT_ADD(1, q6 - q0);
  SL_STAT_ADD(2, q1 - q0);
  SL_STAT_ADD(3, q2 - q1);
  SL_STAT_ADD(4, q3 - q2);
  SL_STAT_ADD(5, q4 - q3);
  SL_STAT_ADD(6, q5 - q4);
  SL_STAT_ADD(7, q6 - q5);
  }();
#if SYZ_SL_PERSIST
  __syncthreads();  // the staging buffer is free for the next slab
#endif
  }
}

// P's launch: one workgroup per slab (a bound; slabs past nslab return), the staging sized for the
// launch's widest call (the attribute raised once per instantiation for the largest size asked)
template <bool NOV>
inline void launch_slab(uint64_t nslabs, uint32_t Wmax, hipStream_t s, const uint32_t* pcs, const uint64_t* off,
                        const uint32_t* members, const uint32_t* mlen, const uint64_t* tpos, const uint32_t* sbeg,
                        const PSlab* slabs, const uint64_t* nslab, const SGroup* sg, const uint64_t* gebase,
                        uint32_t lo, uint32_t* elems, uint64_t ecap, uint32_t* D, int* err, uint32_t* wtot,
                        NovSrc ns, int cls, const int* gate = nullptr) {
  if (!nslabs) return;
  const size_t bytes = slab_lds_bytes(Wmax);
  // (per device: the attribute is a property of the device's copy of the kernel)
  static std::atomic<size_t> raised[64];
  int dev = 0;
  SYZ_HIP(hipGetDevice(&dev));
  std::atomic<size_t>& rd = raised[dev & 63];
  if (bytes > rd.load()) {
    SYZ_HIP(hipFuncSetAttribute((const void*)k_slab<SL_BLOCK, SL_TPW, NOV>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    size_t cur = rd.load();
    while (bytes > cur && !rd.compare_exchange_weak(cur, bytes)) {
    }
  }
  unsigned grid = (unsigned)((nslabs + SYZ_SL_SPW - 1) / SYZ_SL_SPW);
  if (SYZ_SL_XCDK) grid = (unsigned)((grid + 8u * SYZ_SL_XCDK - 1) / (8u * SYZ_SL_XCDK) * (8u * SYZ_SL_XCDK));
#if SYZ_SL_PERSIST
  {
    int ncu = 0;
    SYZ_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    grid = (unsigned)std::min<uint64_t>(nslabs, 2ull * (uint64_t)std::max(1, ncu));
  }
#endif
  k_slab<SL_BLOCK, SL_TPW, NOV><<<grid, SL_BLOCK, bytes, s>>>(pcs, off, members, mlen, tpos, sbeg, slabs,
                                                                         nslab, sg, gebase, lo, elems, D, err, Wmax,
                                                                         ecap, wtot, ns, cls, gate);
  SYZ_LAUNCHED();
}

// ---- M walk over a window's slab runs ---------------------------------------------------------------
// The runs of (call g, window w): run j = [D[w][j], D[w + 1][j]) from the group's first element (both
// multiples of 4: runs are padded to 16 bytes with SL_NONE), its members from slab j's first member.
// Batches of blockDim runs (one per thread), numbered in 16-byte VECTORS by one workgroup scan; the
// waves stream the concatenation in blocks of 64 vectors (a lane's run: the run holding its block's
// first vector plus a mbcnt of the mask of runs starting inside the block), U blocks in flight per
// wave, one 16-byte load and four elements per lane. f(offset, rank) for every element slot; rank
// RANK_NONE for padding and lanes past the window. IDENT: rank = member position (the new-coverage
// check). scratch: 2 * blockDim + 3 * NBLK words (callers alias it with their emit bitmap); red64: 2
// words per wave. NBLK: blocks per element window of a batch.
template <int U, bool IDENT, uint32_t NBLK = PK_NBLK, class F>
__device__ __forceinline__ void for_slab_window(const PItem it, const SGroup* __restrict__ sg,
                                                const uint32_t* __restrict__ gslab, const uint64_t* __restrict__ gebase,
                                                const uint32_t* __restrict__ D, const PSlab* __restrict__ slabs,
                                                const uint32_t* __restrict__ elems,
                                                const uint32_t* __restrict__ rank_of_member, uint32_t* scratch,
                                                uint64_t* red64, F f) {
  const uint32_t g = it.g, w = it.w;
  const uint32_t c0 = gslab[g], ns = gslab[g + 1] - c0;
  if (ns == 0) return;
  const SGroup p = sg[g];
  const uint32_t S = p.S, omask = (1u << S) - 1;
  const uint32_t* Dw = D + p.dbase + (uint64_t)w * p.stride;
  const uint32_t* Dw1 = Dw + p.stride;
  const uint4* gel4 = reinterpret_cast<const uint4*>(elems + gebase[g]);
  const uint32_t BD = blockDim.x;        // runs per batch: one per thread
  uint32_t* rrel = scratch;              // [BD] vector offset of run k's vector 0 - its prefix
  uint32_t* rmb = scratch + BD;          // [BD] first member of run k's slab
  uint32_t* bstart = scratch + 2 * BD;   // [NBLK] run holding block j's first vector
  uint32_t* bmask = bstart + NBLK;       // [2 NBLK] runs starting inside block j (bit = offset)
  const int nwaves = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  auto load_run = [&](uint32_t j, uint32_t& len, uint32_t& rel, uint32_t& mb) {
    len = rel = mb = 0;
    if (j < ns) {
      const uint32_t a = Dw[j];
      rel = a >> 2;
      len = (Dw1[j] - a) >> 2;
      mb = slabs[c0 + j].m0;
    }
  };
  uint32_t nlen, nrel, nmb;
  load_run(threadIdx.x, nlen, nrel, nmb);
  SM_STAT_ADD(11, ns);
  for (uint32_t rb = 0; rb < ns; rb += BD) {
    [[maybe_unused]] uint64_t tb = SM_T();
    SM_STAT_ADD(5, 1);
    const uint32_t len = nlen, rel = nrel, mb = nmb;
    uint32_t pre, k, T;
    pk_scan(len, reinterpret_cast<uint32_t*>(red64), pre, k, T);
    if (len) {
      rrel[k] = rel - pre;
      rmb[k] = mb;
    }
    load_run(rb + BD + threadIdx.x, nlen, nrel, nmb);
    SM_STAT_ADD(10, T / 4);
    for (uint32_t ew = 0; ew < T; ew += 64 * NBLK) {
      SM_STAT_ADD(6, 1);
      const uint32_t te = min(T, ew + 64 * NBLK);
      for (uint32_t j = threadIdx.x; j < 2 * NBLK; j += blockDim.x) bmask[j] = 0;
      __syncthreads();
      if (len && pre < te && pre + len > ew) {
        const uint32_t a = max(pre, ew) - ew, b = min(pre + len, te) - ew;
        for (uint32_t j = (a + 63) >> 6; (j << 6) < b; j++) bstart[j] = k;
        if (pre >= ew && (pre & 63)) {
          const uint32_t o = pre - ew;
          atomicOr(&bmask[2 * (o >> 6) + ((o >> 5) & 1)], 1u << (o & 31));
        }
      }
      __syncthreads();
      [[maybe_unused]] const uint64_t ts = SM_T();
      SM_STAT_ADD(8, ts - tb);
      const uint32_t nblk = (te - ew + 63) >> 6;
      const uint32_t step = (uint32_t)nwaves * U;
      // a step's runs (LDS) and vector loads; a lane past the window reads its block's first vector
      uint32_t mbr[U], mbn[U];
      bool ok[U], okn[U];
      uint4 ev[U];
      auto prep_load = [&](uint32_t j0, uint32_t* mb_, bool* ok_) {
        uint32_t vi[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t j = j0 + (uint32_t)nwaves * u, jj = min(j, nblk - 1);
          const uint32_t r0 = bstart[jj];
          const uint32_t mlo_ = bmask[2 * jj], mhi_ = bmask[2 * jj + 1];
          const uint32_t slo = (mlo_ >> 1) | (mhi_ << 31), shi = mhi_ >> 1;
          const uint32_t idx = ew + (j << 6) + lane;
          ok_[u] = j < nblk && idx < te;
          const uint32_t r = r0 + __builtin_amdgcn_mbcnt_hi(shi, __builtin_amdgcn_mbcnt_lo(slo, 0u));
          const uint32_t rr = ok_[u] ? r : r0;
          vi[u] = rrel[rr] + (ok_[u] ? idx : ew + (jj << 6));
          mb_[u] = rmb[rr];
        }
#pragma unroll
        for (int u = 0; u < U; u++) ev[u] = ld_once4<SYZ_M_NT != 0>(gel4 + vi[u]);
      };
      if ((uint32_t)wv < nblk) prep_load(wv, mbr, ok);
      for (uint32_t j0 = wv; j0 < nblk; j0 += step) {
        SM_STAT_ADD(7, 1);
        // this step's ranks (gathers) and offsets; then the next step's loads into the same registers
        // (this step's elements are dead by then); then the updates, which wait only for the gathers
        uint32_t R[4 * U], o[4 * U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t q[4] = {ev[u].x, ev[u].y, ev[u].z, ev[u].w};
#pragma unroll
          for (int t = 0; t < 4; t++) {
            const bool val = ok[u] && q[t] != SL_NONE;
            if constexpr (IDENT)
              R[4 * u + t] = val ? mbr[u] + (q[t] >> S) : RANK_NONE;
            else
              R[4 * u + t] = rank_of_member[mbr[u] + (val ? (q[t] >> S) : 0u)];
            o[4 * u + t] = val ? (q[t] & omask) : 0xFFFFFFFFu;
          }
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        const bool more = j0 + step < nblk;  // wave-uniform
        if (more) prep_load(j0 + step, mbn, okn);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 4 * U; k++) f(o[k] & omask, o[k] == 0xFFFFFFFFu ? RANK_NONE : R[k]);
#pragma unroll
        for (int u = 0; u < U; u++) {
          mbr[u] = mbn[u];
          ok[u] = okn[u];
        }
      }
      __syncthreads();
      SM_STAT_ADD(9, SM_T() - ts);
      tb = SM_T();
    }
  }
}

// The same walk with every WAVE on its own runs (the direct tables' form): the window's runs are dealt to
// the waves (run j to wave j mod waves, 64 runs a wave-batch, one per lane), each wave numbers its
// wave-batch's vectors with a DPP scan and builds its run maps in its own LDS slice, then streams its
// vectors in blocks of 64 with U blocks in flight. No workgroup barrier between the table's clear and its
// emit: a wave waiting on its loads or rank gathers leaves the SIMD to the other waves of the workgroup
// (the workgroup form above stops all 16 waves at five barriers per batch of runs, and a batch holds ~3
// load round trips per wave). wsc: WW_WORDS(NBW) words per wave; NBW: blocks per element window of a
// wave-batch. f(offset, rank) as above.
__host__ __device__ constexpr uint32_t ww_words(uint32_t nbw) { return 128 + 3 * nbw; }
template <int U, uint32_t NBW, class F>
__device__ __forceinline__ void for_slab_window_w(const PItem it, const SGroup* __restrict__ sg,
                                                  const uint32_t* __restrict__ gslab, const uint64_t* __restrict__ gebase,
                                                  const uint32_t* __restrict__ D, const PSlab* __restrict__ slabs,
                                                  const uint32_t* __restrict__ elems,
                                                  const uint32_t* __restrict__ rank_of_member, uint32_t* wsc, F f) {
  const uint32_t g = it.g, w = it.w;
  const uint32_t c0 = gslab[g], ns = gslab[g + 1] - c0;
  if (ns == 0) return;
  const SGroup p = sg[g];
  const uint32_t S = p.S, omask = (1u << S) - 1;
  const uint32_t* Dw = D + p.dbase + (uint64_t)w * p.stride;
  const uint32_t* Dw1 = Dw + p.stride;
  const uint4* gel4 = reinterpret_cast<const uint4*>(elems + gebase[g]);
  const uint32_t nwaves = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  uint32_t* rrel = wsc + wv * ww_words(NBW);  // [64] vector offset of run k's vector 0 - its prefix
  uint32_t* rmb = rrel + 64;                  // [64] first member of run k's slab
  uint32_t* bstart = rmb + 64;                // [NBW] run holding block j's first vector
  uint32_t* bmask = bstart + NBW;             // [2 NBW] runs starting inside block j (bit = offset)
  // wave-batch b of this wave: runs wv + nwaves * (64 b + lane)
  auto load_run = [&](uint32_t b, uint32_t& len, uint32_t& rel, uint32_t& mb) {
    len = rel = mb = 0;
    const uint32_t j = wv + nwaves * (64 * b + lane);
    if (j < ns) {
      const uint32_t a = Dw[j];
      rel = a >> 2;
      len = (Dw1[j] - a) >> 2;
      mb = slabs[c0 + j].m0;
    }
  };
  const uint32_t nb = (ns + 64 * nwaves - 1) / (64 * nwaves);  // wave-batches (every wave the same count)
  uint32_t nlen, nrel, nmb;
  load_run(0, nlen, nrel, nmb);
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t len = nlen, rel = nrel, mb = nmb;
    if (b + 1 < nb) load_run(b + 1, nlen, nrel, nmb);  // the next wave-batch's runs in flight
    // this wave's vectors: an exclusive DPP scan of the run lengths; k: non-empty runs before this one
    const uint32_t inc = wave_incl_scan<uint32_t>(len);
    const uint32_t pre = inc - len;
    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    if (T == 0) continue;  // (wave-uniform)
    const uint64_t bal = __ballot(len != 0);
    const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    wave_sync();  // (the previous wave-batch's map reads are done)
    if (len) {
      rrel[k] = rel - pre;
      rmb[k] = mb;
    }
    for (uint32_t ew = 0; ew < T; ew += 64 * NBW) {
      const uint32_t te = min(T, ew + 64 * NBW);
      for (uint32_t j = lane; j < 2 * NBW; j += 64) bmask[j] = 0;
      wave_sync();
      if (len && pre < te && pre + len > ew) {
        const uint32_t a = max(pre, ew) - ew, e = min(pre + len, te) - ew;
        for (uint32_t j = (a + 63) >> 6; (j << 6) < e; j++) bstart[j] = k;
        if (pre >= ew && (pre & 63)) {
          const uint32_t o = pre - ew;
          atomicOr(&bmask[2 * (o >> 6) + ((o >> 5) & 1)], 1u << (o & 31));
        }
      }
      wave_sync();
      const uint32_t nblk = (te - ew + 63) >> 6;
      uint32_t mbr[U], mbn[U];
      bool ok[U], okn[U];
      uint4 ev[U];
      auto prep_load = [&](uint32_t j0, uint32_t* mb_, bool* ok_) {
        uint32_t vi[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t j = j0 + (uint32_t)u, jj = min(j, nblk - 1);
          const uint32_t r0 = bstart[jj];
          const uint32_t mlo_ = bmask[2 * jj], mhi_ = bmask[2 * jj + 1];
          const uint32_t slo = (mlo_ >> 1) | (mhi_ << 31), shi = mhi_ >> 1;
          const uint32_t idx = ew + (j << 6) + lane;
          ok_[u] = j < nblk && idx < te;
          const uint32_t r = r0 + __builtin_amdgcn_mbcnt_hi(shi, __builtin_amdgcn_mbcnt_lo(slo, 0u));
          const uint32_t rr = ok_[u] ? r : r0;
          vi[u] = rrel[rr] + (ok_[u] ? idx : ew + (jj << 6));
          mb_[u] = rmb[rr];
        }
#pragma unroll
        for (int u = 0; u < U; u++) ev[u] = ld_once4<SYZ_M_NT != 0>(gel4 + vi[u]);
      };
      prep_load(0, mbr, ok);
      for (uint32_t j0 = 0; j0 < nblk; j0 += U) {
        uint32_t R[4 * U], o[4 * U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t q[4] = {ev[u].x, ev[u].y, ev[u].z, ev[u].w};
#pragma unroll
          for (int t = 0; t < 4; t++) {
            const bool val = ok[u] && q[t] != SL_NONE;
            R[4 * u + t] = rank_of_member[mbr[u] + (val ? (q[t] >> S) : 0u)];
            o[4 * u + t] = val ? (q[t] & omask) : 0xFFFFFFFFu;
          }
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        const bool more = j0 + U < nblk;  // wave-uniform
        if (more) prep_load(j0 + U, mbn, okn);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4 * U; q++) f(o[q] & omask, o[q] == 0xFFFFFFFFu ? RANK_NONE : R[q]);
#pragma unroll
        for (int u = 0; u < U; u++) {
          mbr[u] = mbn[u];
          ok[u] = okn[u];
        }
      }
    }
  }
}

// elements of one (call, window): the lengths of its slab runs
template <int BLOCK>
__device__ __forceinline__ uint32_t slab_window_count(const PItem it, const SGroup* sg, const uint32_t* gslab,
                                                      const uint32_t* D, uint32_t* red) {
  const SGroup p = sg[it.g];
  const uint32_t ns = gslab[it.g + 1] - gslab[it.g];
  const uint32_t* Dw = D + p.dbase + (uint64_t)it.w * p.stride;
  uint32_t s = 0;
  for (uint32_t j = threadIdx.x; j < ns; j += blockDim.x) s += Dw[j + p.stride] - Dw[j];
  return block_sum<BLOCK>(s, red);
}

}  // namespace syz

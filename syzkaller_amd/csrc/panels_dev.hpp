// Device code shared by the raw-cover pipelines: minimizeCorpus (panels.hip) and the new-coverage
// check on windows (novelty_win.hip): window planning constants, the region form of the transpose
// (k_region, the A/B alternative to slab_dev.hpp's k_slab) with its M walk (for_region), the packed
// walk's scan and the min-table helpers. The default slab pipeline is slab_dev.hpp.
#pragma once
#include "panels.hpp"

namespace syz {

#ifndef SYZ_PCAP
#define SYZ_PCAP 16384
#endif
constexpr uint32_t PCAP = SYZ_PCAP;  // PCs per chunk (the LDS staging buffer of the transpose)
constexpr uint32_t MEMB = 64;     // members per block: a 6-bit member tag in each element
constexpr uint32_t WMAX = 1024;   // windows per call group
#ifndef SYZ_DS
#define SYZ_DS 14
#endif
#ifndef SYZ_PBM_WORDS
#define SYZ_PBM_WORDS 6144
#endif
#ifndef SYZ_DIRECT_RB
#define SYZ_DIRECT_RB 16
#endif
#ifndef SYZ_DIRECT_WPE
#define SYZ_DIRECT_WPE 1
#endif
constexpr uint32_t DS = SYZ_DS;  // direct-mode window bits: a 2^DS-entry u32 min table
constexpr uint32_t PBM_WORDS = SYZ_PBM_WORDS;  // LDS winner bitmap of the direct kernel
constexpr uint32_t SMAX = 26;     // 32 - 6 tag bits
constexpr int PP_BLOCK = 1024;
constexpr int PP_WAVES = PP_BLOCK / 64;
constexpr int PP_U = 4;     // 64-PC tiles per wave in flight in k_part's passes
#ifndef SYZ_HS_BITS
#define SYZ_HS_BITS 13
#endif
constexpr uint32_t HS_BITS = SYZ_HS_BITS;
constexpr uint32_t HS = 1u << HS_BITS;  // open-addressing slots of a sparse-window table (8 B each)
#ifndef SYZ_HCAP
#define SYZ_HCAP 16384
#endif
#ifndef SYZ_HTARGET
#define SYZ_HTARGET 8192
#endif
constexpr uint32_t HCAP = SYZ_HCAP;  // PCs per round of a sparse window: twice the slots, i.e. the table
                                     // fills only if no PC repeats (then the probe limit redoes the
                                     // window in more rounds); a tighter cap reads most windows twice
constexpr uint32_t HPROBE = 128; // a longer probe run means the table is full after all
constexpr uint32_t HBM_WORDS = 2048;  // LDS winner bitmap of the sparse kernel (65536 ranks per pass)
// packed sparse windows (call groups of < 8192 entries): one u32 per slot, offset << 13 | rank in the
// group, 16K slots in the same 64 KB, so twice the PCs per window (half the workgroups)
constexpr uint32_t PK_RBITS = 13;
constexpr uint32_t PSMAX = 32 - PK_RBITS;  // window bits a packed slot holds
constexpr uint32_t PHS_BITS = 14;
constexpr uint32_t PHS = 1u << PHS_BITS;
constexpr uint32_t PHCAP = 2 * PHS;       // PCs per round of a packed window
constexpr uint32_t DENSE = 8192u >> (15 - DS);  // PCs per window (per 32K addresses: 8192) above which a call is direct-mode
constexpr uint32_t HTARGET = SYZ_HTARGET;  // PCs per window a sparse call's window size aims at
constexpr uint32_t PHTARGET = 2 * HTARGET;  // the same for packed windows



// elements the element buffer needs for `pcs` PCs in at most `chunks` chunks (k_chunks' alignment)
inline uint64_t elem_bound(uint64_t pcs, uint64_t chunks) { return pcs + 4 * chunks + 8; }

// ---- blocks of 64 members and chunks of <= PCAP PCs -------------------------------------------------
static __global__ void k_blocks(const uint32_t* bgroup, uint32_t B, const uint32_t* gblock, const uint64_t* gstart,
                         const uint64_t* mpos, uint32_t* nsub) {
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x) {
    const uint32_t g = bgroup[b];
    const uint64_t mb = gstart[g] + (uint64_t)(b - gblock[g]) * MEMB;
    const uint64_t me = min<uint64_t>(mb + MEMB, gstart[g + 1]);
    const uint64_t sl = mpos[me] - mpos[mb];
    nsub[b] = (uint32_t)((sl + PCAP - 1) / PCAP);
  }
}

static __global__ void k_chunks(const uint32_t* bgroup, uint32_t B, const uint32_t* gblock, const uint64_t* gstart,
                         const uint64_t* mpos, const uint64_t* cstart, PChunk* chunks) {
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x) {
    const uint32_t g = bgroup[b];
    const uint64_t mb = gstart[g] + (uint64_t)(b - gblock[g]) * MEMB;
    const uint64_t me = min<uint64_t>(mb + MEMB, gstart[g + 1]);
    const uint64_t base = mpos[mb], sl = mpos[me] - base;
    uint64_t c = cstart[b];
    // a chunk's elements start on a 16-byte boundary (P stores them as 16-byte vectors): chunk c sits
    // at its first PC's position + 4c, rounded up to 4 elements (elem_bound)
    for (uint64_t s = 0; s < sl; s += PCAP, c++)
      chunks[c] = PChunk{(base + s + 4 * c + 3) & ~3ull, (uint32_t)min<uint64_t>(PCAP, sl - s), (uint32_t)mb,
                         (uint32_t)(me - mb), (uint32_t)s, g};
  }
}

// gchunk[g] = first chunk of group g (chunks are group-major); gdesc[g] = its first desc row
static __global__ __launch_bounds__(1024) void k_gchunk(const uint32_t* gblock, uint32_t G, const uint64_t* cstart,
                                                 const PGroup* pg, uint64_t* gchunk, uint64_t* gdesc) {
  __shared__ uint64_t red[1024 / 64 + 1];
  uint64_t run = 0;
  for (uint32_t g0 = 0; g0 <= G; g0 += 1024) {
    const uint32_t g = g0 + threadIdx.x;
    uint64_t rows = 0;
    if (g < G) rows = (cstart[gblock[g + 1]] - cstart[gblock[g]]) * (uint64_t)(pg[g].W + 1);
    uint64_t tot;
    const uint64_t pre = block_excl_scan<1024>(rows, red, &tot);
    if (g <= G) {
      gchunk[g] = cstart[gblock[g]];
      gdesc[g] = run + pre;
    }
    run += tot;
  }
}


constexpr uint32_t TMAX = PCAP / 64 + MEMB;  // tiles per chunk

// ---- runs of equal windows in a tile (the region form's passes) ------------------------------------
// The 64 lanes of a tile hold consecutive PCs of one (sorted) cover, so neighbouring lanes mostly share
// a window; a run's head lane can take the run's slots with one LDS atomic.
struct TileRun {
  uint32_t start, len;
  bool head;
};

// lanes with `valid` (of a tile) and their window w: the maximal runs of equal w between invalid lanes
__device__ __forceinline__ TileRun tile_run(uint32_t w, bool valid, unsigned lane) {
  const uint32_t wp = __shfl_up(w, 1, 64);
  const uint64_t vm = __ballot(valid);
  const bool pv = lane > 0 && ((vm >> (lane - 1)) & 1ull);
  const bool head = valid && (!pv || wp != w);
  const uint64_t hm = __ballot(head);
  const uint64_t le = (2ull << lane) - 1;  // lanes <= this one (all 64 for lane 63)
  TileRun r;
  r.head = head;
  r.start = 63u - (uint32_t)__clzll(hm & le);
  const uint64_t stop = (hm | ~vm) & ~le;
  r.len = (stop ? (uint32_t)__ffsll((unsigned long long)stop) - 1u : 64u) - r.start;
  return r;
}

// The second source of the new-coverage check (novelty_win.hip): members with an entry id >= n1 are
// maxCover tables (mc/mc_off, table e - n1), the others covers; every list must be strictly increasing
// (err 1 for a table, 4 for a cover), which P checks as it reads: lane neighbours in a tile, tile
// neighbours through LDS, and a member's first PC in a chunk against its previous one.
struct NovSrc {
  const uint32_t* mc = nullptr;
  const uint64_t* mc_off = nullptr;
  uint32_t n1 = 0xFFFFFFFFu;
};

// ---- P, region form: every (call group, member segment, window) contiguous in HBM -----------------
// The element buffer is laid out by REGION r = pg[g].rb + s * W + w: all PCs of call group g's member
// segment s (members [s << (32 - S), (s + 1) << (32 - S)) of the group, in partition order) that fall
// into window w, as elements (member - segment base) << S | offset in the window. M then streams a
// region as one contiguous range (no per-chunk runs, no member-block bookkeeping), and an element names
// its member itself, so no pass of P depends on the Go-sort ranks.
//   COUNT     (k_region<.., true>)  every chunk's window histogram as a row of u16 counts (desc layout:
//             gdesc[g] + (c - gchunk[g]) * (W + 1));
//   k_colscan each (group, segment, window) column of counts over the segment's chunks: the chunk's
//             place in its region (colpre, same layout) and the region's total; an exclusive scan of
//             the totals gives every region its start;
//   scatter   (k_region<.., false>) the chunk's PCs again, rewritten window-major through LDS and
//             stored as one contiguous run per window at its place: runs of consecutive chunks land
//             side by side, and no global atomics are taken.
// NOV: the new-coverage check's second source (maxCover tables as members, lists checked strictly
// increasing in the COUNT pass).
template <int BLOCK, int TPW, bool NOV = false, bool COUNT = false>
__global__ __launch_bounds__(BLOCK) void k_region(
    const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off, const uint32_t* __restrict__ members,
    const uint64_t* __restrict__ mpos, const uint32_t* __restrict__ sbeg, const PChunk* chunks,
    uint32_t g0, uint32_t g1, const PGroup* pg, const uint64_t* gstart, const uint64_t* gchunk,
    const uint64_t* gdesc, uint32_t lo, uint16_t* cnt, const uint32_t* colpre, const uint64_t* rstart,
    uint32_t* __restrict__ elems, int* err, NovSrc ns = NovSrc{}, int dbg = 0) {
  constexpr int WAVES = BLOCK / 64;
  static_assert(TMAX <= (uint32_t)(TPW * WAVES), "k_region: tiles per wave");
  __shared__ __align__(16) uint32_t obuf[COUNT ? 1 : PCAP];
  __shared__ uint32_t hist[WMAX + 1];
  __shared__ uint32_t posl[COUNT ? 1 : WMAX];  // the run's place: its region start - the group's first + colpre
  __shared__ uint32_t tpre[MEMB + 1];
  __shared__ uint32_t mlo[MEMB], mhi[MEMB];
  __shared__ uint64_t mraw[MEMB];
  __shared__ uint32_t red[WAVES + 1];
  __shared__ uint4 tinfo[TMAX];
  __shared__ uint32_t tlast[NOV && COUNT ? TMAX : 1];
  __shared__ uint8_t mtab[NOV ? MEMB : 1];
  const uint64_t c = gchunk[g0] + blockIdx.x;  // the chunks of call groups [g0, g1)
  if (c >= gchunk[g1]) return;
  const int wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  const PChunk ch = chunks[c];
  const PGroup gp = pg[ch.g];
  const uint32_t S = gp.S, W = gp.W;
  const uint32_t sb = 32 - S;  // member bits of an element
  const uint64_t mig = ch.mb - gstart[ch.g];  // the chunk's first member inside its group
  const uint32_t rbase = gp.rb + (uint32_t)(mig >> sb) * W;  // region of window 0 of this segment
  const uint32_t mseg0 = (uint32_t)(mig & ((1ull << sb) - 1));
  const uint64_t row = gdesc[ch.g] + (c - gchunk[ch.g]) * (uint64_t)(W + 1);
  if constexpr (!COUNT) {  // the runs' places (used after pass 2; the loads fly meanwhile)
    const uint64_t g0 = rstart[gp.rb];
    for (uint32_t w = threadIdx.x; w < W; w += BLOCK) posl[w] = (uint32_t)(rstart[rbase + w] - g0) + colpre[row + w];
  }
  const uint32_t cb = ch.sub, ce = ch.sub + ch.len;
  int bad = 0;
  if (threadIdx.x < 64) {
    const uint32_t m = threadIdx.x;
    uint32_t nt = 0;
    if (m < ch.nmem) {
      const uint64_t p0 = mpos[ch.mb], a = mpos[ch.mb + m] - p0, b = mpos[ch.mb + m + 1] - p0;
      const uint32_t x = (uint32_t)max<uint64_t>(a, cb), y = (uint32_t)min<uint64_t>(b, ce);
      mlo[m] = x;
      mhi[m] = y;
      const uint32_t e = members[ch.mb + m];
      const uint32_t* src;
      if constexpr (NOV) {
        src = e >= ns.n1 ? ns.mc + ns.mc_off[e - ns.n1] : pcs + off[e];
        mtab[m] = e >= ns.n1;
      } else
        src = pcs + off[e] + (sbeg ? sbeg[ch.mb + m] : 0u);
      mraw[m] = (uint64_t)(uintptr_t)src - a * 4;
      nt = y > x ? (y - x + 63) / 64 : 0;
      if constexpr (NOV) {
        if (x > a && y > x && src[x - a - 1] >= src[x - a]) bad |= e >= ns.n1 ? 1 : 4;
      }
    }
    const uint32_t inc = wave_incl_scan<uint32_t>(nt);
    tpre[m] = inc - nt;
    if (m == 63) tpre[64] = inc;
  }
  for (uint32_t i = threadIdx.x; i <= W; i += BLOCK) hist[i] = 0;
  __syncthreads();
  const uint32_t ntiles = tpre[64];
  for (uint32_t t = threadIdx.x; t < ntiles; t += BLOCK) {
    uint32_t lo_m = 0, hi_m = ch.nmem;  // largest m < nmem with tpre[m] <= t
    while (hi_m - lo_m > 1) {
      const uint32_t mid = (lo_m + hi_m) >> 1;
      if (tpre[mid] <= t)
        lo_m = mid;
      else
        hi_m = mid;
    }
    const uint32_t m = lo_m;
    const uint32_t q0 = mlo[m] + (t - tpre[m]) * 64;
    const uint64_t base = mraw[m] + (uint64_t)q0 * 4;
    uint32_t fl = 0;
    if constexpr (NOV) fl = (mtab[m] ? 1u : 0u) | (t > tpre[m] ? 2u : 0u);
    tinfo[t] = make_uint4((uint32_t)base, (uint32_t)(base >> 32), min(64u, mhi[m] - q0) | (m << 8), fl);
  }
  __syncthreads();
  uint32_t v[TPW];
#pragma unroll
  for (int k = 0; k < TPW; k++) {
    const uint32_t t = wv + WAVES * k;
    v[k] = 0;
    if (t < ntiles) {
      const uint4 ti = tinfo[t];
      if (lane < (ti.z & 0xFFu))
        v[k] = reinterpret_cast<const uint32_t*>((uintptr_t)((((uint64_t)ti.y << 32) | ti.x) + 4ull * lane))[0];
    }
  }
  // timing only (SYZGPU_RG_DBG 16): the loads alone
  if (dbg & 16) {
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < TPW; k++) acc += v[k];
    if (acc == 0x9E3779B9u) err[1] = 1;
    return;
  }
  if constexpr (COUNT) {
    // window histogram: one LDS atomic per PC where the tile's PCs mostly sit in windows of their own
    // (sparse covers), one per run of equal windows otherwise (dense covers: no same-address pile-up)
#pragma unroll
    for (int k = 0; k < TPW; k++) {
      const uint32_t t = wv + WAVES * k;
      if (t >= ntiles) break;  // wave-uniform
      const uint32_t cnt = tinfo[t].z & 0xFFu;
      const uint32_t w = (v[k] - lo) >> S;
      const bool in = lane < cnt;
      if constexpr (NOV) {
        const uint32_t pv = __shfl_up(v[k], 1, 64);
        const uint32_t eb = (tinfo[t].w & 1u) ? 1u : 4u;
        if (in && (w >= W || (lane > 0 && pv >= v[k]))) bad |= eb;
        if (lane + 1 == cnt) tlast[t] = v[k];
      } else {
        if (in && w >= W) bad |= 1;  // outside [lo, hi]: an unsorted cover; redone on exact bounds
      }
      const bool ok = in && w < W;
      const TileRun r = tile_run(w, ok, lane);
      const uint32_t runs = (uint32_t)__popcll(__ballot(r.head)), pcs = (uint32_t)__popcll(__ballot(ok));
      if (2 * runs > pcs) {
        if (ok) atomicAdd(&hist[w], 1u);
      } else if (r.head) {
        atomicAdd(&hist[w], r.len);
      }
    }
  } else {
    // the count pass's histogram of this chunk
    for (uint32_t w = threadIdx.x; w < W; w += BLOCK) hist[w] = cnt[row + w];
  }
  __syncthreads();
  if constexpr (NOV && COUNT) {  // the member's previous tile ends below this tile's first PC
#pragma unroll
    for (int k = 0; k < TPW; k++) {
      const uint32_t t = wv + WAVES * k;
      if (t >= ntiles) break;
      const uint32_t f = tinfo[t].w;
      if (lane == 0 && (f & 2u) && tlast[t - 1] >= v[k]) bad |= (f & 1u) ? 1 : 4;
    }
  }
  if constexpr (COUNT) {
    const uint64_t bm = __ballot(bad != 0);
    if (bm) {
      int all = bad;
#pragma unroll
      for (int dd = 32; dd >= 1; dd >>= 1) all |= __shfl_xor(all, dd, 64);
      if (lane == (unsigned)(__ffsll((unsigned long long)bm) - 1)) atomicOr(err, all);
    }
    for (uint32_t w = threadIdx.x; w < W; w += BLOCK) cnt[row + w] = (uint16_t)hist[w];
  } else {
    // window starts (exclusive scan) -> LDS cursors
    uint32_t run = 0;
    for (uint32_t b0 = 0; b0 <= W; b0 += BLOCK) {
      const uint32_t i = b0 + threadIdx.x;
      const uint32_t x = i < W ? hist[i] : 0;
      uint32_t tot;
      const uint32_t pre = block_excl_scan<BLOCK>(x, red, &tot) + run;
      if (i <= W) hist[i] = pre;
      run += tot;
    }
    __syncthreads();
    if (dbg & 32) return;  // timing only: no staging, no stores
    // element = member in segment << S | offset in window, window-major into obuf: a slot per PC from a
    // returning LDS atomic, or per run (dense covers) broadcast from the run's head
    const uint32_t omask = (1u << S) - 1;
#pragma unroll
    for (int k = 0; k < TPW; k++) {
      const uint32_t t = wv + WAVES * k;
      if (t >= ntiles) break;
      const uint32_t z = tinfo[t].z;
      const uint32_t d = v[k] - lo, w = d >> S;
      const bool in = lane < (z & 0xFFu) && w < W;
      const uint32_t el = (d & omask) | ((mseg0 + (z >> 8)) << S);
      const TileRun r = tile_run(w, in, lane);
      const uint32_t runs = (uint32_t)__popcll(__ballot(r.head)), pcs = (uint32_t)__popcll(__ballot(in));
      if (2 * runs > pcs) {
        if (in) obuf[atomicAdd(&hist[w], 1u)] = el;
      } else {
        uint32_t base = r.head ? atomicAdd(&hist[w], r.len) : 0u;
        base = (uint32_t)__shfl((int)base, (int)r.start, 64);
        if (in) obuf[base + (lane - r.start)] = el;
      }
    }
    __syncthreads();
    if (dbg & 64) return;  // timing only: no stores
    // one contiguous run per window at its place (hist[w] is now window w's end): wave wv takes windows
    // wv, wv + WAVES, ...; 64 of them at a time have their start, length and place read at once, and
    // four runs' first 64 elements are read before their stores
    uint32_t* gel = elems + rstart[gp.rb];
    for (uint32_t j0 = 0; wv + WAVES * j0 < W; j0 += 64) {
      const uint32_t wl = wv + WAVES * (j0 + lane);
      uint32_t a = 0, n = 0, ps = 0;
      if (wl < W) {
        a = wl ? hist[wl - 1] : 0u;
        n = hist[wl] - a;
        ps = posl[wl];
      }
      const uint32_t nj = min(64u, (W - wv + WAVES - 1) / WAVES - j0);
      for (uint32_t j = 0; j < nj; j += 4) {
        uint32_t x[4], aj[4], njj[4], pj[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int jj = (int)min(j + u, 63u);
          aj[u] = (uint32_t)__builtin_amdgcn_readlane((int)a, jj);
          njj[u] = j + u < nj ? (uint32_t)__builtin_amdgcn_readlane((int)n, jj) : 0u;
          pj[u] = (uint32_t)__builtin_amdgcn_readlane((int)ps, jj);
          x[u] = lane < njj[u] ? obuf[aj[u] + lane] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
          if (lane < njj[u]) gel[pj[u] + lane] = x[u];
          for (uint32_t i = lane + 64; i < njj[u]; i += 64) gel[pj[u] + i] = obuf[aj[u] + i];
        }
      }
    }
  }
}

// Region starts of call groups [g0, g1) (one workgroup per group): the group's first element (gel0, its
// place in the element buffer) + the exclusive scan of its regions' totals.
constexpr int RS_BLOCK = 1024;
static __global__ __launch_bounds__(RS_BLOCK) void k_rstart(uint32_t g0, const PGroup* pg, const uint64_t* gstart,
                                                           const uint64_t* gel0, const uint32_t* rtot,
                                                           uint64_t* rstart) {
  __shared__ uint64_t red[RS_BLOCK / 64 + 1];
  const uint32_t g = g0 + blockIdx.x;
  const PGroup gp = pg[g];
  const uint32_t sb = 32 - gp.S;
  const uint64_t ng = gstart[g + 1] - gstart[g];
  const uint32_t nr = (uint32_t)((ng + (1ull << sb) - 1) >> sb) * gp.W;
  uint64_t run = gel0[g];
  for (uint32_t b0 = 0; b0 < nr; b0 += RS_BLOCK) {
    const uint32_t i = b0 + threadIdx.x;
    const uint64_t x = i < nr ? rtot[gp.rb + i] : 0;
    uint64_t tot;
    const uint64_t pre = block_excl_scan<RS_BLOCK>(x, red, &tot) + run;
    if (i < nr) rstart[gp.rb + i] = pre;
    run += tot;
  }
}

// Column scan of the COUNT rows: one workgroup per (group, member segment, 64 windows); lane = window,
// wave k takes the k-th slice of the segment's chunks. colpre[row(c) + w] = PCs of window w in the
// segment's chunks before c; rtot[region] = the column's total.
struct ColItem {
  uint32_t g, seg, w0, pad;
};
constexpr int CS_BLOCK = 1024;
static __global__ __launch_bounds__(CS_BLOCK) void k_colscan(const ColItem* items, const PGroup* pg, const uint64_t* gstart,
                                                      const uint32_t* gblock, const uint64_t* cstart,
                                                      const uint64_t* gchunk, const uint64_t* gdesc,
                                                      const uint16_t* __restrict__ cnt, uint32_t* colpre,
                                                      uint32_t* rtot) {
  constexpr int WAVES = CS_BLOCK / 64;
  __shared__ uint32_t part[WAVES][64];
  const ColItem it = items[blockIdx.x];
  const PGroup gp = pg[it.g];
  const uint32_t W = gp.W, sb = 32 - gp.S;
  const int wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  const uint32_t w = it.w0 + lane;
  // the segment's chunks: those of its blocks (2^sb members = 2^(sb - 6) blocks)
  const uint64_t nbg = gblock[it.g + 1] - gblock[it.g];
  const uint64_t bpseg = 1ull << (sb - 6);
  const uint64_t b0 = gblock[it.g] + min<uint64_t>(nbg, it.seg * bpseg);
  const uint64_t b1 = gblock[it.g] + min<uint64_t>(nbg, (it.seg + 1) * bpseg);
  const uint64_t c0 = cstart[b0], c1 = cstart[b1];
  const uint64_t nch = c1 - c0, per = (nch + WAVES - 1) / WAVES;
  const uint64_t k0 = c0 + min<uint64_t>(nch, per * wv), k1 = c0 + min<uint64_t>(nch, per * (wv + 1));
  const uint64_t rowbase = gdesc[it.g] - gchunk[it.g] * (uint64_t)(W + 1);  // row(c) = rowbase + c * (W + 1)
  const bool on = w < W;
  constexpr int UN = 16;
  uint32_t sum = 0;
  for (uint64_t k = k0; k < k1; k += UN) {
    uint32_t x[UN];
#pragma unroll
    for (int u = 0; u < UN; u++) x[u] = (on && k + u < k1) ? cnt[rowbase + (k + u) * (W + 1) + w] : 0u;
#pragma unroll
    for (int u = 0; u < UN; u++) sum += x[u];
  }
  part[wv][lane] = sum;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
  for (int k = 0; k < WAVES; k++) {
    const uint32_t y = part[k][lane];
    pre += k < wv ? y : 0u;
    tot += y;
  }
  if (wv == 0 && on) rtot[gp.rb + it.seg * W + w] = tot;
  if (!on) return;
  for (uint64_t k = k0; k < k1; k += UN) {
    uint32_t x[UN];
#pragma unroll
    for (int u = 0; u < UN; u++) x[u] = k + u < k1 ? cnt[rowbase + (k + u) * (W + 1) + w] : 0u;
#pragma unroll
    for (int u = 0; u < UN; u++) {
      if (k + u < k1) colpre[rowbase + (k + u) * (W + 1) + w] = pre;
      pre += x[u];
    }
  }
}

// ---- M walk over regions ----------------------------------------------------------------------------
// Every element of (call g, window w): the regions of g's member segments in turn, each one contiguous
// range streamed as 16-byte vectors (from the range's 16-byte-aligned floor; lanes outside the range
// are masked), U vectors per thread in flight; the element's member is the segment base + its high
// bits, its rank a gather from rank_of_member (the members of one chunk's run are 64 consecutive
// entries, so a wave's gathers touch a few lines). f(offset, rank) is called for every element slot of
// every step, with RANK_NONE for slots outside the range. IDENT: the rank is the member's position.
// The next step's vector loads are issued behind this step's rank gathers (two register sets in turn:
// a copy between them would wait for the loads), so a wave waits on its gathers with loads in flight.
template <int U, bool IDENT, class F>
__device__ __forceinline__ void for_region(const PItem it, const PGroup* pg, const uint64_t* gstart,
                                           const uint64_t* rstart, const uint32_t* rtot, const uint32_t* elems,
                                           const uint32_t* __restrict__ rank_of_member, F f) {
  const uint32_t g = it.g, w = it.w;
  const PGroup p = pg[g];
  const uint32_t S = p.S, sb = 32 - S, omask = (1u << S) - 1;
  const uint64_t g0 = gstart[g], ng = gstart[g + 1] - g0;
  const uint32_t nseg = (uint32_t)((ng + (1ull << sb) - 1) >> sb);
  const uint32_t BD = blockDim.x;
  for (uint32_t s = 0; s < nseg; s++) {
    const uint32_t r = p.rb + s * p.W + w;
    const uint64_t a = rstart[r], b = a + rtot[r];
    if (a == b) continue;
    const uint64_t a4 = a & ~3ull;
    const uint32_t lo4 = (uint32_t)(a - a4), hi4 = (uint32_t)(b - a4);  // valid slots [lo4, hi4)
    const uint32_t n4 = (hi4 + 3) >> 2;                                  // vectors
    const uint4* ev = reinterpret_cast<const uint4*>(elems + a4);
    const uint64_t mbase = g0 + ((uint64_t)s << sb);
    const uint32_t* __restrict__ rk = rank_of_member + (IDENT ? 0 : mbase);
    auto load = [&](uint4* x, uint32_t v0) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t v = v0 + (uint32_t)u * BD;
        x[u] = ev[v < n4 ? v : 0];
      }
    };
    // one step: this step's gathers and offsets, then the next step's loads (the elements are dead by
    // then, so the loads can reuse their registers), then the updates
    uint4 en[U];
    load(en, threadIdx.x);
    for (uint32_t v0 = threadIdx.x; v0 < n4; v0 += BD * U) {
      uint32_t R[4 * U], o[4 * U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t q[4] = {en[u].x, en[u].y, en[u].z, en[u].w};
        const uint32_t i0 = 4 * (v0 + (uint32_t)u * BD);
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if constexpr (IDENT)
            R[4 * u + k] = (uint32_t)(mbase + (q[k] >> S));
          else
            R[4 * u + k] = rk[q[k] >> S];
          const uint32_t i = i0 + k;
          // an offset >= 2^S marks a slot outside the range
          o[4 * u + k] = (i >= lo4 && i < hi4) ? (q[k] & omask) : 0xFFFFFFFFu;
        }
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      load(en, v0 + BD * U);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 4 * U; k++) f(o[k] & omask, o[k] == 0xFFFFFFFFu ? RANK_NONE : R[k]);
    }
  }
}

#ifndef SYZ_P3_BLOCK
#define SYZ_P3_BLOCK 512
#endif
constexpr int P3_BLOCK = SYZ_P3_BLOCK;
constexpr int P3_TPW = (int)((TMAX + P3_BLOCK / 64 - 1) / (P3_BLOCK / 64));

// ---- M walk, packed form ------------------------------------------------------------------------------
// A walk with one wave instruction per run leaves lanes idle on short runs and pays per-run bookkeeping
// (profiles/r03_pmin_base: ~0.9 VALU wave instructions per element). Here the workgroup takes up to PK_RUNS runs of the window at once (one per
// thread: desc pair, chunk start, member block), numbers their elements with one workgroup scan, and
// the waves then stream the concatenation in 64-element blocks — every lane of every load holds an
// element whichever run it belongs to, and every wave has blocks whether the window has thousands of
// short runs (dense calls) or a handful of long ones (sparse calls). A block's runs come from two LDS
// maps built per batch: the run holding the block's first element, and a bitmask of the runs that
// start inside the block, so a lane's run is that run plus a mbcnt of the mask. The ranks of a block's
// elements are one gather from rank_of_member (the member blocks of a block's runs: a few hundred bytes,
// L2-resident); PK_U blocks are in flight per wave. f(offset, rank) is called for every lane, with
// rank RANK_NONE for lanes past the window (a min table ignores it). IDENT: the rank is the member's
// position (novelty).
constexpr uint32_t PK_RUNS = 1024;      // runs per batch (one per thread of a 1024-thread workgroup)
constexpr uint32_t PK_NBLK = 256;       // 64-element blocks per element window of a batch
constexpr uint32_t PK_EW = 64 * PK_NBLK;
// LDS words the walk needs (callers may alias them with their emit bitmap)
constexpr uint32_t PK_SCRATCH_WORDS = 2 * PK_RUNS + 3 * PK_NBLK;
#ifndef SYZ_PK_U
#define SYZ_PK_U 4
#endif

// Workgroup exclusive scan of a run length and of "non-empty" at once: pre = elements of the runs
// before this one, k = non-empty runs before it, T = all elements. Wave totals are summed in a rolled
// loop (the unrolled block_excl_scan holds every wave total in registers). lds: 2 * waves words.
__device__ __forceinline__ void pk_scan(uint32_t len, uint32_t* lds, uint32_t& pre, uint32_t& k, uint32_t& T) {
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t inc = wave_incl_scan<uint32_t>(len);
  const uint64_t bal = __ballot(len != 0);
  const uint32_t kin = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
  if (__lane_id() == 63) {
    lds[2 * w] = inc;
    lds[2 * w + 1] = (uint32_t)__popcll(bal);
  }
  __syncthreads();
  uint32_t p = 0, q = 0, tp = 0;
#pragma unroll 1
  for (int i = 0; i < nw; i++) {
    const uint32_t a = lds[2 * i], b = lds[2 * i + 1];
    if (i < w) {
      p += a;
      q += b;
    }
    tp += a;
  }
  __syncthreads();
  pre = inc - len + p;
  k = kin + q;
  T = tp;
}

}  // namespace syz

// Device code shared by the raw-cover pipelines: minimizeCorpus (panels.hip) and the new-coverage
// check on windows (novelty_win.hip). Chunks of <= PCAP PCs of <= 64 members of one call group are
// transposed into PC windows (P, k_part3) and walked per (call, window) (M, for_window_elems).
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


// Diagnostic build only (-DSYZ_STAMPS, tools/build_variant.sh): per-workgroup phase timestamps of the
// transpose and the direct walk (thread 0, s_memtime), read back by syzgpu_debug_stamps.
#ifdef SYZ_STAMPS
constexpr uint32_t STAMP_WG = 1u << 15;
static __device__ unsigned long long g_stamp[2][STAMP_WG][8];
#define SYZ_STAMP(k, slot)                                                                  \
  do {                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < STAMP_WG) g_stamp[k][blockIdx.x][slot] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define SYZ_STAMP(k, slot)
#endif

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

// ---- P, register form (k_part3): each PC read from HBM once ----------------------------------------
// One workgroup per chunk, as k_part, but every wave loads all of its tiles' PCs into registers up
// front (all of them in flight per lane), so the second pass needs no second read; and the LDS
// atomics of both passes are taken once per RUN: the 64 lanes of a tile hold consecutive PCs of one
// (sorted) cover, so neighbouring lanes mostly share a window; a run's head lane adds the run's
// length to the window's count (pass 1) or reserves its slots (pass 2) and the run's lanes write
// consecutive LDS words. 74 KB of LDS: two workgroups per CU.
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

// BLOCK threads per chunk; each wave holds TPW tiles of PCs in registers. 512 threads x 40 tiles:
// two workgroups (74 KB of LDS each) share a CU, so one's dependent metadata loads overlap the
// other's passes.
template <int BLOCK, int TPW, bool NOV = false>
__global__ __launch_bounds__(BLOCK) void k_part3(
    const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off, const uint32_t* __restrict__ members,
    const uint64_t* __restrict__ mpos, const uint32_t* __restrict__ sbeg, const PChunk* chunks,
    const uint64_t* nchunks_dev, const PGroup* pg, const uint64_t* gchunk, const uint64_t* gdesc, uint32_t lo,
    uint32_t* __restrict__ elems, uint16_t* __restrict__ desc, int* err, NovSrc ns = NovSrc{}) {
  constexpr int WAVES = BLOCK / 64;
  static_assert(TMAX <= (uint32_t)(TPW * WAVES), "k_part3: tiles per wave");
  __shared__ uint32_t obuf[PCAP];
  __shared__ uint32_t hist[WMAX + 1];
  __shared__ uint32_t tpre[MEMB + 1];
  __shared__ uint32_t mlo[MEMB], mhi[MEMB];
  __shared__ uint64_t mraw[MEMB];  // byte address of the member's PC at block coordinate 0
  __shared__ uint32_t red[WAVES + 1];
  __shared__ uint4 tinfo[TMAX];
  __shared__ uint32_t tlast[NOV ? TMAX : 1];  // NOV: the last PC of every tile
  __shared__ uint8_t mtab[NOV ? MEMB : 1];    // NOV: the member is a table
  const uint64_t c = blockIdx.x;
  if (c >= *nchunks_dev) return;
  const int wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  const PChunk ch = chunks[c];
  const PGroup gp = pg[ch.g];
  const uint32_t S = gp.S, W = gp.W;
  const uint32_t cb = ch.sub, ce = ch.sub + ch.len;
  int bad = 0;  // NOV: err bits of the lists this thread saw out of order
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
        // the member began in an earlier chunk: its first PC here against the one before
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
    if constexpr (NOV)  // bit 0: a table; bit 1: the member's previous tile is tile t - 1 of this chunk
      fl = (mtab[m] ? 1u : 0u) | (t > tpre[m] ? 2u : 0u);
    tinfo[t] = make_uint4((uint32_t)base, (uint32_t)(base >> 32), min(64u, mhi[m] - q0) | (m << 8), fl);
  }
  __syncthreads();
  // every tile of this wave: t = wv + WAVES k; its PCs into registers, all loads in flight
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
  // pass 1: window histogram, one LDS atomic per run
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
      if (in && (w >= W || (lane > 0 && pv >= v[k]))) bad |= eb;  // out of order (or outside every window)
      if (lane + 1 == cnt) tlast[t] = v[k];
    } else {
      if (in && w >= W) atomicOr(err, 1);  // outside [lo, hi]: an unsorted cover; redone on exact bounds
    }
    const TileRun r = tile_run(w, in && w < W, lane);
    if (r.head) atomicAdd(&hist[w], r.len);
  }
  __syncthreads();
  // window starts (exclusive scan) -> desc row and cursors
  uint16_t* drow = desc + gdesc[ch.g] + (c - gchunk[ch.g]) * (uint64_t)(W + 1);
  {
    uint32_t run = 0;
    for (uint32_t b0 = 0; b0 <= W; b0 += BLOCK) {
      const uint32_t i = b0 + threadIdx.x;
      const uint32_t x = i < W ? hist[i] : 0;
      uint32_t tot;
      const uint32_t pre = block_excl_scan<BLOCK>(x, red, &tot) + run;
      if (i <= W) {
        drow[i] = (uint16_t)pre;
        hist[i] = pre;
      }
      run += tot;
    }
  }
  __syncthreads();
  // pass 2: element = offset in window | member tag, window-major into obuf, a run's slots reserved
  // by its head
  const uint32_t omask = (1u << S) - 1;
#pragma unroll
  for (int k = 0; k < TPW; k++) {
    const uint32_t t = wv + WAVES * k;
    if (t >= ntiles) break;
    const uint32_t z = tinfo[t].z;
    const uint32_t d = v[k] - lo, w = d >> S;
    const bool in = lane < (z & 0xFFu) && w < W;
    if constexpr (NOV) {
      const uint32_t f = tinfo[t].w;
      if (lane == 0 && (f & 2u) && tlast[t - 1] >= v[k]) bad |= (f & 1u) ? 1 : 4;
    }
    const TileRun r = tile_run(w, in, lane);
    uint32_t base = r.head ? atomicAdd(&hist[w], r.len) : 0u;
    base = (uint32_t)__shfl((int)base, (int)r.start, 64);
    if (in) obuf[base + (lane - r.start)] = (d & omask) | ((z >> 8) << S);
  }
  if constexpr (NOV) {
    const uint64_t bm = __ballot(bad != 0);
    if (bm) {
      int all = bad;
#pragma unroll
      for (int dd = 32; dd >= 1; dd >>= 1) all |= __shfl_xor(all, dd, 64);
      if (lane == (unsigned)(__ffsll((unsigned long long)bm) - 1)) atomicOr(err, all);
    }
  }
  __syncthreads();
  uint32_t* dst = elems + ch.elem;
  for (uint32_t i = threadIdx.x; i < ch.len; i += BLOCK) dst[i] = obuf[i];
}

// ---- P, lean form (k_part4) ---------------------------------------------------------------------
// The transpose of k_part3 with its per-tile instruction count cut: k_part3 issued ~89 VALU per 64-PC
// tile (profiles/r03_pmin_base: 590M VALU for 6.6M tiles, ~1 ms of issue on 256 CUs for a 1.4 ms
// kernel) on run detection, 64-bit tile addresses and per-lane tile-table loads. Here:
//   * a tile's count, member tag and address are wave-uniform (readfirstlane into SGPRs), so its load
//     is a saddr global load and its bookkeeping is scalar;
//   * one LDS atomic per PC instead of run detection: covers are sparse against the windows (a
//     256-PC median cover over 256 windows), so a tile's PCs rarely share a window and the atomics
//     rarely collide; when they do (dense covers) the LDS serializes only those lanes;
//   * the chunk leaves as aligned 16-byte vector stores (k_chunks aligns chunk starts).
// Same inputs and outputs as k_part3 (elements in a window's run are in atomic order, which neither
// consumer depends on).
template <int BLOCK, int TPW, bool NOV = false>
__global__ __launch_bounds__(BLOCK) void k_part4(
    const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off, const uint32_t* __restrict__ members,
    const uint64_t* __restrict__ mpos, const uint32_t* __restrict__ sbeg, const PChunk* chunks,
    const uint64_t* nchunks_dev, const PGroup* pg, const uint64_t* gchunk, const uint64_t* gdesc, uint32_t lo,
    uint32_t* __restrict__ elems, uint16_t* __restrict__ desc, int* err, NovSrc ns = NovSrc{}) {
  constexpr int WAVES = BLOCK / 64;
  static_assert(TMAX <= (uint32_t)(TPW * WAVES), "k_part4: tiles per wave");
  __shared__ __align__(16) uint32_t obuf[PCAP + 64];  // + a slot per lane for lanes with no element
  __shared__ uint32_t hist[WMAX + 1 + 64];             // + a counter per lane for them
  __shared__ uint32_t tpre[MEMB + 1];
  __shared__ uint32_t mlo[MEMB], mhi[MEMB];
  __shared__ uint64_t mraw[MEMB];
  __shared__ uint32_t red[WAVES + 1];
  __shared__ uint4 tinfo[TMAX];
  __shared__ uint32_t tlast[NOV ? TMAX : 1];
  __shared__ uint8_t mtab[NOV ? MEMB : 1];
  const uint64_t c = blockIdx.x;
  if (c >= *nchunks_dev) return;
  const int wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  SYZ_STAMP(0, 0);
  const PChunk ch = chunks[c];
  const PGroup gp = pg[ch.g];
  const uint32_t S = gp.S, W = gp.W;
  const uint32_t cb = ch.sub, ce = ch.sub + ch.len;
  int bad = 0;  // err bits this thread found (1: outside the windows / a table out of order, 4: a cover)
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
  SYZ_STAMP(0, 1);
  // this wave's tiles t = wv + WAVES k: PCs into registers, all loads in flight. Straight-line code
  // (a lane past its tile re-reads the tile's last PC, a tile past the chunk re-reads the last tile
  // with count 0), so the compiler counts its waits instead of draining at every branch join; a
  // tile's count and member tag stay in SGPRs.
  const uint32_t DUMMY = WMAX + 1 + lane;  // the histogram slot of a lane with no element (one per lane:
                                          // a shared one serializes every idle lane's atomic)
  static_assert(TPW <= 64, "a tile's count and tag per lane of one register");
  // lane k of czv: count | tag << 8 of this wave's tile k (count 0 past the chunk); v_readlane per use
  uint32_t czv = 0;
  {
    const uint32_t t = wv + WAVES * lane;
    const uint32_t z = tinfo[min(t, ntiles - 1)].z;
    czv = lane < (unsigned)TPW ? (t < ntiles ? z : (z & ~0xFFu)) : 0u;
  }
  auto cz = [&](int k) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)czv, k); };
  uint32_t v[TPW];
#pragma unroll
  for (int k = 0; k < TPW; k++) {
    const uint32_t t = wv + WAVES * k;
    const uint4 ti = tinfo[min(t, ntiles - 1)];
    const uint32_t z = (uint32_t)__builtin_amdgcn_readfirstlane((int)ti.z);
    const uint64_t base = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)ti.y) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)ti.x);
    v[k] = reinterpret_cast<const uint32_t*>((uintptr_t)base)[min(lane, (z & 0xFFu) - 1)];
    // tile-table reads in groups of 8: the scheduler would otherwise hoist all of them (and their
    // addresses) ahead of the first load
    if ((k & 7) == 7) __builtin_amdgcn_sched_barrier(0);
  }
  // pass 1: window histogram, one LDS atomic per PC
#pragma unroll
  for (int k = 0; k < TPW; k++) {
    const uint32_t t = wv + WAVES * k;
    const uint32_t w = (v[k] - lo) >> S;
    const bool in = lane < (cz(k) & 0xFFu);
    if constexpr (NOV) {
      if (t < ntiles) {
        const uint32_t pv = __shfl_up(v[k], 1, 64);
        const uint32_t eb = (tinfo[t].w & 1u) ? 1u : 4u;
        if (in && (w >= W || (lane > 0 && pv >= v[k]))) bad |= eb;
        if (lane + 1 == (cz(k) & 0xFFu)) tlast[t] = v[k];
      }
    } else {
      bad |= (in && w >= W) ? 1 : 0;  // outside [lo, hi]: an unsorted cover; redone on exact bounds
    }
    atomicAdd(&hist[in && w < W ? w : DUMMY], 1u);
    if ((k & 7) == 7) __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  // window starts (exclusive scan) -> desc row and cursors
  uint16_t* drow = desc + gdesc[ch.g] + (c - gchunk[ch.g]) * (uint64_t)(W + 1);
  {
    uint32_t run = 0;
    for (uint32_t b0 = 0; b0 <= W; b0 += BLOCK) {
      const uint32_t i = b0 + threadIdx.x;
      const uint32_t x = i < W ? hist[i] : 0;
      uint32_t tot;
      const uint32_t pre = block_excl_scan<BLOCK>(x, red, &tot) + run;
      if (i <= W) {
        drow[i] = (uint16_t)pre;
        hist[i] = pre;
      }
      run += tot;
    }
  }
  __syncthreads();
  SYZ_STAMP(0, 3);
  // pass 2: element = offset in window | member tag, window-major into obuf through the cursors; the
  // cursor atomics of PB tiles are issued before their stores wait on them
  const uint32_t omask = (1u << S) - 1;
  constexpr int PB = 8;
#pragma unroll
  for (int k0 = 0; k0 < TPW; k0 += PB) {
    uint32_t pos[PB], el[PB];
    bool ok[PB];
#pragma unroll
    for (int k = k0; k < k0 + PB && k < TPW; k++) {
      const uint32_t d = v[k] - lo, w = d >> S;
      ok[k - k0] = lane < (cz(k) & 0xFFu) && w < W;
      el[k - k0] = (d & omask) | ((cz(k) >> 8) << S);
      pos[k - k0] = atomicAdd(&hist[ok[k - k0] ? w : DUMMY], 1u);
    }
#pragma unroll
    for (int k = k0; k < k0 + PB && k < TPW; k++) obuf[ok[k - k0] ? pos[k - k0] : PCAP + lane] = el[k - k0];
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (NOV) {
#pragma unroll
    for (int k = 0; k < TPW; k++) {
      const uint32_t t = wv + WAVES * k;
      if (t < ntiles) {
        const uint32_t f = tinfo[t].w;
        if (lane == 0 && (f & 2u) && tlast[t - 1] >= v[k]) bad |= (f & 1u) ? 1 : 4;
      }
    }
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
  SYZ_STAMP(0, 4);
  // chunk starts are 16-byte aligned (k_chunks): vector stores, then the tail
  uint32_t* dst = elems + ch.elem;
  const uint32_t n4 = ch.len >> 2;
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  const uint4* o4 = reinterpret_cast<const uint4*>(obuf);
  for (uint32_t i = threadIdx.x; i < n4; i += BLOCK) d4[i] = o4[i];
  for (uint32_t i = (n4 << 2) + threadIdx.x; i < ch.len; i += BLOCK) dst[i] = obuf[i];
  SYZ_STAMP(0, 5);
}

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
// increasing in the COUNT pass, as k_part3).
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

// ---- M: min rank per key of one (call, window) ------------------------------------------------------
// A wave takes the window's runs of 64 chunks at a time (one chunk's run per lane of metadata) and
// then walks them RB runs at a time: for each run one coalesced 256-byte load brings the Go-sort
// ranks of the run's 64-member block into a register (lane m = member m), and the run's elements are
// loaded one per lane; an element's rank is then a register shuffle by its member tag. RB runs'
// loads are in flight together.
#ifndef SYZ_RB
#define SYZ_RB 16
#endif
constexpr int RB = SYZ_RB;
constexpr int TU = 4;  // slices in flight per long run
// IDENT: the rank of a member is its position (the new-coverage check: batch order), no rank loads.
template <int RBN = RB, bool IDENT = false, class F>
__device__ __forceinline__ void for_window_elems(const PItem it, const PChunk* __restrict__ chunks,
                                                 const uint64_t* gchunk, const uint64_t* gdesc, const PGroup* pg,
                                                 const uint16_t* __restrict__ desc, const uint32_t* __restrict__ elems,
                                                 const uint32_t* __restrict__ rank_of_member, uint32_t nmem_total,
                                                 int nwaves, F f) {
  const uint32_t g = it.g, w = it.w;
  const uint64_t c0 = gchunk[g], c1 = gchunk[g + 1];
  const uint32_t W = pg[g].W, S = pg[g].S;
  const uint32_t omask = (1u << S) - 1;
  const uint16_t* d0 = desc + gdesc[g] + w;
  const int wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  const uint32_t last_m = nmem_total ? nmem_total - 1 : 0;
  // wave wv takes runs c0 + wv, c0 + wv + nwaves, ... (64 of them per batch), so a window with few
  // chunks still spreads over every wave
  const uint64_t nrun = c1 - c0;
  for (uint64_t b0 = (uint64_t)wv; b0 < nrun; b0 += (uint64_t)nwaves * 64) {
    const uint64_t c = c0 + b0 + (uint64_t)lane * nwaves;
    uint32_t len = 0, mb = 0, stl = 0, sth = 0;
    if (c < c1) {
      const uint16_t* d = d0 + (c - c0) * (uint64_t)(W + 1);
      const uint32_t s0 = d[0], s1 = d[1];
      len = s1 - s0;
      const uint64_t st = chunks[c].elem + s0;
      stl = (uint32_t)st;
      sth = (uint32_t)(st >> 32);
      mb = chunks[c].mb;
    }
    const uint32_t nr = (uint32_t)min<uint64_t>(64, (nrun - b0 + nwaves - 1) / nwaves);
    for (uint32_t r0 = 0; r0 < nr; r0 += RBN) {
      uint32_t rk[RBN], e0[RBN], e1[RBN], ln[RBN];
      uint64_t sts[RBN];
#pragma unroll
      for (int r = 0; r < RBN; r++) {
        const uint32_t j = r0 + r;
        ln[r] = j < nr ? (uint32_t)__builtin_amdgcn_readlane((int)len, (int)j) : 0u;
        const uint32_t mbj = (uint32_t)__builtin_amdgcn_readlane((int)mb, (int)j);
        sts[r] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)sth, (int)j) << 32) |
                 (uint32_t)__builtin_amdgcn_readlane((int)stl, (int)j);
        rk[r] = IDENT ? mbj : 0u;
        e0[r] = 0;
        e1[r] = 0;
        if (ln[r]) {
          if constexpr (!IDENT) rk[r] = rank_of_member[min(mbj + lane, last_m)];
          if (lane < ln[r]) e0[r] = elems[sts[r] + lane];
          if (lane + 64 < ln[r]) e1[r] = elems[sts[r] + 64 + lane];
        }
      }
#pragma unroll
      for (int r = 0; r < RBN; r++) {
        if (!ln[r]) continue;
        {
          const uint32_t R = IDENT ? rk[r] + (e0[r] >> S) : (uint32_t)__shfl((int)rk[r], (int)(e0[r] >> S), 64);
          if (lane < ln[r]) f(e0[r] & omask, R);
        }
        if (ln[r] > 64) {
          const uint32_t R = IDENT ? rk[r] + (e1[r] >> S) : (uint32_t)__shfl((int)rk[r], (int)(e1[r] >> S), 64);
          if (lane + 64 < ln[r]) f(e1[r] & omask, R);
          for (uint32_t k = 128; k < ln[r]; k += 64 * TU) {  // long runs: TU 64-PC slices in flight
            uint32_t x[TU];
#pragma unroll
            for (int u = 0; u < TU; u++) {
              const uint32_t i = k + 64 * u + lane;
              x[u] = i < ln[r] ? elems[sts[r] + i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < TU; u++) {
              const uint32_t R2 =
                  IDENT ? rk[r] + (x[u] >> S) : (uint32_t)__shfl((int)rk[r], (int)(x[u] >> S), 64);
              if (k + 64 * u + lane < ln[r]) f(x[u] & omask, R2);
            }
          }
        }
      }
    }
  }
}

// ---- M walk, packed form ------------------------------------------------------------------------------
// for_window_elems spends one wave instruction per run: a run of ~50 elements leaves a quarter of the
// lanes idle and pays ~47 VALU of per-run bookkeeping (profiles/r03_pmin_base: ~0.9 VALU wave
// instructions per element). Here the workgroup takes up to PK_RUNS runs of the window at once (one per
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

template <int U, bool IDENT, class F>
__device__ __forceinline__ void for_window_packed(const PItem it, const PChunk* __restrict__ chunks,
                                                  const uint64_t* gchunk, const uint64_t* gdesc, const PGroup* pg,
                                                  const uint16_t* __restrict__ desc,
                                                  const uint32_t* __restrict__ elems,
                                                  const uint32_t* __restrict__ rank_of_member, uint32_t* scratch,
                                                  uint64_t* red64, F f) {
  static_assert(PK_RUNS == 1024, "one run per thread");
  const uint32_t g = it.g, w = it.w;
  const uint64_t c0 = gchunk[g], c1 = gchunk[g + 1];
  if (c1 == c0) return;
  const uint32_t W = pg[g].W, S = pg[g].S;
  const uint32_t omask = (1u << S) - 1;
  const uint16_t* d0 = desc + gdesc[g] + w;
  const uint64_t gbase = chunks[c0].elem;  // element offsets of the group fit 32 bits from here
  const uint32_t* gel = elems + gbase;
  uint32_t* rrel = scratch;                 // [PK_RUNS] element offset of run k's element 0 - its prefix
  uint32_t* rmb = scratch + PK_RUNS;        // [PK_RUNS] first member of run k's chunk
  uint32_t* bstart = scratch + 2 * PK_RUNS;  // [PK_NBLK] run holding block j's first element
  uint32_t* bmask = bstart + PK_NBLK;        // [2 PK_NBLK] runs starting inside block j (bit = offset)
  const int nwaves = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  // a thread's run of a batch: desc pair and chunk (loaded one batch ahead)
  auto load_run = [&](uint64_t c, uint32_t& len, uint32_t& rel, uint32_t& mb) {
    len = rel = mb = 0;
    if (c < c1) {
      const uint16_t* d = d0 + (c - c0) * (uint64_t)(W + 1);
      const uint32_t s0 = d[0];
      len = (uint32_t)d[1] - s0;
      const PChunk ch = chunks[c];
      rel = (uint32_t)(ch.elem - gbase) + s0;
      mb = ch.mb;
    }
  };
  uint32_t nlen, nrel, nmb;
  load_run(c0 + threadIdx.x, nlen, nrel, nmb);
  for (uint64_t rb = c0; rb < c1; rb += PK_RUNS) {
    // ---- batch: one run per thread, non-empty runs compacted in element order ----
    const uint32_t len = nlen, rel = nrel, mb = nmb;
    uint32_t pre, k, T;
    pk_scan(len, reinterpret_cast<uint32_t*>(red64), pre, k, T);
    if (len) {
      rrel[k] = rel - pre;  // (rel - pre + idx) mod 2^32 = rel + (idx - pre): the element's offset
      rmb[k] = mb;
    }
    load_run(rb + PK_RUNS + threadIdx.x, nlen, nrel, nmb);  // the next batch's runs, in flight meanwhile
    for (uint32_t ew = 0; ew < T; ew += PK_EW) {
      const uint32_t te = min(T, ew + PK_EW);
      for (uint32_t j = threadIdx.x; j < 2 * PK_NBLK; j += blockDim.x) bmask[j] = 0;
      __syncthreads();
      if (len && pre < te && pre + len > ew) {
        // block starts inside [max(pre, ew), min(pre + len, te)) belong to run k
        const uint32_t a = max(pre, ew) - ew, b = min(pre + len, te) - ew;
        for (uint32_t j = (a + 63) >> 6; (j << 6) < b; j++) bstart[j] = k;
        if (pre >= ew && (pre & 63)) {
          const uint32_t o = pre - ew;
          atomicOr(&bmask[2 * (o >> 6) + ((o >> 5) & 1)], 1u << (o & 31));
        }
      }
      __syncthreads();
      // ---- the waves stream the window's blocks, U at a time, straight-line (no per-lane branches,
      // so the compiler's waits are counted, not vmcnt(0) at every join): a lane past the window
      // reads its block's first element and applies RANK_NONE, a no-op for a min table ----
      const uint32_t nblk = (te - ew + 63) >> 6;
      const uint32_t step = (uint32_t)nwaves * U;
      for (uint32_t j0 = wv; j0 < nblk; j0 += step) {
        uint32_t r0[U], slo[U], shi[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t jj = min(j0 + (uint32_t)nwaves * u, nblk - 1);
          r0[u] = bstart[jj];
          const uint32_t mlo = bmask[2 * jj], mhi = bmask[2 * jj + 1];
          slo[u] = (mlo >> 1) | (mhi << 31);  // runs starting at offsets 1..lane: mbcnt of mask >> 1
          shi[u] = mhi >> 1;
        }
        uint32_t rl[U], mbr[U], id[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t j = j0 + (uint32_t)nwaves * u, jj = min(j, nblk - 1);
          const uint32_t idx = ew + (j << 6) + lane;
          ok[u] = j < nblk && idx < te;
          const uint32_t r = r0[u] + __builtin_amdgcn_mbcnt_hi(shi[u], __builtin_amdgcn_mbcnt_lo(slo[u], 0u));
          const uint32_t rr = ok[u] ? r : r0[u];
          id[u] = ok[u] ? idx : ew + (jj << 6);  // the block's first element lies in run r0
          rl[u] = rrel[rr];
          mbr[u] = rmb[rr];
        }
        uint32_t e[U];
#pragma unroll
        for (int u = 0; u < U; u++) e[u] = gel[rl[u] + id[u]];
        uint32_t R[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          if constexpr (IDENT)
            R[u] = mbr[u] + (e[u] >> S);
          else
            R[u] = rank_of_member[mbr[u] + (e[u] >> S)];
        }
#pragma unroll
        for (int u = 0; u < U; u++) f(e[u] & omask, ok[u] ? R[u] : RANK_NONE);
      }
      __syncthreads();  // bstart / bmask are rebuilt for the next element window
    }
  }
}

}  // namespace syz

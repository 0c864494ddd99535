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
#define SYZ_DS 15
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
constexpr uint32_t DENSE = 8192u >> (15 - DS);  // PCs per window (per 32K addresses: 8192) above which a call is direct-mode
constexpr uint32_t HTARGET = SYZ_HTARGET;  // PCs per window a sparse call's window size aims at


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
    for (uint64_t s = 0; s < sl; s += PCAP, c++)
      chunks[c] = PChunk{base + s, (uint32_t)min<uint64_t>(PCAP, sl - s), (uint32_t)mb, (uint32_t)(me - mb),
                         (uint32_t)s, g};
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

}  // namespace syz

// syz-fuzzer's new-coverage check over a batch on PC windows (syz-fuzzer/fuzzer.go:446-470 execute;
// the same rule as syz-manager NewInput, manager.go:609-616) — the default strategy of
// syzgpu_novelty_batch(_dev), on the raw-cover pipeline of the Minimize step (panels_dev.hpp).
//
// The rule (novelty.hip's header): cover k of call g is new iff one of its PCs —
// not 0xFFFFFFFF, not a flake, not in maxCover0[g] — occurs first, among the covers of g in batch
// order, in cover k; the updated table is maxCover0[g] plus every such PC, minus the table's
// 0xFFFFFFFF when it took a Union. So per (call, PC) key only the FIRST holder matters, with
// maxCover0[g] ahead of every cover: exactly the min-rank-per-key of Minimize with the batch order as
// the rank. Each call group's members are [its maxCover0 table, its covers in batch order]; a member's
// rank is its position in that list, so the table is the group's smallest rank.
//
//   G  group partition (stable) + members + lengths (a trailing 0xFFFFFFFF dropped) + the PC span
//   P  k_slab<NOV> (slab_dev.hpp): the members' PCs transposed into 2^DB-address windows (one HBM read per PC), every
//      list checked strictly increasing on the way
//   M  k_nw_min: a workgroup per (call, window): a direct min-rank table in LDS (and a presence bitmap
//      the element that finds an entry empty sets), the LDS updates of 16 runs issued before one
//      wait; then the present keys in PC order: a key is kept if the table holds it or a non-flake
//      cover does (the window's flakes in an LDS bitmap), a cover that wins a kept key is new (byte
//      stores, deduplicated by an LDS rank bitmap); the kept keys leave as a bitmap per window (2^DB
//      bits), their count beside it
//   E  scan of the counts, then every window's bitmap expands to its PCs at its offset (the updated
//      tables, sorted by (call, PC)), a table's 0xFFFFFFFF last unless the call took a Union
//
// Integer work throughout; bit-exact by construction. Direct windows need the PC span to fit WMAX
// windows (2^15 x 1024 = 32M addresses); a wider span takes hashed windows (k_nw_hash: a window size
// per call, an open-addressing LDS table, the kept keys sorted per address sub-range and stored as a
// list), up to the whole u32 space. Only G > 4096 falls back to the keyed table (novelty.hip).
// Inside a narrow span the calls with few PCs per direct window take hashed windows too (NW_HSPARSE;
// measured slower in round 2, before the slab transpose, and faster since: 4.30 -> 3.92 ms at config
// 3). Measured and dropped (profiles/r02_ab/novelty_ab.md): persistent workgroups with the next item
// prefetched, branch-free batches.
#include <algorithm>
#include <cstdlib>
#include <numeric>

#include "panels_dev.hpp"
#include "pipeline.hpp"
#include "slab_dev.hpp"

namespace syz {

// Direct windows (calls with many PCs per window): 2^DB addresses, a 2^DB-entry min table. DB = 14: 64 KB
// of LDS, two 512-thread workgroups per CU, so one's metadata and table set-up overlap the other's walk
// (15 when the span needs it: 128 KB, one 1024-thread workgroup).
template <uint32_t SB>
struct NwCfg {
  static constexpr uint32_t BITS = 1u << SB;      // addresses per window
  static constexpr uint32_t FLK = BITS / 32;      // u32 words of a window's bitmaps
  static constexpr int BLOCK = SB >= 15 ? 1024 : 512;
  static constexpr uint32_t BMW = SB >= 15 ? 5120 : 2048;  // LDS rank bitmap words (winner dedup)
};
constexpr int NE_BLOCK = 256;  // k_nw_emit

// per call: window layout of the kept bitmaps (u32 words) and of the count slots
struct NwGroup {
  uint64_t kbase;  // first kept-bitmap word of the call's window 0
  uint64_t sbase;  // first count slot (W + 1 slots: the windows, then the table's 0xFFFFFFFF)
};

// the per-call state of one batch: error word, sentinel and Union flags, kept ranks, the span
__global__ void k_nw_init(int* perr, uint8_t* has_sent, uint8_t* upd, uint32_t G, uint8_t* sel8, size_t nsel,
                          uint32_t* span) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nsel; i += (size_t)gridDim.x * blockDim.x) {
    sel8[i] = 0;
    if (i <= G) {
      has_sent[i] = 0;
      upd[i] = 0;
    }
    if (i < 2) {
      perr[i] = 0;
      span[i] = i ? 0u : 0xFFFFFFFFu;
    }
  }
}

// combined members: call g's list is [table g (entry id n + g), its covers in batch order], with the
// members' lengths gathered from the entry-order lengths (elen: covers, then tables)
__global__ void k_nw_members(const uint32_t* members, const uint64_t* gstart, const uint32_t* group, size_t n,
                             uint32_t G, const uint32_t* elen, uint32_t* cmem, uint64_t* cstart, uint32_t* mlen) {
  const size_t tot = n > (size_t)G + 1 ? n : (size_t)G + 1;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
    if (i < n) {
      const uint32_t e = members[i];
      const uint32_t g = group[e] < G ? group[e] : 0u;  // an invalid id was counted in group 0
      cmem[i + g + 1] = e;
      mlen[i + g + 1] = elen[e];
    }
    if (i < G) {
      cmem[gstart[i] + i] = (uint32_t)n + (uint32_t)i;
      mlen[gstart[i] + i] = elen[n + i];
    }
    if (i <= G) cstart[i] = gstart[i] + i;
  }
}

// member lengths without a trailing 0xFFFFFFFF (foreach never matches it, cover.go:81-102; a table's
// is put back after the windows), which tables had one, and the span of the other PCs; in entry order
// (coalesced offsets and lengths, the first and last PC of neighbouring entries on neighbouring lines)
__global__ __launch_bounds__(256) void k_nw_meta(const uint32_t* pcs, const uint64_t* off, const uint32_t* mc,
                                                 const uint64_t* mc_off, size_t n, uint32_t G, uint32_t* elen,
                                                 uint8_t* has_sent, uint32_t* span) {
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n + G; i += (size_t)gridDim.x * blockDim.x) {
    const bool tab = i >= n;
    const uint32_t* src = tab ? mc + mc_off[i - n] : pcs + off[i];
    uint64_t len = tab ? mc_off[i - n + 1] - mc_off[i - n] : off[i + 1] - off[i];
    uint32_t first = 0, last = 0;
    if (len) {
      first = src[0];
      last = src[len - 1];
      if (last == SENT) {
        len--;
        if (tab) has_sent[i - n] = 1;
        if (len) last = src[len - 1];
      }
    }
    elen[i] = (uint32_t)len;
    if (len) {
      lo = min(lo, first);
      hi = max(hi, last);
    }
  }
  block_span_update<256>(lo, hi, span);
}

// a table slot: the window offset rotated right by 2 bits, so PCs on 4-byte boundaries spread over
// every LDS bank
template <uint32_t SB>
__device__ __forceinline__ uint32_t nw_index(uint32_t o) {
  return ((o >> 2) | (o << (SB - 2))) & ((1u << SB) - 1);
}

#ifndef SYZ_NW_U
#define SYZ_NW_U 2
#endif

// M: one (call, window). tab = min member position per window offset; the table's position cstart[g]
// is OLD.
template <uint32_t SB>
__global__ __launch_bounds__(NwCfg<SB>::BLOCK) void k_nw_min(
    const uint32_t* order, uint32_t W, const SGroup* sg, const uint32_t* gslab, const uint64_t* gebase,
    const uint32_t* D, const PSlab* slabs, const uint32_t* elems, const uint64_t* cstart, uint32_t lo, const uint32_t* __restrict__ fl, const uint32_t* __restrict__ fstart,
    const NwGroup* ng_, uint32_t* kbits, uint32_t* wcount, uint8_t* sel8, uint8_t* upd, int dbg) {
  using K = NwCfg<SB>;
  constexpr int BLOCK = K::BLOCK;
  __shared__ __align__(16) uint32_t tab[K::BITS];
  __shared__ uint32_t bm[K::BMW];
  __shared__ uint32_t flk[K::FLK];
  __shared__ uint32_t pres[K::FLK];  // offsets some member holds (set by the element that lowers NONE)
  __shared__ uint32_t red[BLOCK / 64 + 1];
  __shared__ uint64_t red64[BLOCK / 64 + 1];
  static_assert(K::BMW >= 2 * BLOCK + 3 * PK_NBLK, "the walk's scratch in the rank bitmap");
  const PItem it{order[blockIdx.x / W], blockIdx.x % W};
  const uint32_t g = it.g, w = it.w;
  {
    uint4* t4 = reinterpret_cast<uint4*>(tab);
    const uint4 none4 = make_uint4(RANK_NONE, RANK_NONE, RANK_NONE, RANK_NONE);
    for (uint32_t i = threadIdx.x; i < K::BITS / 4; i += BLOCK) t4[i] = none4;
  }
  for (uint32_t i = threadIdx.x; i < K::FLK; i += BLOCK) {
    flk[i] = 0;
    pres[i] = 0;
  }
  __syncthreads();
  // the flakes inside this window's addresses: fl[fstart[w], fstart[w + 1])
  const uint32_t wlo = lo + (w << SB);
  for (uint32_t i = fstart[w] + threadIdx.x; i < fstart[w + 1]; i += BLOCK) {
    const uint32_t o = fl[i] - wlo;  // flakes not increasing (rejected after the batch) land anywhere
    if (o < K::BITS) atomicOr(&flk[o >> 5], 1u << (o & 31));
  }
  // the window's slab runs; a member's rank is its position (the table first, then batch order); the
  // rank bitmap is the walk's scratch until the walk is done
  if (!(dbg & 1))
    for_slab_window<SYZ_NW_U, true>(it, sg, gslab, gebase, D, slabs, elems, nullptr, bm, red64,
                                    [&](uint32_t o, uint32_t R) {
                                      // (a plain read first: an input that loses to the rank there
                                      // issues no atomic; a slot below NONE is already present)
                                      uint32_t* t = &tab[nw_index<SB>(o)];
                                      if (R != RANK_NONE && *t > R && atomicMin(t, R) == RANK_NONE)
                                        atomicOr(&pres[o >> 5], 1u << (o & 31));
                                    });
  __syncthreads();
  if (dbg & 2) return;
  const uint64_t gb = cstart[g], ng = cstart[g + 1] - gb;
  const uint32_t span = (uint32_t)min<uint64_t>((uint64_t)K::BMW * 32, ng);
  const uint32_t words = (span + 31) / 32;
  for (uint32_t i = threadIdx.x; i < words; i += BLOCK) bm[i] = 0;
  __syncthreads();
  // the present offsets in PC order, a 32-offset word per thread: kept keys as bitmap words (coalesced
  // u32 stores), new covers marked
  const NwGroup gl = ng_[g];
  uint32_t* kb32 = kbits + gl.kbase + (uint64_t)w * K::FLK;
  uint32_t cnt = 0;
  int anynew = 0;
  for (uint32_t wd = threadIdx.x; wd < K::FLK; wd += BLOCK) {
    uint32_t m = pres[wd], kw = 0;
    const uint32_t fw = flk[wd];
    while (m) {
      const uint32_t b = __ffs(m) - 1;
      m &= m - 1;
      const uint32_t r = tab[nw_index<SB>(32 * wd + b)];
      const bool old = r == (uint32_t)gb;
      if (!old && ((fw >> b) & 1u)) continue;  // a flake no table holds: never new, never kept
      kw |= 1u << b;
      if (!old) {
        anynew = 1;
        const uint64_t lr = (uint64_t)r - gb;
        if (lr < span) {
          const uint32_t bit = 1u << (lr & 31);
          if (!(bm[lr >> 5] & bit)) atomicOr(&bm[lr >> 5], bit);
        } else {
          sel8[r] = 1;
        }
      }
    }
    kb32[wd] = kw;
    cnt += (uint32_t)__popc(kw);
  }
  const uint32_t tot = block_sum<BLOCK>(cnt, red);
  if (threadIdx.x == 0) wcount[gl.sbase + w] = tot;
  if (__syncthreads_or(anynew) && threadIdx.x == 0) upd[g] = 1;
  for (uint32_t i = threadIdx.x; i < words; i += BLOCK) {
    uint32_t v = bm[i];
    while (v) {
      const uint32_t b = __ffs(v) - 1;
      sel8[gb + 32ull * i + b] = 1;
      v &= v - 1;
    }
  }
}

// fstart[w] = the first flake at or above direct-size window w's first address (w in [0, W]; nfl past
// the span)
__global__ void k_nw_fstart(const uint32_t* fl, uint64_t nfl, uint32_t lo, uint32_t W, uint32_t sb, uint32_t* fstart) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w <= W; w += gridDim.x * blockDim.x) {
    const uint64_t a = (uint64_t)lo + ((uint64_t)w << sb);
    fstart[w] = a > 0xFFFFFFFFull ? (uint32_t)nfl : (uint32_t)lower_bound_dev<uint32_t>(fl, 0, nfl, (uint32_t)a);
  }
}

// the last slot of every call: its table's 0xFFFFFFFF stays unless the call took a Union (Union goes
// through foreach, cover.go:81-102)
__global__ void k_nw_sent(const uint8_t* has_sent, const uint8_t* upd, const NwGroup* ng_, uint32_t G, uint32_t* wcount) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x)
    wcount[ng_[g + 1].sbase - 1] = has_sent[g] && !upd[g] ? 1u : 0u;
}

// ---- wide spans: hashed windows -----------------------------------------------------------------
// When the span does not fit 1024 direct windows, every call gets its own window size (2^S addresses,
// S in [15, 26], about NW_HTARGET PCs per window, <= 1024 windows) and a workgroup per (call, window)
// keeps an open-addressing table in LDS: key = window offset, value = min member position. The
// window's offsets are done in R contiguous address sub-ranges (R a power of two, doubled and the
// unfinished sub-ranges redone when a probe run exceeds HPROBE), so each round's kept keys, sorted in
// LDS (bitonic), extend the window's PC-ordered kept list at hkeys[hbase[slot]]: no bitmap of 2^S bits.
constexpr uint32_t NW_HTARGET = 8192;
constexpr int NH_BLOCK = 512;             // two workgroups per CU (74 KB of LDS each)
constexpr uint32_t NH_PER = HS / NH_BLOCK;  // table slots per thread at compaction
constexpr uint32_t NH_FLK = 256;         // flakes of a window kept in LDS for the lookup (more: global)
constexpr uint32_t NH_FHS = 2 * NH_FLK;  // ... as an open-addressing set of window offsets (half full at most;
                                         // 2 KB: two workgroups per CU)
__device__ __forceinline__ uint32_t nh_fslot(uint32_t o) { return (o * 0x9E3779B1u) >> (32 - 9); }
static_assert(NH_FHS == 512, "nh_fslot");
constexpr uint32_t NH_NB_BITS = 11;      // order buckets of a sub-range: 2048
constexpr uint32_t NH_NB = 1u << NH_NB_BITS;
constexpr uint32_t NH_BSCAN = 64;        // keys of a bucket placed by a scan of it; more: the sort
static_assert(NH_NB + HS <= 2 * HS && NH_NB % NH_BLOCK == 0, "bucket counts and list in the table's space");

__device__ __forceinline__ uint32_t hslot_nw(uint32_t o) { return (o * 0x9E3779B1u) >> (32 - HS_BITS); }

// the call of count slot `slot`: the last g with sbase <= slot
__device__ __forceinline__ uint32_t nw_slot_group(const NwGroup* ng_, uint32_t G, uint64_t slot) {
  uint32_t g0 = 0, g1 = G;
  while (g1 - g0 > 1) {
    const uint32_t mid = (g0 + g1) >> 1;
    if (ng_[mid].sbase <= slot)
      g0 = mid;
    else
      g1 = mid;
  }
  return g0;
}

// capacity of every count slot's kept list (its window's PCs; 0 for the table-sentinel slot)
__global__ void k_nw_hcap(const NwGroup* ng_, const SGroup* sg, const uint32_t* wtot, uint32_t G, uint64_t slots,
                          uint32_t* hcap) {
  for (uint64_t sl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; sl < slots; sl += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = nw_slot_group(ng_, G, sl);
    const uint32_t w = (uint32_t)(sl - ng_[g].sbase);
    hcap[sl] = w < sg[g].W && sg[g].wbase != SG_NO_WTOT ? wtot[sg[g].wbase + w] : 0u;  // (direct windows: none)
  }
}

// M (hashed): item i is window i - iofs[j] of call order[j] (larger calls first)
__global__ __launch_bounds__(NH_BLOCK) void k_nw_hash(const uint32_t* order, const uint32_t* iofs, uint32_t G,
                                                  const SGroup* sg, const uint32_t* gslab, const uint64_t* gebase,
                                                  const uint32_t* D, const PSlab* slabs, const uint32_t* wtot,
                                                  const uint32_t* elems, const uint64_t* cstart, uint32_t lo,
                                                  const uint32_t* __restrict__ fl, uint64_t nfl, const NwGroup* ng_,
                                                  const uint64_t* hbase, uint32_t* hkeys, uint32_t* wcount,
                                                  uint8_t* sel8, uint8_t* upd, int* err, int dbg) {
  __shared__ uint32_t tabs[2 * HS];  // keys, values; then the sub-range's kept-offset bitmap
  __shared__ uint32_t bm[HBM_WORDS];
  __shared__ uint32_t red[NH_BLOCK / 64 + 1];
  __shared__ uint32_t fhs[NH_FHS];  // the window's flakes as offsets (when they fit): a hash set
  __shared__ int full;
  constexpr uint32_t NH_WBLK = 128;  // the walk's element windows: 8K elements (its scratch fits beside)
  __shared__ uint32_t wsc[2 * NH_BLOCK + 3 * NH_WBLK];
  __shared__ uint64_t red64[NH_BLOCK / 64 + 1];
  __shared__ uint32_t bmax;  // the largest order bucket of the sub-range
  uint32_t* keys = tabs;
  uint32_t* vals = tabs + HS;
  const uint32_t j = (uint32_t)upper_bound_dev<uint32_t>(iofs, 0, G + 1, blockIdx.x) - 1;
  const uint32_t g = order[j], w = blockIdx.x - iofs[j];
  const PItem it{g, w};
  const uint32_t S = sg[g].S;
  const uint64_t gb = cstart[g], ng = cstart[g + 1] - gb;
  const uint64_t slot = ng_[g].sbase + w;
  const uint32_t E = wtot[sg[g].wbase + w];
  if (E == 0) {
    if (threadIdx.x == 0) wcount[slot] = 0;
    return;
  }
  // the flakes inside the window's addresses [wlo, wlo + 2^S)
  const uint32_t wlo = lo + (w << S);
  const uint64_t whi = (uint64_t)wlo + (1ull << S);
  const uint64_t f0 = lower_bound_dev<uint32_t>(fl, 0, nfl, wlo);
  const uint64_t f1 = whi > 0xFFFFFFFFull ? nfl : lower_bound_dev<uint32_t>(fl, f0, nfl, (uint32_t)whi);
  const bool flds = f1 - f0 <= NH_FLK;  // searched in LDS, else in the global list
  const uint32_t nf = flds ? (uint32_t)(f1 - f0) : 0u;
  // (a set, not a sorted list searched per key: most keys of a batch are new, and each one's binary
  // search was a chain of dependent LDS reads)
  for (uint32_t i = threadIdx.x; i < NH_FHS; i += NH_BLOCK) fhs[i] = 0xFFFFFFFFu;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nf; i += NH_BLOCK) {
    const uint32_t o = fl[f0 + i] - wlo;  // < 2^S <= 2^26: never the empty mark
    for (uint32_t h = nh_fslot(o);; h = (h + 1) & (NH_FHS - 1)) {
      const uint32_t prev = atomicCAS(&fhs[h], 0xFFFFFFFFu, o);
      if (prev == 0xFFFFFFFFu || prev == o) break;
    }
  }
  const uint32_t span = (uint32_t)min<uint64_t>((uint64_t)HBM_WORDS * 32, ng);
  const uint32_t words = (span + 31) / 32;
  for (uint32_t i = threadIdx.x; i < words; i += NH_BLOCK) bm[i] = 0;
  uint32_t* out = hkeys + hbase[slot];
  uint32_t lr2 = 0;  // log2 R: one round unless the table fills
  uint32_t kc = 0;
  int anynew = 0;
  for (uint32_t round = 0; round < (1u << lr2);) {
    for (uint32_t i = threadIdx.x; i < HS; i += NH_BLOCK) {
      keys[i] = 0xFFFFFFFFu;
      vals[i] = RANK_NONE;
    }
    if (threadIdx.x == 0) full = 0;
    __syncthreads();
    const uint32_t sh = S - lr2, rr = round;
    const bool split = lr2 > 0;
    uint32_t acc = 0;
    for_slab_window<SYZ_NW_U, true, NH_WBLK>(it, sg, gslab, gebase, D, slabs, elems, nullptr, wsc, red64,
                                             [&](uint32_t o, uint32_t R) {
      if (R == RANK_NONE || (split && (o >> sh) != rr)) return;
      if (dbg & 1) {
        acc += o ^ R;
        return;
      }
      uint32_t h = hslot_nw(o);
      for (uint32_t probes = 0; probes < HPROBE; probes++) {
        uint32_t k = keys[h];
        if (k == 0xFFFFFFFFu) {
          k = atomicCAS(&keys[h], 0xFFFFFFFFu, o);
          if (k == 0xFFFFFFFFu) k = o;
        }
        if (k == o) {
          if (vals[h] > R) atomicMin(&vals[h], R);
          return;
        }
        h = (h + 1) & (HS - 1);
      }
      full = 1;
    });
    if (acc == 0x9E3779B9u) sel8[0] = 1;
    __syncthreads();
    if (dbg & 2) return;
    if (full) {  // twice the sub-ranges; the finished ones stay done
      if (lr2 == S) {
        if (threadIdx.x == 0) atomicOr(err, 32);
        return;
      }
      lr2++;
      round *= 2;
      __syncthreads();
      continue;
    }
    // the kept keys of this sub-range: held by the table, or by a cover when not a flake
    uint32_t kk[NH_PER];
    bool kp[NH_PER];
#pragma unroll
    for (uint32_t q = 0; q < NH_PER; q++) {
      const uint32_t i = threadIdx.x + q * NH_BLOCK;
      kp[q] = false;
      kk[q] = keys[i];
      if (kk[q] == 0xFFFFFFFFu) continue;
      const uint32_t v = vals[i];
      const bool old = v == (uint32_t)gb;
      if (!old && f1 > f0) {  // a flake no table holds: never new, never kept
        const uint32_t pc = wlo + kk[q];
        if (flds) {
          bool isf = false;
          for (uint32_t h = nh_fslot(kk[q]);; h = (h + 1) & (NH_FHS - 1)) {
            const uint32_t x = fhs[h];
            if (x == kk[q]) isf = true;
            if (x == kk[q] || x == 0xFFFFFFFFu) break;
          }
          if (isf) continue;
        } else {
          const uint64_t x = lower_bound_dev<uint32_t>(fl, f0, f1, pc);
          if (x < f1 && fl[x] == pc) continue;
        }
      }
      kp[q] = true;
      if (!old && !(dbg & 4)) {
        anynew = 1;
        const uint64_t lr = (uint64_t)v - gb;
        if (lr < span) {
          const uint32_t bit = 1u << (lr & 31);
          if (!(bm[lr >> 5] & bit)) atomicOr(&bm[lr >> 5], bit);
        } else {
          sel8[v] = 1;
        }
      }
    }
    __syncthreads();  // the table is read: its space takes the order
    if (dbg & 8) {  // timing only: no order, no output
      round++;
      continue;
    }
    // Order: 2048 buckets by the top address bits of the sub-range (counts, a scan, the keys listed
    // by bucket), then a key's place = its bucket's start + the keys of its bucket below it (buckets
    // hold a few keys: PCs are spread over the window's addresses)
    uint32_t* bcnt = tabs;               // [NH_NB] keys per bucket, then their starts
    uint32_t* blist = tabs + NH_NB;      // [HS] the keys, bucket by bucket
    const uint32_t bsh = sh > NH_NB_BITS ? sh - NH_NB_BITS : 0u;
    const uint32_t sbase = split ? rr << sh : 0u;
    for (uint32_t i = threadIdx.x; i < NH_NB; i += NH_BLOCK) bcnt[i] = 0;
    if (threadIdx.x == 0) bmax = 0;
    __syncthreads();
    uint32_t pib[NH_PER];  // place inside the bucket, or none
#pragma unroll
    for (uint32_t q = 0; q < NH_PER; q++)
      pib[q] = kp[q] ? atomicAdd(&bcnt[(kk[q] - sbase) >> bsh], 1u) : 0xFFFFFFFFu;
    __syncthreads();
    {
      constexpr uint32_t PERB = NH_NB / NH_BLOCK;  // buckets per thread
      uint32_t x[PERB], c = 0, mx = 0;
#pragma unroll
      for (uint32_t k = 0; k < PERB; k++) {
        x[k] = bcnt[threadIdx.x * PERB + k];
        c += x[k];
        mx = max(mx, x[k]);
      }
      if (mx > NH_BSCAN || (dbg & 16)) atomicMax(&bmax, mx + 1);
      uint32_t nk;
      uint32_t pre = block_excl_scan<NH_BLOCK>(c, red, &nk);
#pragma unroll
      for (uint32_t k = 0; k < PERB; k++) {
        bcnt[threadIdx.x * PERB + k] = pre;
        pre += x[k];
      }
      __syncthreads();
#pragma unroll
      for (uint32_t q = 0; q < NH_PER; q++)
        if (pib[q] != 0xFFFFFFFFu) blist[bcnt[(kk[q] - sbase) >> bsh] + pib[q]] = kk[q];
      __syncthreads();
      if (bmax == 0) {  // every bucket holds a few keys: a key's place by a scan of its bucket
#pragma unroll
        for (uint32_t q = 0; q < NH_PER; q++)
          if (pib[q] != 0xFFFFFFFFu) {
            const uint32_t bk = (kk[q] - sbase) >> bsh;
            const uint32_t b0 = bcnt[bk], b1 = bk + 1 < NH_NB ? bcnt[bk + 1] : nk;
            uint32_t r = b0;
            for (uint32_t i = b0; i < b1; i++) r += blist[i] < kk[q] ? 1u : 0u;
            out[kc + r] = kk[q];
          }
      } else {  // clustered PCs (a bucket past NH_BSCAN keys): a bitonic sort of the sub-range's keys
        uint32_t P = 64;
        while (P < nk) P <<= 1;
        for (uint32_t i = nk + threadIdx.x; i < P; i += NH_BLOCK) blist[i] = 0xFFFFFFFFu;
        __syncthreads();
        for (uint32_t k = 2; k <= P; k <<= 1)
          for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            for (uint32_t t = threadIdx.x; t < P / 2; t += NH_BLOCK) {
              const uint32_t i = ((t & ~(jj - 1)) << 1) | (t & (jj - 1)), ij = i | jj;
              const uint32_t a = blist[i], b = blist[ij];
              if ((a > b) == ((i & k) == 0)) {
                blist[i] = b;
                blist[ij] = a;
              }
            }
            __syncthreads();
          }
        for (uint32_t i = threadIdx.x; i < nk; i += NH_BLOCK) out[kc + i] = blist[i];
      }
      kc += nk;
    }
    round++;
    __syncthreads();
  }
  if (threadIdx.x == 0) wcount[slot] = kc;
  if (__syncthreads_or(anynew) && threadIdx.x == 0) upd[g] = 1;
  for (uint32_t i = threadIdx.x; i < words; i += NH_BLOCK) {
    uint32_t v = bm[i];
    while (v) {
      const uint32_t b = __ffs(v) - 1;
      sel8[gb + 32ull * i + b] = 1;
      v &= v - 1;
    }
  }
}

// E: one slot per workgroup; the window's kept bitmap (or, hashed windows, its sorted kept offsets at
// hkeys[hbase[slot]]) -> its PCs at wpos[slot]
__global__ __launch_bounds__(NE_BLOCK) void k_nw_emit(const uint32_t* __restrict__ kbits,
                                                      const uint64_t* __restrict__ wpos, const NwGroup* ng_,
                                                      const PGroup* pg, uint32_t G, uint32_t lo, uint32_t* out,
                                                      uint64_t cap, uint64_t* ooff, int* err,
                                                      const uint64_t* __restrict__ hbase,
                                                      const uint32_t* __restrict__ hkeys) {
  __shared__ uint32_t red[NE_BLOCK / 64 + 1];
  const uint64_t slot = blockIdx.x;
  const uint32_t g = nw_slot_group(ng_, G, slot);
  const NwGroup gl = ng_[g];
  const uint32_t w = (uint32_t)(slot - gl.sbase), W = pg[g].W, S = pg[g].S;
  const uint64_t p0 = wpos[slot], c = wpos[slot + 1] - p0;
  if (threadIdx.x == 0 && w == 0) {
    ooff[g] = p0;
    if (g + 1 == G) ooff[G] = wpos[ng_[G].sbase];
  }
  if (c == 0) return;
  if (p0 + c > cap) {
    if (threadIdx.x == 0) atomicOr(err, 8);
    return;
  }
  if (w == W) {
    if (threadIdx.x == 0) out[p0] = SENT;
    return;
  }
  if (hbase && pg[g].mode == PMODE_HASH) {
    const uint32_t wlo = lo + (w << S);
    const uint32_t* src = hkeys + hbase[slot];
    for (uint64_t i = threadIdx.x; i < c; i += NE_BLOCK) out[p0 + i] = wlo + src[i];
    return;
  }
  const uint32_t q = (1u << S) / 32 / NE_BLOCK;  // words per thread (2 .. 16)
  const uint32_t* kb = kbits + gl.kbase + (uint64_t)w * ((1u << S) / 32) + (uint64_t)threadIdx.x * q;
  uint32_t pc = 0;
  for (uint32_t i = 0; i < q; i++) pc += (uint32_t)__popc(kb[i]);
  uint32_t tot;
  uint64_t p = p0 + block_excl_scan<NE_BLOCK>(pc, red, &tot);
  const uint32_t a0 = lo + (w << S) + 32u * q * threadIdx.x;
  for (uint32_t i = 0; i < q; i++) {
    uint32_t m = kb[i];
    while (m) {
      const uint32_t b = __ffs(m) - 1;
      m &= m - 1;
      out[p++] = a0 + 32u * i + b;
    }
  }
}

__global__ void k_nw_isnew(const uint32_t* cmem, const uint8_t* sel8, size_t nm, uint32_t n1, uint8_t* is_new) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nm; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t e = cmem[i];
    if (e < n1) is_new[e] = sel8[i];
  }
}

// timing experiments only (results are wrong when set): SYZGPU_NW_DBG 1 = tables not walked, 2 = no emit
static int nw_dbg() {
  static const int v = dev_env("SYZGPU_NW_DBG") ? atoi(dev_env("SYZGPU_NW_DBG")) : 0;
  return v;
}

// timing experiments only (results are wrong when set): SYZGPU_NWH_DBG 1 = hashed windows walked
// without table updates, 2 = tables built, nothing after, 4 = no new-cover marks, 8 = no ordered
// output
static int nwh_dbg() {
  static const int v = dev_env("SYZGPU_NWH_DBG") ? atoi(dev_env("SYZGPU_NWH_DBG")) : 0;
  // SYZGPU_NWH_SORT=1 (read per call; results unchanged): every sub-range ordered by the sort
  const char* so = getenv("SYZGPU_NWH_SORT");
  return v | (so && atoi(so) ? 16 : 0);
}

// SYZGPU_NW_BITS=14|15: direct window bits (default: 14 while the span fits 1024 such windows, else 15;
// 13-bit windows measured slower, r05: 5.83 vs 4.61 ms at config 3)
// Inside a span that fits direct windows, the calls with fewer than NW_HSPARSE PCs per direct window
// take hashed windows: a direct window's fixed costs (its 64 KB table cleared and scanned, a 2 KB
// bitmap out, one run per slab of the call) outweigh its few elements there. Config 3 (r05_novmix2):
// 4.30 ms all direct; 256 4.35, 512 4.09, 1024 3.92 ms. SYZGPU_NW_HSPARSE=t overrides (0: all direct).
constexpr uint64_t NW_HSPARSE = 1024;
static uint64_t nw_hsparse() {
  static const uint64_t v =
      dev_env("SYZGPU_NW_HSPARSE") ? (uint64_t)atoll(dev_env("SYZGPU_NW_HSPARSE")) : NW_HSPARSE;
  return v;
}

static uint32_t nw_bits_forced() {
  static const uint32_t v = dev_env("SYZGPU_NW_BITS") ? (uint32_t)atoi(dev_env("SYZGPU_NW_BITS")) : 0u;
  return v == 14 || v == 15 ? v : 0u;
}

__global__ void k_nw_gpcs(const uint64_t* mpos, const uint64_t* cstart, uint32_t G, uint64_t* gpcs) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x)
    gpcs[g] = mpos[cstart[g + 1]] - mpos[cstart[g]];
}

// Direct windows while the span fits 1024 of them, else (or force_hash) hashed windows. false: G is
// too large (or the batch too long) for the windows: use another strategy. err gets novelty.hip's bits
// (1 table, 2 group id, 4 cover, 8 capacity, 32 internal).
bool novelty_windows(const uint32_t* d_pcs, const uint64_t* d_off, const uint32_t* d_grp, size_t n, uint32_t G,
                     const uint32_t* d_mc, const uint64_t* d_mco, const uint32_t* d_fl, size_t nfl, uint8_t* d_new,
                     uint32_t* d_out, size_t out_cap, uint64_t* d_ooff, int* err, bool force_hash, hipStream_t s) {
  if (G == 0 || G > MAX_GROUPS_PM || (uint64_t)n + G >= 0xFFFFFFF0ull) return false;
  Context& c = ctx();
  Scratch& sc = c.scratch;
  const size_t nm = n + G;
  uint64_t* gstart = sc.get<uint64_t>("nw_gstart", G + 1);
  uint64_t* cstart = sc.get<uint64_t>("nw_cstart", G + 1);
  uint32_t* members = sc.get<uint32_t>("mz_members", n + 1);
  uint64_t* el = sc.get<uint64_t>("mz_el", n + 1);
  uint32_t* cmem = sc.get<uint32_t>("nw_cmem", nm + 1);
  uint32_t* mlen = sc.get<uint32_t>("nw_mlen", nm + 1);
  uint32_t* elen = sc.get<uint32_t>("nw_elen", nm + 1);
  uint64_t* mpos = sc.get<uint64_t>("nw_mpos", nm + 1);
  uint8_t* has_sent = sc.get<uint8_t>("nw_has_sent", G + 1);
  uint8_t* upd = sc.get<uint8_t>("nw_upd", G + 1);
  uint32_t* span = sc.get<uint32_t>("nw_span", 4);
  int* perr = sc.get<int>("nw_perr", 2);
  uint8_t* sel8 = sc.get<uint8_t>("nw_sel8", nm + 1);
  k_nw_init<<<grid_for(nm + 1, 256, 1024), 256, 0, s>>>(perr, has_sent, upd, G, sel8, nm + 1, span);
  SYZ_LAUNCHED();
  {
    ProfScope ps("novelty_group", s, (uint64_t)n * 28 + (uint64_t)nm * 24);
    group_partition_dev(d_grp, d_off, n, G, gstart, members, el, perr, s);
    k_nw_meta<<<grid_for(nm, 256, 4096), 256, 0, s>>>(d_pcs, d_off, d_mc, d_mco, n, G, elen, has_sent, span);
    SYZ_LAUNCHED();
    k_nw_members<<<grid_for(std::max<size_t>(n, G + 1), 256, 8192), 256, 0, s>>>(members, gstart, d_grp, n, G, elen,
                                                                                 cmem, cstart, mlen);
    SYZ_LAUNCHED();
    exclusive_scan_u32(mlen, mpos, nm, s);
  }
  uint64_t* gpcs = sc.get<uint64_t>("nw_gpcs", G + 1);
  k_nw_gpcs<<<grid_for(G, 256, 64), 256, 0, s>>>(mpos, cstart, G, gpcs);
  SYZ_LAUNCHED();
  uint64_t* hbuf = c.pinned.get<uint64_t>(2 * (size_t)G + 8);
  SYZ_HIP(hipMemcpyAsync(hbuf, cstart, (G + 1) * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hbuf + G + 1, mpos + nm, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hbuf + G + 2, span, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hbuf + G + 3, perr, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hbuf + G + 4, gpcs, G * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (*reinterpret_cast<int*>(hbuf + G + 3)) fail(SYZGPU_EINVAL, "group id >= ngroups");
  const std::vector<uint64_t> hstart(hbuf, hbuf + G + 1), hpcs(hbuf + G + 4, hbuf + 2 * G + 4);
  const uint64_t total = hbuf[G + 1];
  uint32_t lo = reinterpret_cast<uint32_t*>(hbuf + G + 2)[0], hi = reinterpret_cast<uint32_t*>(hbuf + G + 2)[1];
  if (lo > hi) lo = hi = 0;  // no PCs outside the sentinel
  lo &= ~((1u << 15) - 1);  // windows on 2^15 boundaries: a window's addresses never wrap
  auto nwin = [&](uint32_t sb) { return (((uint64_t)hi - lo) >> sb) + 1; };
  uint32_t DB = nw_bits_forced();
  if (!DB) DB = nwin(14) <= WMAX ? 14 : 15;
  const bool hashed = force_hash || nwin(DB) > WMAX;  // every call on hashed windows
  uint32_t smin = 15;  // hashed windows: the narrowest size whose windows fit WMAX
  while (nwin(smin) > WMAX) smin++;
  const uint32_t WD = hashed ? 0u : (uint32_t)nwin(DB);
  const uint64_t hsparse = nw_hsparse();
  // ---- plan: direct — a call on WD windows of 2^DB addresses; hashed — a window size per call (about
  // NW_HTARGET PCs per window): every call when the span is too wide for direct windows, else the calls
  // with fewer than hsparse PCs per direct window (SYZGPU_NW_HSPARSE); regions, blocks, work items ----
  std::vector<PGroup> hpg(G);
  std::vector<NwGroup> hng(G + 1);
  uint64_t kw = 0, slots = 0;
  bool any_hash = false, any_direct = false;
  for (uint32_t g = 0; g < G; g++) {
    uint32_t S = DB, W = WD;
    const bool hg = hashed || hpcs[g] < hsparse * WD;
    any_hash |= hg;
    any_direct |= !hg;
    if (hg) {
      const uint64_t want = std::max<uint64_t>(1, std::min<uint64_t>(WMAX, (hpcs[g] + NW_HTARGET - 1) / NW_HTARGET));
      S = smin;
      while (S < SMAX && nwin(S + 1) >= want) S++;
      W = (uint32_t)nwin(S);
    }
    hpg[g] = PGroup{S, W, (uint32_t)(hg ? PMODE_HASH : PMODE_DIRECT), 0};
    hng[g] = NwGroup{kw, slots};
    if (!hg) kw += (uint64_t)W << (S - 5);
    slots += W + 1;
  }
  hng[G] = NwGroup{kw, slots};
  // slabs of the combined members (slab_dev.hpp); hashed windows need their per-window totals
  SlabJob SJ;
  slab_plan(SJ, hstart, hpcs.data(), hpg, G, any_hash);
  const uint32_t B = SJ.B;
  // items (call, window), larger calls first (their windows are the long ones) so the grid's tail is
  // short. order = the direct calls (Gd), then the hashed ones (Gh); direct item i is window i % WD of
  // call order[i / WD]; hashed item i is window i - iofs[j] of call order[Gd + j]
  std::vector<uint32_t> order(G);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
    const bool hx = hpg[x].mode == PMODE_HASH, hy = hpg[y].mode == PMODE_HASH;
    return hx != hy ? hy : hpcs[x] > hpcs[y];
  });
  uint32_t Gd = 0;
  while (Gd < G && hpg[order[Gd]].mode == PMODE_DIRECT) Gd++;
  const uint32_t Gh = G - Gd;
  std::vector<uint32_t> iofs(G + 1, 0);  // hashed: the items of order[Gd + j] are [iofs[j], iofs[j + 1])
  for (uint32_t j = 0; j < Gh; j++) iofs[j + 1] = iofs[j] + hpg[order[Gd + j]].W;
  const size_t nitems_d = (size_t)Gd * WD, nitems_h = iofs[Gh];
  // one staging copy: PGroup[G+1], NwGroup[G+1], SGroup[G+1], gblock[G+1], bgroup[B+1], order[G+1], iofs[G+1]
  auto al16 = [](size_t x) { return (x + 15) & ~size_t(15); };
  const size_t o_ng = al16((G + 1) * sizeof(PGroup)), o_sg = o_ng + al16((G + 1) * sizeof(NwGroup));
  const size_t o_gb = o_sg + al16((G + 1) * sizeof(SGroup)), o_bg = o_gb + al16((G + 1) * 4);
  const size_t o_or = o_bg + al16(((size_t)B + 1) * 4), o_io = o_or + al16((G + 1) * 4);
  const size_t stage_bytes = o_io + al16((G + 1) * 4);
  uint8_t* stage = c.pinned.get<uint8_t>(stage_bytes + 64);
  uint8_t* dstage = sc.get<uint8_t>("nw_stage", stage_bytes + 64);
  std::memcpy(stage, hpg.data(), G * sizeof(PGroup));
  std::memcpy(stage + o_ng, hng.data(), (G + 1) * sizeof(NwGroup));
  std::memcpy(stage + o_sg, SJ.hsg.data(), G * sizeof(SGroup));
  std::memcpy(stage + o_gb, SJ.hgblock.data(), (G + 1) * 4);
  if (B) std::memcpy(stage + o_bg, SJ.hbgroup.data(), (size_t)B * 4);
  std::memcpy(stage + o_or, order.data(), G * 4);
  std::memcpy(stage + o_io, iofs.data(), (G + 1) * 4);
  SYZ_HIP(hipMemcpyAsync(dstage, stage, stage_bytes, hipMemcpyHostToDevice, s));
  const PGroup* dpg = reinterpret_cast<const PGroup*>(dstage);
  const NwGroup* dng = reinterpret_cast<const NwGroup*>(dstage + o_ng);
  const SGroup* dsg = reinterpret_cast<const SGroup*>(dstage + o_sg);
  SJ.dsg = dsg;
  SJ.dgblock = reinterpret_cast<const uint32_t*>(dstage + o_gb);
  SJ.dbgroup = reinterpret_cast<const uint32_t*>(dstage + o_bg);
  const uint32_t* dorder = reinterpret_cast<const uint32_t*>(dstage + o_or);
  const uint32_t* diofs = reinterpret_cast<const uint32_t*>(dstage + o_io);
  uint32_t* kbits = sc.get<uint32_t>("nw_kbits", kw + 1);
  uint32_t* wcount = sc.get<uint32_t>("nw_wcount", slots + 1);
  uint64_t* wpos = sc.get<uint64_t>("nw_wpos", slots + 1);
  {
    // byte model (as the Minimize transpose's): every PC read once + 10 B per member
    // (offset, group id); the element buffer it writes is intermediate traffic, not algorithmic bytes
    ProfScope ps("novelty_part", s, total * 4 + (uint64_t)nm * 10);
    slab_build(SJ, "nw", mlen, mpos, nm, cstart, s);
    NovSrc ns;
    ns.mc = d_mc;
    ns.mc_off = d_mco;
    ns.n1 = (uint32_t)n;
    if (SJ.slab_bound) {
      launch_slab<true>(SJ.slab_bound, SJ.wmax, s, d_pcs, d_off, cmem, mlen, SJ.tpos, nullptr, SJ.slabs, SJ.cstart + B,
                        dsg, SJ.gebase, lo, SJ.elems, SJ.ecap, SJ.D, err, SJ.wtot, ns, 0);
      SYZ_LAUNCHED();
    }
  }
  const uint32_t* gslab = SJ.gslab;
  const uint64_t* gebase = SJ.gebase;
  const uint32_t* D = SJ.D;
  const PSlab* slabs = SJ.slabs;
  const uint32_t* elems = SJ.elems;
  uint64_t* hbase = nullptr;
  uint32_t* hkeys = nullptr;
  if (any_hash) {
    ProfScope ps("novelty_min_hash", s, total * 8 + slots * 20);
    uint32_t* hcap = sc.get<uint32_t>("nw_hcap", slots + 1);
    hbase = sc.get<uint64_t>("nw_hbase", slots + 1);
    hkeys = sc.get<uint32_t>("nw_hkeys", total + 8);
    k_nw_hcap<<<grid_for(slots, 256, 4096), 256, 0, s>>>(dng, dsg, SJ.wtot, G, slots, hcap);
    SYZ_LAUNCHED();
    exclusive_scan_u32(hcap, hbase, slots, s);
    if (nitems_h) {
      k_nw_hash<<<(unsigned)nitems_h, NH_BLOCK, 0, s>>>(dorder + Gd, diofs, Gh, dsg, gslab, gebase, D, slabs, SJ.wtot, elems,
                                                      cstart, lo, d_fl, nfl, dng, hbase, hkeys, wcount, sel8, upd, err,
                                                      nwh_dbg());
      SYZ_LAUNCHED();
    }
  }
  uint32_t* fstart = sc.get<uint32_t>("nw_fstart", (size_t)WD + 2);
  if (any_direct) {
    ProfScope ps("novelty_min", s, total * 4 + kw * 4);
    k_nw_fstart<<<grid_for(WD + 1, 256, 64), 256, 0, s>>>(d_fl, nfl, lo, WD, DB, fstart);
    SYZ_LAUNCHED();
    if (nitems_d) {
      if (DB == 14)
        k_nw_min<14><<<(unsigned)nitems_d, NwCfg<14>::BLOCK, 0, s>>>(dorder, WD, dsg, gslab, gebase, D, slabs, elems,
                                                                   cstart, lo, d_fl, fstart, dng, kbits, wcount, sel8,
                                                                   upd, nw_dbg());
      else
        k_nw_min<15><<<(unsigned)nitems_d, NwCfg<15>::BLOCK, 0, s>>>(dorder, WD, dsg, gslab, gebase, D, slabs, elems,
                                                                   cstart, lo, d_fl, fstart, dng, kbits, wcount, sel8,
                                                                   upd, nw_dbg());
      SYZ_LAUNCHED();
    }
  }
  {
    ProfScope ps("novelty_emit", s, kw * 4 + (uint64_t)nm * 6);
    k_nw_sent<<<grid_for(G, 256, 64), 256, 0, s>>>(has_sent, upd, dng, G, wcount);
    SYZ_LAUNCHED();
    exclusive_scan_u32(wcount, wpos, slots, s);
    k_nw_emit<<<(unsigned)slots, NE_BLOCK, 0, s>>>(kbits, wpos, dng, dpg, G, lo, d_out, out_cap, d_ooff, err, hbase,
                                                   hkeys);
    SYZ_LAUNCHED();
    k_nw_isnew<<<grid_for(nm, 256, 8192), 256, 0, s>>>(cmem, sel8, nm, (uint32_t)n, d_new);
    SYZ_LAUNCHED();
  }
  return true;
}

}  // namespace syz

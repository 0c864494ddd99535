// minimizeCorpus from raw covers in HBM (syz-manager/manager.go:507-527 over cover/cover.go:105-131),
// every step from the covers themselves: no dictionary or store built ahead of time.
//
// Minimize keeps input k (Go-sort position k of its call group) iff some PC of its cover first occurs
// at k, so the work is a min-rank per (call, PC) key. Keys are split by PC value into
// windows so that each key's min fits a workgroup's LDS, and the covers are transposed into those
// windows by one streaming pass:
//
//   P  (k_part)  a workgroup per chunk (<= 16384 PCs of <= 64 consecutive members of one call group):
//                window w = (pc - lo) >> S_g of every PC, histogram in LDS, the chunk's PCs rewritten
//                window-major through an LDS staging buffer as u32 elements (pc offset in the window |
//                member tag << S_g) and the window starts as a u16 row `desc` per chunk.
//   M  (k_pmin)  a workgroup per (call, window): every chunk's run of that window, min Go-sort rank per
//                offset in LDS — a direct-mapped 32K-entry table for dense calls (S = 15), an
//                open-addressing table for sparse ones (wider windows) — and the rank that wins a key
//                marks its input kept in a rank bitmap.
//
// P depends only on the covers, so it runs while gosort.hip computes the ranks; M waits for both.
// Selection order, kept flags, the len(p.Calls) histogram and the group-major kept list
// (syzgpu_minimize_grouped's output) are produced on the device in the same call.
// Integer work throughout: bit-exact by construction (F2); tests/test_gpu_raw.py checks every output.
#include <algorithm>
#include <array>
#include <cstdlib>
#include <memory>
#include <numeric>

#include "panels_dev.hpp"
#include "pipeline.hpp"
#include "slab_dev.hpp"

namespace syz {


// workgroups of k_span_sums: each adds its G per-group sums to gpcs with global atomics, G x blocks
// of them on G addresses; SYZGPU_SPAN_BLOCKS overrides (A/B)
static unsigned span_blocks() {
  const char* e = dev_env("SYZGPU_SPAN_BLOCKS");
  return e && *e ? (unsigned)std::max(1, atoi(e)) : 512u;
}

// ---- per-entry statistics: PCs per call group and the PC span --------------------------------------
// (*mlmax: the longest cover, which tells the Go sort whether a pack can need its u64 element)
// (gpcs may be null: the per-group sums come from the member prefix instead, no per-group atomics)
__global__ __launch_bounds__(256) void k_span_sums(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                   size_t n, uint32_t G, uint64_t* gpcs, uint32_t* span,
                                                   uint32_t* mlmax) {
  extern __shared__ unsigned long long lsum[];
  __shared__ uint32_t lmax;
  if (gpcs)
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) lsum[g] = 0;
  if (threadIdx.x == 0) lmax = 0;
  __syncthreads();
  uint32_t lo = 0xFFFFFFFFu, hi = 0, mx = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t a = off[i], b = off[i + 1];
    const uint32_t g = group[i];
    mx = max(mx, (uint32_t)min<uint64_t>(b - a, 0xFFFFFFFFull));
    if (b > a) {
      if (gpcs && g < G) atomicAdd(&lsum[g], (unsigned long long)(b - a));
      // covers are sorted (executor.cc:572-585): the first and last PC bound them; k_part checks
      // every PC against the resulting windows and the call is redone on exact bounds otherwise
      lo = min(lo, pcs[a]);
      hi = max(hi, pcs[b - 1]);
    }
  }
  if (mx) atomicMax(&lmax, mx);
  block_span_update<256>(lo, hi, span);  // (its barrier also completes lsum and lmax)
  if (gpcs)
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x)
      if (lsum[g]) atomicAdd((unsigned long long*)&gpcs[g], lsum[g]);
  if (threadIdx.x == 0 && lmax) atomicMax(mlmax, lmax);
}

// exact bounds (the slow path when some cover is not sorted)
__global__ __launch_bounds__(256) void k_minmax(const uint32_t* pcs, size_t L, uint32_t* span) {
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < L; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t v = pcs[i];
    lo = min(lo, v);
    hi = max(hi, v);
  }
  block_span_update<256>(lo, hi, span);
}

// the job's per-step state: error word, speculation gate (err[2]), per-group PC sums, the PC span
__global__ void k_pm_init(int* err, uint64_t* gpcs, uint32_t G, uint32_t* span, uint32_t* mlmax, uint32_t* mctr) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g <= max(G, 15u); g += gridDim.x * blockDim.x) {
    if (g < 16) mctr[g] = 0;  // M's item counters (m_items)
    if (g > G) continue;
    gpcs[g] = 0;
    if (g < 2) {
      err[g] = 0;
      span[g] = g ? 0u : 0xFFFFFFFFu;
    }
    if (g == 0) err[2] = 0;  // the speculation gate (k_gpack)
    if (g == 0) *mlmax = 0;
  }
}

// What the host plans the windows from, in one buffer (one copy back): gstart[G + 1], the PCs of each
// call group gpcs[G], the span, the error word, and the PCs of each call group this job reads (its
// members' slices: the exact byte model of the kernels) gsl[G]
// exp (a step speculated on a cached plan): the words the plan was made from, in the same places
// (the per-group PC sums at [G + 1, 2G] are not part of the plan's key; exp[2G + 2] = 0, exp[3G + 3] =
// may_bounce); any difference sets *gate, and the speculated P and M kernels then return at once (a
// stale plan's M could read D rows past their length), so a miss costs the Go sort's rounds, not a step.
__global__ void k_gpack(const uint64_t* gstart, const uint64_t* gpcs, const uint32_t* span, const int* err,
                        const uint64_t* mpos, uint32_t G, const uint32_t* mlmax, uint64_t* out,
                        const uint64_t* exp, int* gate) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < 3 * G + 4; i += gridDim.x * blockDim.x) {
    uint64_t v;
    if (i == 3 * G + 3)
      v = *mlmax;
    else if (i <= G)
      v = gstart[i];
    else if (i < 2 * G + 1)
      v = gpcs[i - G - 1];
    else if (i == 2 * G + 1)
      v = ((uint64_t)span[1] << 32) | span[0];
    else if (i == 2 * G + 2)
      v = ((uint64_t)(uint32_t)err[1] << 32) | (uint32_t)err[0];
    else {
      const uint32_t g = i - 2 * G - 3;
      v = mpos[gstart[g + 1]] - mpos[gstart[g]];
    }
    out[i] = v;
    if (exp && (i <= G || i > 2 * G)) {
      const uint64_t want = exp[i];
      const uint64_t got = i == 3 * G + 3 ? (uint64_t)(v >= GS_U32_LEN_LIMIT) : v;
      if (got != want) atomicOr(gate, 1);
    }
  }
}

// Winners of a window table -> the job's rank bitmap (bit r of selbits: rank r kept). A window's winners
// are deduplicated through an LDS bitmap aligned to the global words (the group's first BMW * 32 ranks
// from its first word), which leaves as one atomicOr per nonzero word; a winner past it goes straight to
// its global word. The atomics return nothing, so no wave waits for them (a read of the word first, to
// skip an atomic that is not needed, cost more than it saved: the read is waited for).
struct RankIdentity {
  __device__ uint32_t operator()(uint32_t v) const { return v; }
};
#ifndef SYZ_EMIT_RFIRST
#define SYZ_EMIT_RFIRST 0
#endif
#ifndef SYZ_SMIN_NOATOM
#define SYZ_SMIN_NOATOM 0  // timing experiment only (results wrong when 1): plain stores for the winner bits
#endif
__device__ __forceinline__ void set_bits(uint32_t* w, uint32_t bits) {
  if (SYZ_SMIN_NOATOM)
    *w = bits;
  else
    atomicOr(w, bits);
}
template <uint32_t BMW, class D = RankIdentity>
__device__ __forceinline__ void emit_winner_bits(const uint32_t* tab, uint32_t nids, uint64_t gbase, uint64_t ng,
                                                 uint32_t* bm, uint32_t* selbits, D decode = D{}) {
  const uint64_t base = gbase & ~31ull;  // rank of bitmap word 0, bit 0
  const uint32_t words = (uint32_t)min<uint64_t>(BMW, (gbase + ng - base + 31) / 32);
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) bm[i] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nids; i += blockDim.x) {
    const uint32_t r = decode(tab[i]);
    if (r == RANK_NONE) continue;
    const uint64_t lr = (uint64_t)r - base;
    const uint32_t bit = 1u << (r & 31);
    if (lr < 32ull * words) {
      if (!(bm[lr >> 5] & bit)) atomicOr(&bm[lr >> 5], bit);
    } else {
      set_bits(&selbits[r >> 5], bit);
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
    if (const uint32_t v = bm[i]) set_bits(&selbits[(base >> 5) + i], v);
  __syncthreads();
}


// The direct table's index: the offset rotated right by 2 bits inside the window, so PCs on 4-byte
// instruction boundaries (arm64, and the synthetic corpora) fill every LDS bank, not a quarter of them
__device__ __forceinline__ uint32_t tab_index(uint32_t o) { return ((o >> 2) | (o << (DS - 2))) & ((1u << DS) - 1); }
__device__ __forceinline__ uint32_t hslot(uint32_t o) { return (o * 0x9E3779B1u) >> (32 - HS_BITS); }

// ---- M over slab runs (slab_dev.hpp): the same tables, the window's runs from every slab --------------
#ifndef SYZ_SMIN_NOEMIT
#define SYZ_SMIN_NOEMIT 0  // timing experiment only (results wrong when 1)
#endif
#ifndef SYZ_SMIN_NOF
#define SYZ_SMIN_NOF 0  // timing experiment only (results wrong when 1)
#endif
#ifndef SYZ_SMIN_IDENT
#define SYZ_SMIN_IDENT false  // timing experiment only (results wrong when true)
#endif
#define SMIN_WALK(U, it, sg, gslab, gebase, D, slabs, elems, rom, wsc, red64, f) \
  for_slab_window<U, SYZ_SMIN_IDENT>(it, sg, gslab, gebase, D, slabs, elems, rom, wsc, red64, f)
// the direct tables' walk: the workgroup form (for_slab_window); SYZ_SMIN_WW=1: every wave on its own
// runs (slab_dev.hpp for_slab_window_w) — fewer cycles per workgroup, the same time at config 4 (2.559
// vs 2.535 ms) and 1 ms slower at config 5 (17.80 vs 16.76 ms, profiles/r06_ab/r06_ww5_pm.log): off
#ifndef SYZ_SMIN_WW
#define SYZ_SMIN_WW 0
#endif
#ifndef SYZ_SMIN_NBW
#define SYZ_SMIN_NBW 16
#endif
#ifndef SYZ_SMIN_WWP
#define SYZ_SMIN_WWP 0  // the packed tables' walk in the wave form too
#endif
constexpr uint32_t SMIN_NBW = SYZ_SMIN_NBW;
static_assert(16 * (128 + 3 * SMIN_NBW) <= 2 * 1024 + 3 * PK_NBLK, "the wave walk's maps in the walk scratch");
#ifndef SYZ_SL_MU
#define SYZ_SL_MU 2
#endif
#if SYZ_DS < 15
#define SYZ_SMIN_OCC __attribute__((amdgpu_waves_per_eu(8, 8)))  // 64 KB tables: two workgroups per CU
#else
#define SYZ_SMIN_OCC
#endif
// LDS of one M workgroup: the window's table (direct: 2^DS u32; hashed: keys + values or packed slots),
// the walk's scratch (then the emit bitmap) and reductions
template <int BLOCK, uint32_t TWORDS, uint32_t TOUCH, uint32_t NB>
struct SminLdsT {
  __align__(16) uint32_t tabs[TWORDS];
  __align__(16) uint32_t wsc[2 * BLOCK + 3 * NB];
  uint32_t touched[TOUCH];  // a bit per table entry / slot some element wrote (the emit walks only those)
  uint64_t red64[BLOCK / 64 + 1];
  int full;
  static constexpr uint32_t WSC = 2 * BLOCK + 3 * NB;
  static constexpr uint32_t NBLK = NB;  // the workgroup walk's blocks per element window
};
using SminLds = SminLdsT<1024, ((1u << DS) > 2 * HS ? (1u << DS) : 2 * HS), (1u << DS) / 32, PK_NBLK>;
// packed windows: their slots only; a 128-block walk window keeps four workgroups per CU
using SminPkLds = SminLdsT<PK_BLOCK, PHS, PHS / 32, 128>;
static_assert(sizeof(SminLds) <= 80 * 1024, "two direct-table workgroups per CU");
static_assert(sizeof(SminPkLds) + 16 <= 40 * 1024, "four packed-table workgroups per CU");
static_assert(HS / 32 <= (1u << DS) / 32, "the hashed table's touched bits in the direct table's");
static_assert(PHS <= 2 * HS, "packed slots in the key/value space");

// The direct table's winners -> the job's rank bitmap, like emit_winner_bits but over the touched entries
// only: a window holds a few thousand keys in 2^DS slots, so walking the 512 words of the touched bitmap
// and their set bits replaces a scan of every slot (r06: the full scan was 16 % of the kernel's cycles)
template <uint32_t BMW, class Dec = RankIdentity>
__device__ __forceinline__ void emit_touched(const uint32_t* tab, const uint32_t* touched, uint32_t ntw, uint64_t gbase,
                                             uint64_t ng, uint32_t* bm, uint32_t* selbits, Dec decode = Dec{}) {
  const uint64_t base = gbase & ~31ull;  // rank of bitmap word 0, bit 0
  // The LDS bitmap over the group's first BMW rank words merges the winners of a word before the global
  // ORs. It must stay: the winners of every window of a call concentrate on its lowest ranks (the longest
  // covers), and one global atomic per winner put all of a call's windows on the same few words (r06: 4.8
  // instead of 1.0 ms for the direct tables)
  const uint32_t words = (uint32_t)min<uint64_t>(BMW, (gbase + ng - base + 31) / 32);
  constexpr bool dedupe = true;
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) bm[i] = 0;
  __syncthreads();
  // two threads per touched word (16 bits each): the walk over set bits is a chain of LDS reads
  for (uint32_t hw = threadIdx.x; hw < 2 * ntw; hw += blockDim.x) {
    const uint32_t wi = hw >> 1;
    uint32_t m = (touched[wi] >> (16 * (hw & 1))) & 0xFFFFu;
    while (m) {
      const uint32_t b = __builtin_ctz(m) + 16 * (hw & 1);
      m &= m - 1;
      const uint32_t r = decode(tab[wi * 32 + b]);
      if (r == RANK_NONE) continue;
      const uint64_t lr = (uint64_t)r - base;
      const uint32_t bit = 1u << (r & 31);
      if (lr < 32ull * words) {
        if (!(bm[lr >> 5] & bit)) atomicOr(&bm[lr >> 5], bit);
      } else {
        set_bits(&selbits[r >> 5], bit);
      }
    }
  }
  if (dedupe) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
      if (const uint32_t v = bm[i]) {
        uint32_t* gw = &selbits[(base >> 5) + i];
        // SYZ_EMIT_RFIRST: skip the OR when a plain read already shows the bits (a stale copy can only lack
        // bits: they are set, never cleared, during the step)
        if (!SYZ_EMIT_RFIRST || (*gw & v) != v) set_bits(gw, v);
      }
  }
  __syncthreads();
}

__device__ __forceinline__ void smin_direct(const PItem it, const SGroup* sg, const uint32_t* gslab,
                                            const uint64_t* gebase, const uint32_t* D, const PSlab* slabs,
                                            const uint32_t* __restrict__ elems,
                                            const uint32_t* __restrict__ rank_of_member, const uint64_t* gstart,
                                            uint32_t* selbits, SminLds& L) {
  uint32_t* tab = L.tabs;
  [[maybe_unused]] const uint64_t t0 = SM_T();
  {
    uint4* t4 = reinterpret_cast<uint4*>(tab);
    const uint4 none4 = make_uint4(RANK_NONE, RANK_NONE, RANK_NONE, RANK_NONE);
    for (uint32_t i = threadIdx.x; i < (1u << DS) / 4; i += 1024) t4[i] = none4;
    for (uint32_t i = threadIdx.x; i < (1u << DS) / 32; i += 1024) L.touched[i] = 0;
  }
  __syncthreads();
  [[maybe_unused]] const uint64_t t1 = SM_T();
  auto upd = [&](uint32_t o, uint32_t R) {
                                      if (R == RANK_NONE) return;  // padding or a lane past the window
                                      if (SYZ_SMIN_NOF) {  // timing only: the walk without table updates
                                        if ((o ^ R) == 0x7FFF1234u) tab[0] = 0;
                                        return;
                                      }
                                      // a plain read first: most elements of a PC held by many inputs lose
                                      // to the rank already there, and same-address reads broadcast where
                                      // atomics serialize
                                      const uint32_t ix = tab_index(o);
                                      uint32_t* t = &tab[ix];
                                      const uint32_t cur = *t;
                                      if (cur > R) {
                                        atomicMin(t, R);
                                        // the first writer of an entry saw it empty (and so did any racing
                                        // one): every written entry is marked
                                        if (cur == RANK_NONE) atomicOr(&L.touched[ix >> 5], 1u << (ix & 31));
                                      }
                                    };
  if (SYZ_SMIN_WW)
    for_slab_window_w<SYZ_SL_MU, SMIN_NBW>(it, sg, gslab, gebase, D, slabs, elems, rank_of_member, L.wsc, upd);
  else
    SMIN_WALK(SYZ_SL_MU, it, sg, gslab, gebase, D, slabs, elems, rank_of_member, L.wsc, L.red64, upd);
  __syncthreads();
  [[maybe_unused]] const uint64_t t2 = SM_T();
  if (SYZ_SMIN_NOEMIT) return;  // timing only
  const uint64_t gb = gstart[it.g];
  emit_touched<PK_SCRATCH_WORDS>(tab, L.touched, (1u << DS) / 32, gb, gstart[it.g + 1] - gb, L.wsc, selbits);
  [[maybe_unused]] const uint64_t t3 = SM_T();
  SM_STAT_ADD(0, 1);
  SM_STAT_ADD(1, t3 - t0);
  SM_STAT_ADD(2, t1 - t0);
  SM_STAT_ADD(3, t2 - t1);
  SM_STAT_ADD(4, t3 - t2);
}

#ifndef SYZ_SL_HU
#define SYZ_SL_HU 1
#endif
template <bool PACKED, int BLOCK, class LT>
__device__ __forceinline__ void smin_hash(const PItem it, const SGroup* sg, const uint32_t* gslab,
                                          const uint64_t* gebase, const uint32_t* D, const PSlab* slabs,
                                          const uint32_t* __restrict__ elems,
                                          const uint32_t* __restrict__ rank_of_member, const uint64_t* gstart,
                                          uint32_t* selbits, LT& L) {
  constexpr uint32_t NS = PACKED ? PHS : HS;  // slots
  constexpr uint32_t CAP = PACKED ? PHCAP : HCAP;
  constexpr uint32_t TW = PACKED ? PHS : 2 * HS;  // table words
  uint32_t* tabs = L.tabs;
  uint32_t* keys = tabs;  // PACKED: the slots
  uint32_t* vals = tabs + HS;
  const uint64_t gb = gstart[it.g], ng = gstart[it.g + 1] - gb;
  const uint32_t E = slab_window_count<BLOCK>(it, sg, gslab, D, reinterpret_cast<uint32_t*>(L.red64));
  if (E == 0) return;
  uint32_t R = (E + CAP - 1) / CAP;
  uint32_t* touched = L.touched;
  auto touch = [&](uint32_t h) { atomicOr(&touched[h >> 5], 1u << (h & 31)); };
  for (uint32_t round = 0; round < R;) {
    for (uint32_t i = threadIdx.x; i < TW; i += BLOCK) tabs[i] = (PACKED || i < HS) ? 0xFFFFFFFFu : RANK_NONE;
    for (uint32_t i = threadIdx.x; i < NS / 32; i += BLOCK) touched[i] = 0;
    if (threadIdx.x == 0) L.full = 0;
    __syncthreads();
    const uint32_t RR = R, rr = round;
    auto upd = [&](uint32_t o, uint32_t Rk) {
                                        if (Rk == RANK_NONE) return;  // a lane past the window
                                        if (SYZ_SMIN_NOF) {  // timing only: the walk without table updates
                                          if ((o ^ Rk) == 0x7FFF1234u) L.full = 1;
                                          return;
                                        }
                                        if (RR > 1 && (hash32(o) >> 5) % RR != rr) return;
                                        if constexpr (PACKED) {
                                          const uint32_t pk = (o << PK_RBITS) | (uint32_t)(Rk - gb);
                                          uint32_t h = (o * 0x9E3779B1u) >> (32 - PHS_BITS);
                                          for (uint32_t probes = 0; probes < HPROBE; probes++) {
                                            uint32_t k = keys[h];
                                            if (k == 0xFFFFFFFFu) {
                                              k = atomicCAS(&keys[h], 0xFFFFFFFFu, pk);
                                              if (k == 0xFFFFFFFFu) {
                                                touch(h);
                                                return;
                                              }
                                            }
                                            if ((k >> PK_RBITS) == o) {
                                              if (k > pk) atomicMin(&keys[h], pk);
                                              return;
                                            }
                                            h = (h + 1) & (PHS - 1);
                                          }
                                        } else {
                                          uint32_t h = hslot(o);
                                          for (uint32_t probes = 0; probes < HPROBE; probes++) {
                                            uint32_t k = keys[h];
                                            if (k == 0xFFFFFFFFu) {
                                              k = atomicCAS(&keys[h], 0xFFFFFFFFu, o);
                                              if (k == 0xFFFFFFFFu) {
                                                k = o;
                                                touch(h);
                                              }
                                            }
                                            if (k == o) {
                                              if (vals[h] > Rk) atomicMin(&vals[h], Rk);
                                              return;
                                            }
                                            h = (h + 1) & (HS - 1);
                                          }
                                        }
                                        L.full = 1;
                                      };
    if (PACKED && SYZ_SMIN_WWP)
      for_slab_window_w<SYZ_SL_HU, 16>(it, sg, gslab, gebase, D, slabs, elems, rank_of_member, L.wsc, upd);
    else
      for_slab_window<SYZ_SL_HU, SYZ_SMIN_IDENT, LT::NBLK>(it, sg, gslab, gebase, D, slabs, elems, rank_of_member,
                                                           L.wsc, L.red64, upd);
    __syncthreads();
    if (L.full) {
      R *= 2;
      round = 0;
      __syncthreads();
      continue;
    }
    if (SYZ_SMIN_NOEMIT) {  // timing only
      round++;
      __syncthreads();
      continue;
    }
    if constexpr (PACKED) {
      const uint32_t g32 = (uint32_t)gb;
      emit_touched<LT::WSC>(keys, touched, NS / 32, gb, ng, L.wsc, selbits, [g32](uint32_t v) {
        return v == 0xFFFFFFFFu ? RANK_NONE : g32 + (v & ((1u << PK_RBITS) - 1));
      });
    } else {
      emit_touched<LT::WSC>(vals, touched, NS / 32, gb, ng, L.wsc, selbits);
    }
    round++;
    __syncthreads();  // the emit's bitmap and table reads are done before the next round clears them
  }
}

// The items of an M launch: a workgroup per item (ctr null: items blockIdx.x, + gridDim.x, ...), or a grid
// of resident workgroups that take the next item from a counter when they finish one (ctr: zeroed by
// k_pm_init), so no slot waits for a workgroup launch between items and the largest items still go first
#if defined(SYZ_SMIN_DYN) || defined(SYZ_SMIN_PERSIST) || defined(SYZ_SMIN_IPW_D) || defined(SYZ_SMIN_IPW_H) || \
    defined(SYZ_SMIN_IPW_P)
#define SYZ_SMIN_LOOP 1
#else
#define SYZ_SMIN_LOOP 0  // one item per workgroup: no item loop in the kernels (the loop costs registers)
#endif
#ifndef SYZ_SMIN_XCD
// > 0: M's items in XCD chunks of this many (m_items). 8: step 2.484-2.485 against 2.499-2.503 ms, 32:
// 2.500-2.517 ms (profiles/r06_ab/r06_xcd_items_pm.log)
#define SYZ_SMIN_XCD 8
#endif
template <class Fn>
__device__ __forceinline__ void m_items(uint32_t nitems, uint32_t* ctr, Fn fn) {
  if (!SYZ_SMIN_LOOP) {
    (void)ctr;
    uint32_t i = blockIdx.x;
    if (SYZ_SMIN_XCD) {
      // chunks of SYZ_SMIN_XCD consecutive items (windows of one call) on one XCD (blocks b and b + 8
      // share one), chunk c on XCD c mod 8: the call's rank lines are re-read from that XCD's L2, and the
      // heaviest items still go first on every XCD (the grid is a multiple of 8 chunks)
      constexpr uint32_t K = SYZ_SMIN_XCD > 0 ? SYZ_SMIN_XCD : 1;
      const uint32_t x = blockIdx.x & 7u, r = blockIdx.x >> 3;
      i = ((r / K) * 8u + x) * K + r % K;
    }
    if (i < nitems) fn(i);
    return;
  }
  if (!ctr) {
    for (uint32_t i = blockIdx.x; i < nitems; i += gridDim.x) {
      fn(i);
      __syncthreads();
    }
    return;
  }
  __shared__ uint32_t next;
  for (;;) {
    if (threadIdx.x == 0) next = atomicAdd(ctr, 1u);
    __syncthreads();
    const uint32_t i = next;
    if (i >= nitems) break;
    fn(i);
    __syncthreads();  // (and every thread has read `next` before thread 0 writes it again)
  }
}

__global__ __launch_bounds__(1024) SYZ_SMIN_OCC void k_smin_direct(const PItem* items, const SGroup* sg,
                                                                   const uint32_t* gslab, const uint64_t* gebase,
                                                                   const uint32_t* D, const PSlab* slabs,
                                                                   const uint32_t* __restrict__ elems,
                                                                   const uint32_t* __restrict__ rank_of_member,
                                                                   const uint64_t* gstart, uint32_t* selbits,
                                                                   const int* gate, uint32_t nitems, uint32_t* ctr) {
  if (*gate) return;  // a speculated step on a plan that does not fit this layout (k_gpack)
  __shared__ SminLds L;
  m_items(nitems, ctr, [&](uint32_t i) {
    smin_direct(items[i], sg, gslab, gebase, D, slabs, elems, rank_of_member, gstart, selbits, L);
  });
}

// (one launch for a class's three table kinds measured no better and spills: M is throughput-bound)
// PACKED: PK_BLOCK threads with a PHS-slot table (SminPkLds); otherwise 1024 threads, keys + values
template <bool PACKED>
__global__ __launch_bounds__(PACKED ? PK_BLOCK : 1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_smin_hash(
    const PItem* items, const SGroup* sg, const uint32_t* gslab, const uint64_t* gebase, const uint32_t* D,
    const PSlab* slabs, const uint32_t* __restrict__ elems, const uint32_t* __restrict__ rank_of_member,
    const uint64_t* gstart, uint32_t* selbits, const int* gate, uint32_t nitems, uint32_t* ctr) {
  if (*gate) return;  // (see k_smin_direct)
  if constexpr (PACKED) {
    __shared__ SminPkLds L;
    m_items(nitems, ctr, [&](uint32_t i) {
      smin_hash<true, PK_BLOCK>(items[i], sg, gslab, gebase, D, slabs, elems, rank_of_member, gstart, selbits, L);
    });
  } else {
    __shared__ SminLds L;
    m_items(nitems, ctr, [&](uint32_t i) {
      smin_hash<false, 1024>(items[i], sg, gslab, gebase, D, slabs, elems, rank_of_member, gstart, selbits, L);
    });
  }
}

// Items per workgroup of the M kernels: a workgroup takes items i, i + grid, i + 2 grid, ... so the
// launch dispatches nitems / IPW workgroups (a 1024-thread, 79 KB-LDS workgroup per item made the direct
// kernel's dispatch its bound, r06). SYZ_SMIN_PERSIST=1: a grid of resident workgroups instead (per CU:
// two direct / hashed, four packed), which starves the kernels beside it.
#ifndef SYZ_SMIN_PERSIST
#define SYZ_SMIN_PERSIST 0
#endif
#ifndef SYZ_SMIN_IPW_D
#define SYZ_SMIN_IPW_D 1
#endif
#ifndef SYZ_SMIN_IPW_H
#define SYZ_SMIN_IPW_H 1
#endif
#ifndef SYZ_SMIN_IPW_P
#define SYZ_SMIN_IPW_P 1
#endif
static unsigned m_grid(size_t nitems, unsigned per_cu, unsigned ipw) {
  Context& c = ctx();
  if (SYZ_SMIN_PERSIST && !c.ncu) SYZ_HIP(hipDeviceGetAttribute(&c.ncu, hipDeviceAttributeMultiprocessorCount, c.device));
  const unsigned cap = SYZ_SMIN_PERSIST ? (unsigned)std::max(1, c.ncu) * per_cu : 0xFFFFFFFFu;
  if (SYZ_SMIN_XCD && !SYZ_SMIN_LOOP) {  // (m_items: whole chunks on every XCD)
    const size_t q = 8ull * (SYZ_SMIN_XCD > 0 ? SYZ_SMIN_XCD : 1);
    return (unsigned)((nitems + q - 1) / q * q);
  }
  return (unsigned)std::min<size_t>((nitems + ipw - 1) / ipw, cap);
}
// SYZ_SMIN_DYN: the launches that take their items from a counter (bit 0 / 1: direct small / big, 2 / 3:
// packed small / big, 4 / 5: hashed small / big), on SYZ_SMIN_DYN_CU resident workgroups per CU x their
// per-CU capacity
#ifndef SYZ_SMIN_DYN
#define SYZ_SMIN_DYN 0
#endif
#ifndef SYZ_SMIN_DYN_CU
#define SYZ_SMIN_DYN_CU 1.0
#endif
static unsigned m_dyn_grid(size_t nitems, unsigned per_cu) {
  Context& c = ctx();
  if (!c.ncu) SYZ_HIP(hipDeviceGetAttribute(&c.ncu, hipDeviceAttributeMultiprocessorCount, c.device));
  const unsigned cap = std::max(1u, (unsigned)(SYZ_SMIN_DYN_CU * per_cu * std::max(1, c.ncu)));
  return (unsigned)std::min<size_t>(nitems, cap);
}

// ---- outputs: the group-major kept list in selection order ----------------------------------------
// kept inputs per 32 ranks (bytes are 0/1)
// kept ranks per 32-rank word: the compaction scan's input
struct SelWordsFn {
  const uint32_t* selbits;
  __device__ void operator()(size_t i, uint64_t* v) const { v[0] = __popc(selbits[i]); }
};

__device__ __forceinline__ uint64_t sel_pos(const uint32_t* selbits, const uint64_t* wpos, uint64_t r) {
  return wpos[r >> 5] + __popc(selbits[r >> 5] & ((1u << (r & 31)) - 1u));
}
__device__ __forceinline__ bool sel_bit(const uint32_t* selbits, uint64_t r) { return (selbits[r >> 5] >> (r & 31)) & 1u; }

__global__ void k_sel_compact(const uint32_t* selbits, const uint64_t* wpos, const uint32_t* ent_of_rank, size_t n,
                              int64_t* out) {
  // one wave per 64 ranks: positions by a ballot prefix
  for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r - __lane_id() < n;
       r += (size_t)gridDim.x * blockDim.x) {
    const bool s = r < n && sel_bit(selbits, r);
    const uint64_t bal = __ballot(s);
    if (s) {
      const uint64_t base = r - __lane_id();
      const uint64_t lo32 = base >> 5;  // base is a multiple of 64
      const uint64_t pos = wpos[lo32] + __popcll(bal & lanemask_lt());
      out[pos] = (int64_t)ent_of_rank[r];
    }
  }
}

__global__ void k_sel_goff(const uint32_t* selbits, const uint64_t* wpos, const uint64_t* gstart, uint32_t G,
                           uint64_t* goff) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g <= G; g += gridDim.x * blockDim.x)
    goff[g] = sel_pos(selbits, wpos, gstart[g]);
}

// ---- key parts: a call group restricted to a PC range (multi-GPU) --------------------
// slice of member m's (sorted) cover inside [klo, khi]; members of whole groups keep their cover
__global__ void k_slices(const uint32_t* pcs, const uint64_t* off, const uint32_t* members, const uint64_t* el,
                         const uint32_t* group, size_t n, const uint32_t* krange, uint32_t* sbeg, uint32_t* slen) {
  for (size_t m = (size_t)blockIdx.x * blockDim.x + threadIdx.x; m < n; m += (size_t)gridDim.x * blockDim.x) {
    const uint32_t e = members[m];
    const uint32_t L = (uint32_t)(el[m] >> 32);
    const uint32_t klo = krange[2 * group[e]], khi = krange[2 * group[e] + 1];
    if (klo == 0 && khi == 0xFFFFFFFFu) {
      sbeg[m] = 0;
      slen[m] = L;
      continue;
    }
    const uint64_t b = off[e];
    const uint64_t x = lower_bound_dev<uint32_t>(pcs, b, b + L, klo);
    const uint64_t y = khi == 0xFFFFFFFFu ? b + L : lower_bound_dev<uint32_t>(pcs, x, b + L, khi + 1);
    sbeg[m] = (uint32_t)(x - b);
    slen[m] = (uint32_t)(y - x);
  }
}

// ---- host orchestration ---------------------------------------------------------------------------------

// (plan_windows, slab_plan, plan_items: plan_host.cpp)

static bool begin_once(MinJob& J, const RawMinArgs& a, const uint32_t* exact_span);

// the key parts (host arguments) of this call are those the cached plan was made for
static bool spec_parts_match(const MinJob& J, const RawMinArgs& a) {
  const std::vector<uint64_t>& k = J.pcache->key;
  const size_t G = a.G, tail = (size_t)2 * G + 3;  // hstart (G + 1), hsl (G), span, may_bounce
  if (!a.key_lo) return k.size() == tail;
  if (k.size() != tail + G) return false;
  for (size_t g = 0; g < G; g++)
    if (k[tail + g] != (((uint64_t)a.key_lo[g] << 32) | a.key_hi[g])) return false;
  return true;
}

static bool pm_serial() {
  static const bool v = getenv("SYZGPU_PM_SERIAL") && atoi(getenv("SYZGPU_PM_SERIAL")) != 0;
  return v || (prof().on && prof().serial);
}



// SYZGPU_PM_PSPLIT=1 (A/B): P as two launches, the small call groups' slabs first, so their M starts
// beside the big groups' slabs (measured slower: the big groups' LDS sort then waits for CUs behind
// both, r04_q3 3.04 vs 2.96 ms)
static bool pm_psplit() {
  static const bool v = dev_env("SYZGPU_PM_PSPLIT") && atoi(dev_env("SYZGPU_PM_PSPLIT")) != 0;
  return v;
}

// SYZGPU_PM_SPEC=0 (A/B): no speculative step on the last step's plans (begin_once)
static bool pm_spec() {
  static const bool v = !getenv("SYZGPU_PM_SPEC") || atoi(getenv("SYZGPU_PM_SPEC")) != 0;
  return v;
}



// the members' tile prefix (tpos): needs no plan, so it can run before the host's
uint64_t* slab_tiles(const uint32_t* mlen, size_t nmem, const char* prefix, hipStream_t s) {
  uint64_t* tpos = ctx().scratch.get<uint64_t>((std::string(prefix) + "_sl_tpos").c_str(), nmem + 2);
  scan_f<1>(TilesFn{mlen}, nmem, tpos, nullptr, s, prefix);
  return tpos;
}

void slab_build(SlabJob& J, const char* prefix, const uint32_t* mlen, const uint64_t* mpos, size_t nmem,
                const uint64_t* gstart, hipStream_t s, bool tiles_done) {
  Scratch& sc = ctx().scratch;
  auto nm = [&](const char* x) { return std::string(prefix) + x; };
  const uint32_t B = J.B, G = J.G;
  J.tpos = tiles_done ? sc.get<uint64_t>(nm("_sl_tpos").c_str(), nmem + 2) : slab_tiles(mlen, nmem, prefix, s);
  J.cstart = sc.get<uint64_t>(nm("_sl_cstart").c_str(), (size_t)B + 2);
  J.slabs = sc.get<PSlab>(nm("_sl_slabs").c_str(), J.slab_bound + 1);
  J.gslab = sc.get<uint32_t>(nm("_sl_gslab").c_str(), G + 1);
  J.gebase = sc.get<uint64_t>(nm("_sl_gebase").c_str(), G + 1);
  J.D = sc.get<uint32_t>(nm("_sl_D").c_str(), J.dtotal + 1);
  J.ecap = J.total_pcs + J.xtotal + 16;
  J.elems = sc.get<uint32_t>("pm_elems", J.ecap);
  J.wtot = nullptr;
  ProfScope ps("slab_plan", s, 0);
  if (J.wtotal) {
    J.wtot = sc.get<uint32_t>(nm("_sl_wtot").c_str(), J.wtotal + 1);
    SYZ_HIP(hipMemsetAsync(J.wtot, 0, J.wtotal * 4, s));
  }
  scan_f<1>(BlockSlabsFn{J.dbgroup, J.dgblock, gstart, J.dsg, J.tpos}, B, J.cstart, nullptr, s, prefix);
  k_sl_slabs<<<grid_for(std::max<uint64_t>(J.slab_bound, G + 1), 256, 8192), 256, 0, s>>>(
      J.dbgroup, B, J.dgblock, gstart, J.dsg, J.tpos, mpos, J.cstart, J.slab_bound, J.slabs, G, J.gslab, J.gebase);
  SYZ_LAUNCHED();
}


// P for one plan on the part stream (pm_serial: on s): the plan's slab table (slab_build), then the
// transpose, so the main stream goes from the partition straight into the Go sort (the step's critical
// path); SYZGPU_PM_PSPLIT=1: the small call groups' slabs as a launch of their own first. ev_psmall
// marks the small groups' slabs, the caller records the rest.
static hipStream_t launch_p(const RawMinArgs& a, const SlabPlanCache& PC, SlabJob& SJ, const uint32_t* members,
                            const uint32_t* mlen, const uint64_t* mpos, const uint64_t* gstart, const uint32_t* sbeg,
                            int* err) {
  Context& c = ctx();
  hipStream_t s = a.s;
  if (!c.part) {
    int least = 0, greatest = 0;
    SYZ_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    SYZ_HIP(hipStreamCreateWithPriority(&c.part, hipStreamNonBlocking, least));
    SYZ_HIP(hipEventCreateWithFlags(&c.ev_part0, hipEventDisableTiming));
    SYZ_HIP(hipEventCreateWithFlags(&c.ev_part1, hipEventDisableTiming));
  }
  if (!c.ev_psmall) SYZ_HIP(hipEventCreateWithFlags(&c.ev_psmall, hipEventDisableTiming));
  hipStream_t pq = pm_serial() ? s : c.part;
  SYZ_HIP(hipEventRecord(c.ev_part0, s));
  SYZ_HIP(hipStreamWaitEvent(c.part, c.ev_part0, 0));
  slab_build(SJ, "pm", mlen, mpos, a.n, gstart, pq, true);
  if (!SJ.slab_bound) {
    SYZ_HIP(hipEventRecord(c.ev_psmall, pq));
    return pq;
  }
  // byte model: the algorithm's input this pass reads, 4 B per PC + 10 B per entry
  // (offset, group id); the element buffer it writes is intermediate traffic, not algorithmic bytes
  const auto& icount = PC.icount;
  const bool split = pm_psplit() && !pm_serial() && icount[0][0] + icount[0][1] + icount[0][2] > 0;
  for (int cls = split ? 1 : 0; cls <= (split ? 2 : 0); cls++) {
    const uint64_t bytes = cls ? PC.cpcs[cls - 1] * 4 + PC.cent[cls - 1] * 10
                               : (PC.cpcs[0] + PC.cpcs[1]) * 4 + (uint64_t)a.n * 10;
    ProfScope ps("k_slab", pq, bytes);
    launch_slab<false>(SJ.slab_bound, SJ.wmax, pq, a.pcs, a.off, members, mlen, SJ.tpos, sbeg, SJ.slabs,
                       SJ.cstart + SJ.B, SJ.dsg, SJ.gebase, PC.lo, SJ.elems, SJ.ecap, SJ.D, err, nullptr, NovSrc{},
                       cls, err + 2);
    SYZ_LAUNCHED();
    if (cls == 1) SYZ_HIP(hipEventRecord(c.ev_psmall, pq));
  }
  if (!split) SYZ_HIP(hipEventRecord(c.ev_psmall, pq));
  return pq;
}

// The plan of a layout: the slabs' layout and the M work items, a pure function of the group sizes, the
// PCs each group reads, the span and the key ranges (plan_key). A step on the same layout reuses the
// previous one's (host structures and the staged device copy owned by the job).
static std::vector<uint64_t> plan_key(const RawMinArgs& a, const std::vector<uint64_t>& hstart, const uint64_t* hsl,
                                      uint32_t lo, uint32_t hi, bool may_bounce) {
  const uint32_t G = a.G;
  std::vector<uint64_t> key(hstart);
  key.insert(key.end(), hsl, hsl + G);
  key.push_back(((uint64_t)lo << 32) | hi);
  key.push_back(may_bounce);
  if (a.key_lo)
    for (uint32_t g = 0; g < G; g++) key.push_back(((uint64_t)a.key_lo[g] << 32) | a.key_hi[g]);
  return key;
}

static void plan_layout(MinJob& J, const RawMinArgs& a, const std::vector<uint64_t>& hstart,
                        const std::vector<uint64_t>& hpcs, const uint64_t* hsl_in, const std::vector<PGroup>& hpg,
                        uint32_t lo, uint32_t hi, uint64_t span_raw) {
  Context& c = ctx();
  const size_t n = a.n;
  const uint32_t G = a.G;
  hipStream_t s = a.s;
  // (hsl points into the lane's pinned buffer, which the plan's staging copy below reuses)
  const std::vector<uint64_t> hslv(hsl_in, hsl_in + G);
  const uint64_t* hsl = hslv.data();
  const auto is_big = [&](uint32_t g) { return hstart[g + 1] - hstart[g] > GS_T_SEG; };
  std::vector<uint64_t> key = plan_key(a, hstart, hsl, lo, hi, J.may_bounce);
  J.spec_ok = J.pcache && J.pcache->key == key;  // the layout repeated: the next call may speculate
  if (!J.pcache || J.pcache->key != key) {
    auto P = std::make_shared<SlabPlanCache>();
    if (J.pcache) {  // the device staging of the last plan is reused (grow-only): no hipMalloc / hipFree
      std::swap(P->dstage.p, J.pcache->dstage.p);
      std::swap(P->dstage.cap, J.pcache->dstage.cap);
    }
    P->key = std::move(key);
    SlabJob& SJ = P->SJ;
    slab_plan(SJ, hstart, hsl, hpg, G, false);
    const uint32_t B = SJ.B;
    ItemPlan ip;
    plan_items(hstart, hpcs, hsl, hpg, G, a.key_lo, a.key_hi, lo, hi, ip);
    const size_t nitems = ip.items.size();
    std::memcpy(P->icount, ip.icount, sizeof(P->icount));
    std::memcpy(P->item_pcs, ip.item_pcs, sizeof(P->item_pcs));
    std::memcpy(P->cpcs, ip.cpcs, sizeof(P->cpcs));
    std::memcpy(P->cent, ip.cent, sizeof(P->cent));
    P->ifirst = ip.ifirst;
    // the plan goes over in one copy: SGroup[G], gblock[G + 1], bgroup[B + 1], items[nitems + 1]
    auto al16 = [](size_t x) { return (x + 15) & ~size_t(15); };
    P->o_gb = al16((G + 1) * sizeof(SGroup));
    P->o_bg = P->o_gb + al16((G + 1) * 4);
    P->o_it = P->o_bg + al16(((size_t)B + 1) * 4);
    P->o_exp = P->o_it + al16((nitems + 1) * sizeof(PItem));
    const size_t stage_bytes = P->o_exp + al16((3 * (size_t)G + 4) * 8);
    uint8_t* stage = c.pinned.get<uint8_t>(stage_bytes + 64);
    P->dstage.ensure(stage_bytes + 64);
    for (uint32_t g = 0; g < G; g++) SJ.hsg[g].pad = is_big(g) ? 1u : 0u;
    std::memcpy(stage, SJ.hsg.data(), G * sizeof(SGroup));
    std::memcpy(stage + P->o_gb, SJ.hgblock.data(), (G + 1) * 4);
    if (B) std::memcpy(stage + P->o_bg, SJ.hbgroup.data(), (size_t)B * 4);
    if (nitems) std::memcpy(stage + P->o_it, ip.items.data(), nitems * sizeof(PItem));
    // the words a step speculated on this plan must read back (k_gpack's gate)
    uint64_t* ex = reinterpret_cast<uint64_t*>(stage + P->o_exp);
    std::memset(ex, 0, (3 * (size_t)G + 4) * 8);
    for (uint32_t g = 0; g <= G; g++) ex[g] = hstart[g];
    ex[2 * G + 1] = span_raw;
    for (uint32_t g = 0; g < G; g++) ex[2 * G + 3 + g] = hsl[g];
    ex[3 * G + 3] = J.may_bounce ? 1 : 0;
    SYZ_HIP(hipMemcpyAsync(P->dstage.p, stage, stage_bytes, hipMemcpyHostToDevice, s));
    SJ.dsg = reinterpret_cast<SGroup*>(P->dstage.p);
    SJ.dgblock = reinterpret_cast<uint32_t*>(P->dstage.p + P->o_gb);
    SJ.dbgroup = reinterpret_cast<uint32_t*>(P->dstage.p + P->o_bg);
    P->lo = lo;
    P->n = n;
    P->hi = hi;
    J.pcache = P;
  }
}

// The step's device work on the job's plan (J.pcache) and Go-sort plan: P on its own stream beside the
// Go sort, then M per class as soon as its own sort and P are done. Nothing here waits for the device.
static void launch_step(MinJob& J, const RawMinArgs& a, const uint32_t* members, uint64_t* el, const uint32_t* mlen,
                        const uint64_t* mpos, const uint32_t* sbeg, int* err) {
  Context& c = ctx();
  Scratch& sc = c.scratch;
  const size_t n = a.n;
  const uint32_t G = a.G;
  hipStream_t s = a.s;
  uint64_t* gstart = J.gstart.p;
  uint32_t* rank_of_member = J.rank_of_member.p;
  uint32_t* ent_of_rank = J.ent_of_rank.p;
  uint32_t* selbits = J.selbits.p;
  const std::vector<uint64_t>& hstart = J.hstart;
  HostTimer ht("launch_step");
  const SlabPlanCache& PC = *J.pcache;
  SlabJob SJ = PC.SJ;  // (the device members below are this step's)
  const auto& icount = PC.icount;
  const auto& ifirst = PC.ifirst;
  const auto& item_pcs = PC.item_pcs;
  uint8_t* dstage = PC.dstage.p;
  const SGroup* dsg = SJ.dsg;
  const PItem* ditems = reinterpret_cast<const PItem*>(dstage + PC.o_it);
  (void)G;
  // the Go sort's plan of a new layout first, while the device is idle (re-planned in place: grow-only
  // device arrays, the learned round count kept)
  if (!J.plan || J.plan_key != hstart) {
    if (!J.plan) J.plan = std::make_shared<GosortPlan>();
    gosort_plan(*J.plan, hstart, G, s);
    J.plan_key = hstart;
  }
  hipStream_t pq = launch_p(a, PC, SJ, members, mlen, mpos, gstart, sbeg, err);
  ht.mark("slab_build");
  const int* gate = err + 2;
  uint32_t* mctr = sc.get<uint32_t>("pm_mctr", 16);
  const PSlab* slabs = SJ.slabs;
  const uint32_t* gslab = SJ.gslab;
  const uint64_t* gebase = SJ.gebase;
  const uint32_t* D = SJ.D;
  uint32_t* elems = SJ.elems;
  while (c.ev_cnt.size() < 1) {
    hipEvent_t e1, e2;
    SYZ_HIP(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    SYZ_HIP(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    c.ev_cnt.push_back(e1);
    c.ev_sct.push_back(e2);
  }
  int* herr = c.pinned_err.get<int>(4);  // (not the lane's pinned buffer: the read-back may still be read)
  SYZ_HIP(hipMemcpyAsync(herr, err, 12, hipMemcpyDeviceToHost, pq));  // P's flags, the partition's, the gate
  SYZ_HIP(hipEventRecord(c.ev_cnt[0], pq));
  SYZ_HIP(hipEventRecord(c.ev_sct[0], pq));
  SYZ_HIP(hipEventRecord(c.ev_part1, pq));
  // ---- Go-sort ranks, then M per class as soon as its own sort and P are done ----
  uint32_t* perm = sc.get<uint32_t>("mz_perm", n + 1);
  SYZ_HIP(hipMemsetAsync(selbits, 0, (n / 32 + 2) * 4, s));
  GosortPlan& P = *J.plan;
  auto run_m = [&](hipStream_t q, int big) {
    ProfScope ps(big ? "m_big" : "m_small", q, 0);
    const size_t nd = icount[big][PMODE_DIRECT], nh = icount[big][PMODE_HASH], np = icount[big][PMODE_PACKED];
    if (!nd && !nh && !np) return;
    if (SYZ_SL_NOD) return;  // (timing variant without D rows: M would walk garbage)
    SYZ_HIP(hipStreamWaitEvent(q, big ? c.ev_sct[0] : c.ev_psmall, 0));
    const bool dd = (SYZ_SMIN_DYN >> big) & 1, dp = (SYZ_SMIN_DYN >> (2 + big)) & 1,
               dh = (SYZ_SMIN_DYN >> (4 + big)) & 1;
    if (nd) {
      ProfScope pk("k_pmin_direct", q, 4 * item_pcs[big][PMODE_DIRECT]);
      k_smin_direct<<<dd ? m_dyn_grid(nd, 2) : m_grid(nd, 2, SYZ_SMIN_IPW_D), 1024, 0, q>>>(
          ditems + ifirst[big][PMODE_DIRECT], dsg, gslab, gebase, D, slabs, elems, rank_of_member, gstart, selbits, gate,
          (uint32_t)nd, dd ? mctr + 2 * big : nullptr);
      SYZ_LAUNCHED();
    }
    if (nh) {
      ProfScope pk("k_pmin_hash", q, 4 * item_pcs[big][PMODE_HASH]);
      k_smin_hash<false><<<dh ? m_dyn_grid(nh, 2) : m_grid(nh, 2, SYZ_SMIN_IPW_H), 1024, 0, q>>>(
          ditems + ifirst[big][PMODE_HASH], dsg, gslab, gebase, D, slabs, elems, rank_of_member, gstart, selbits, gate,
          (uint32_t)nh, dh ? mctr + 4 + 2 * big : nullptr);
      SYZ_LAUNCHED();
    }
    // (the packed tables on a stream of their own beside the others: slower with the big groups' M
    // running too, the process has 4 hardware queues; and with no big groups, config 1, 0.387 against
    // 0.353 ms: the fork and join cost more than the two small launches overlap)
    if (np) {
      ProfScope pk("k_pmin_packed", q, 4 * item_pcs[big][PMODE_PACKED]);
      k_smin_hash<true><<<dp ? m_dyn_grid(np, 4) : m_grid(np, 4, SYZ_SMIN_IPW_P), PK_BLOCK, 0, q>>>(
          ditems + ifirst[big][PMODE_PACKED], dsg, gslab, gebase, D, slabs, elems, rank_of_member, gstart, selbits,
          gate, (uint32_t)np, dp ? mctr + 8 + 2 * big : nullptr);
      SYZ_LAUNCHED();
    }
  };
  P.may_bounce = J.may_bounce;
  auto small_done = [&](hipStream_t q) {
    if (P.npacks) ranks_packs(el, perm, P, members, rank_of_member, ent_of_rank, q);
    run_m(q, 0);
  };
  auto big_done = [&](hipStream_t q) {
    if (P.nbig) ranks_big(el, perm, P, members, rank_of_member, ent_of_rank, q);
    run_m(q, 1);
  };
  ht.mark("launch_p_plan_sort");
  if (n) {
    gosort_run(el, perm, n, P, s, small_done, big_done);
  } else {
    small_done(s);
    big_done(s);
  }
  ht.mark("gosort_run");
  if (!J.done) SYZ_HIP(hipEventCreateWithFlags(&J.done, hipEventDisableTiming));
  SYZ_HIP(hipEventRecord(J.done, s));
}

// After launch_step: P's flags (herr, copied back behind P). false: a PC outside the windows (an
// unsorted cover): the caller redoes the job on exact bounds.
static bool finish_step(MinJob& J, const uint32_t* exact_span) {
  Context& c = ctx();
  const SlabPlanCache& PC = *J.pcache;
  int* herr = c.pinned_err.get<int>(4);
  SYZ_HIP(hipEventSynchronize(c.ev_cnt[0]));
  J.stats_total_pcs = PC.SJ.total_pcs;
  J.stats_items_direct = PC.icount[0][PMODE_DIRECT] + PC.icount[1][PMODE_DIRECT];
  J.stats_items_hash = PC.icount[0][PMODE_HASH] + PC.icount[1][PMODE_HASH] + PC.icount[0][PMODE_PACKED] +
                       PC.icount[1][PMODE_PACKED];
  if (herr[0] & 64) fail(SYZGPU_EINTERNAL, "minimize: slab plan does not fit the layout");
  // a kept step whose gate closed would have skipped P and M: the host's and the device's key checks agree
  if (herr[2]) fail(SYZGPU_EINTERNAL, "minimize: speculation gate closed on a kept step");
  if (herr[0] & 1) {
    if (exact_span) fail(SYZGPU_EINTERNAL, "minimize: PC outside the exact span");
    return false;
  }
  J.begun = true;
  return true;
}

void minimize_raw_begin(MinJob& J, const RawMinArgs& a) {
  if (a.G == 0 || a.G > MAX_GROUPS_PM) fail(SYZGPU_EINVAL, "ngroups out of range (1..4096)");
  if (a.n >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "too many corpus entries");
  if (!a.off || (a.n && !a.group)) fail(SYZGPU_EINVAL, "null pointer");
  if (begin_once(J, a, nullptr)) return;
  // some cover is not sorted: exact PC bounds, then once more (key parts need sorted covers)
  if (a.key_lo) fail(SYZGPU_EINVAL, "key parts need canonical (sorted) covers");
  Context& c = ctx();
  uint32_t* span = c.scratch.get<uint32_t>("pm_xspan", 2);
  uint32_t* h = c.pinned.get<uint32_t>(4);
  h[0] = 0xFFFFFFFFu;
  h[1] = 0;
  SYZ_HIP(hipMemcpyAsync(span, h, 8, hipMemcpyHostToDevice, a.s));
  uint64_t* L = c.pinned.get<uint64_t>(2) + 1;
  SYZ_HIP(hipMemcpyAsync(L, a.off + a.n, 8, hipMemcpyDeviceToHost, a.s));
  SYZ_HIP(hipStreamSynchronize(a.s));
  if (*L) {
    k_minmax<<<grid_for(*L, 256, 8192), 256, 0, a.s>>>(a.pcs, *L, span);
    SYZ_LAUNCHED();
  }
  uint32_t x[2];
  SYZ_HIP(hipMemcpyAsync(h, span, 8, hipMemcpyDeviceToHost, a.s));
  SYZ_HIP(hipStreamSynchronize(a.s));
  x[0] = h[0];
  x[1] = h[1];
  if (!begin_once(J, a, x)) fail(SYZGPU_EINTERNAL, "minimize: PC outside the exact span");
}

// false: some PC lies outside the planned windows (an unsorted cover)
static bool begin_once(MinJob& J, const RawMinArgs& a, const uint32_t* exact_span) {
  Context& c = ctx();
  Scratch& sc = c.scratch;
  const size_t n = a.n;
  const uint32_t G = a.G;
  hipStream_t s = a.s;
  J.begun = false;
  J.n = n;
  J.G = G;
  J.group = a.group;
  J.prog_len = a.prog_len;
  J.gstart.ensure(G + 1);
  J.selbits.ensure(n / 32 + 2);
  J.ent_of_rank.ensure(n + 1);
  J.rank_of_member.ensure(n + 1);
  uint64_t* gstart = J.gstart.p;
  uint32_t* rank_of_member = J.rank_of_member.p;
  uint32_t* ent_of_rank = J.ent_of_rank.p;
  // ---- group partition (stable), sort keys, per-group PCs, span, member slices and offsets ----
  uint32_t* members = sc.get<uint32_t>("mz_members", n + 1);
  uint64_t* el = sc.get<uint64_t>("mz_el", n + 1);
  uint64_t* gpcs = sc.get<uint64_t>("mz_gpcs", G + 1);
  uint32_t* span = sc.get<uint32_t>("pm_span", 4);
  int* err = sc.get<int>("mz_err", 4);  // [0] P's flags, [1] the partition's, [2] the speculation gate
  uint32_t* mlen = sc.get<uint32_t>("pm_mlen", n + 1);
  uint32_t* sbeg = a.key_lo ? sc.get<uint32_t>("pm_sbeg", n + 1) : nullptr;
  uint64_t* mpos = sc.get<uint64_t>("pm_mpos", n + 1);
  uint64_t* gpack = sc.get<uint64_t>("pm_gpack", 3 * (size_t)G + 4);
  uint32_t* mlmax = sc.get<uint32_t>("pm_mlmax", 1);
  // Only while layouts repeat: after a miss (a corpus that changed since the last call, e.g. NewInputs
  // between the manager's minimizes) the job plans on the read-back layout until a step finds its plan
  // cached again, so a layout that changes on every call pays one miss, not one per call.
  const bool spec = J.spec_ok && !J.nospec && J.pcache && J.plan && !exact_span && pm_spec() && J.pcache->n == n &&
                    J.pcache->SJ.G == G && J.hstart == J.plan_key && J.plan_key.size() == (size_t)G + 1 &&
                    spec_parts_match(J, a);
  J.nospec = false;
  const uint64_t* exp = spec ? reinterpret_cast<const uint64_t*>(J.pcache->dstage.p + J.pcache->o_exp) : nullptr;
  k_pm_init<<<grid_for(std::max<uint32_t>(G + 1, 16), 256, 64), 256, 0, s>>>(err, gpcs, G, span, mlmax,
                                                                             sc.get<uint32_t>("pm_mctr", 16));
  SYZ_LAUNCHED();
  uint32_t* krange = nullptr;
  if (a.key_lo) {
    std::vector<uint32_t> kr(2 * (size_t)G);
    for (uint32_t g = 0; g < G; g++) {
      kr[2 * g] = a.key_lo[g];
      kr[2 * g + 1] = a.key_hi[g];
    }
    krange = sc.get<uint32_t>("pm_krange", 2 * (size_t)G);
    SYZ_HIP(hipMemcpyAsync(krange, kr.data(), kr.size() * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipStreamSynchronize(s));  // kr is a host temporary
  }
  {
    ProfScope ps("group_partition", s, (uint64_t)n * 28);
    // the span pass reads only the covers: on the side stream, beside the partition
    ensure_side(c);
    if (n) {
      SYZ_HIP(hipEventRecord(c.ev_fork, s));
      SYZ_HIP(hipStreamWaitEvent(c.side, c.ev_fork, 0));
      // whole covers: the per-group PCs are the member prefix's group differences (k_gpack), so the
      // span pass takes no per-group atomics (a wider grid measured slower: its span atomics)
      if (krange)
        k_span_sums<<<grid_for(n, 256, span_blocks()), 256, G * 8, c.side>>>(a.pcs, a.off, a.group, n, G, gpcs, span,
                                                                                 mlmax);
      else
        k_span_sums<<<grid_for(n, 256, span_blocks()), 256, 0, c.side>>>(a.pcs, a.off, a.group, n, G, nullptr, span,
                                                                            mlmax);
      SYZ_LAUNCHED();
      SYZ_HIP(hipEventRecord(c.ev_join, c.side));
    }
    // (the partition also writes the identity ranks and, for whole covers, the member lengths)
    PartOut po;
    po.rank_of_member = rank_of_member;
    po.ent_of_rank = ent_of_rank;
    po.mlen = krange ? nullptr : mlen;
    group_partition_dev(a.group, a.off, n, G, gstart, members, el, err, s, po);
    if (n && krange) {
      k_slices<<<grid_for(n, 256, 4096), 256, 0, s>>>(a.pcs, a.off, members, el, a.group, n, krange, sbeg, mlen);
      SYZ_LAUNCHED();
    }
    // the member slices' prefix (mpos) and the slab tiles' (tpos) in one scan
    uint64_t* tpos = sc.get<uint64_t>("pm_sl_tpos", n + 2);
    scan_f<2>(LenTilesFn{mlen}, n, mpos, tpos, s, "pm_mt");
    if (n) SYZ_HIP(hipStreamWaitEvent(s, c.ev_join, 0));
    k_gpack<<<grid_for(3 * (size_t)G + 4, 256, 64), 256, 0, s>>>(gstart, gpcs, span, err, mpos, G, mlmax, gpack, exp,
                                                                 err + 2);
    SYZ_LAUNCHED();
  }
  uint64_t* hbuf = c.pinned.get<uint64_t>(3 * (size_t)G + 8);
  SYZ_HIP(hipMemcpyAsync(hbuf, gpack, (3 * (size_t)G + 4) * 8, hipMemcpyDeviceToHost, s));
  if (!c.ev_spin) SYZ_HIP(hipEventCreateWithFlags(&c.ev_spin, hipEventDisableTiming));
  SYZ_HIP(hipEventRecord(c.ev_spin, s));
  // Speculation: with the last step's plans at hand (a step on the same layout: the common case), the
  // whole step goes out on them before the layout is read back, so the host's read-back and planning
  // leave the device's critical path. It is kept when the layout read back is the one planned (the
  // group starts and plan_key); otherwise it is waited for and the step redone without. P's guards
  // keep a stale plan's slabs inside their buffers (err 64). SYZGPU_PM_SPEC=0: no speculation.
  if (spec) launch_step(J, a, members, el, mlen, mpos, sbeg, err);
  HostTimer ht("begin");
  event_wait_spin(c.ev_spin);
  ht.mark("wait_partition");
  const bool may_bounce = hbuf[3 * G + 3] >= GS_U32_LEN_LIMIT;
  const bool bad_group = *reinterpret_cast<int*>(hbuf + 2 * G + 2) != 0;
  std::vector<uint64_t> hstart(hbuf, hbuf + G + 1), hpcs(hbuf + G + 1, hbuf + 2 * G + 1);
  const std::vector<uint64_t> hslv(hbuf + 2 * G + 3, hbuf + 3 * G + 3);  // PCs this job reads per group
  const uint64_t* hsl = hslv.data();                                     // (key parts: the slices)
  if (!krange) hpcs.assign(hsl, hsl + G);  // (whole covers: the slices are the groups' PCs)
  uint32_t lo = reinterpret_cast<uint32_t*>(hbuf + 2 * G + 1)[0], hi = reinterpret_cast<uint32_t*>(hbuf + 2 * G + 1)[1];
  if (exact_span) {
    lo = exact_span[0];
    hi = exact_span[1];
  }
  if (lo > hi) lo = hi = 0;  // no PCs at all
  if (spec) {
    if (!bad_group && hstart == J.plan_key && plan_key(a, hstart, hsl, lo, hi, may_bounce) == J.pcache->key) {
      ht.mark("spec_kept");
      J.spec_hits++;
      return finish_step(J, exact_span);
    }
    SYZ_HIP(hipEventSynchronize(J.done));  // the speculative step is done with every buffer
    J.spec_ok = false;
    J.spec_misses++;
    if (!bad_group) {
      J.nospec = true;
      return begin_once(J, a, exact_span);  // the partition again, then planned as below
    }
  }
  if (bad_group) fail(SYZGPU_EINVAL, "group id >= ngroups");
  J.may_bounce = may_bounce;
  J.hstart = hstart;
  const uint64_t spanw = (uint64_t)hi - lo + 1;
  // ---- plan: window size per call group, blocks, chunk bound, work items ----
  std::vector<PGroup> hpg;
  plan_windows(spanw, hpcs.data(), hstart.data(), G, hpg);
  ht.mark("plan_windows");
  plan_layout(J, a, hstart, hpcs, hsl, hpg, lo, hi, hbuf[2 * G + 1]);
  ht.mark("plan_layout");
  launch_step(J, a, members, el, mlen, mpos, sbeg, err);
  return finish_step(J, exact_span);
}

__global__ void k_job_xchg(uint32_t* selbits, const uint64_t* gstart, const uint32_t* groups, const uint64_t* boff,
                           uint8_t* buf, int import) {
  const uint32_t g = groups[blockIdx.y];
  const uint64_t gb = gstart[g], ng = gstart[g + 1] - gb, o = boff[blockIdx.y];
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < ng; r += (uint64_t)gridDim.x * blockDim.x) {
    if (import) {
      if (buf[o + r]) set_bits(&selbits[(gb + r) >> 5], 1u << ((gb + r) & 31));
    } else {
      buf[o + r] = (uint8_t)sel_bit(selbits, gb + r);
    }
  }
}

void minimize_raw_xchg(MinJob& J, const uint32_t* groups, const uint64_t* offsets, uint32_t ng, uint8_t* buf,
                       int import, hipStream_t s) {
  if (!J.begun) fail(SYZGPU_EINVAL, "minimize job: begin first");
  if (!ng) return;
  if (!groups || !offsets || !buf) fail(SYZGPU_EINVAL, "null pointer");
  uint64_t maxn = 0;
  for (uint32_t j = 0; j < ng; j++) {
    if (groups[j] >= J.G) fail(SYZGPU_EINVAL, "group id >= ngroups");
    maxn = std::max<uint64_t>(maxn, J.hstart[groups[j] + 1] - J.hstart[groups[j]]);
  }
  std::vector<uint64_t> key(groups, groups + ng);
  key.insert(key.end(), offsets, offsets + ng);
  if (key != J.xkey) {  // the exchange list is the same every step: uploaded once
    J.xg.ensure(ng);
    J.xo.ensure(ng);
    SYZ_HIP(hipMemcpyAsync(J.xg.p, groups, ng * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(J.xo.p, offsets, ng * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipStreamSynchronize(s));
    J.xkey = key;
  }
  SYZ_HIP(hipStreamWaitEvent(s, J.done, 0));
  const unsigned gx = (unsigned)std::min<uint64_t>(std::max<uint64_t>(1, (maxn + 1023) / 1024), 1024);
  k_job_xchg<<<dim3(gx, ng), 256, 0, s>>>(J.selbits.p, J.gstart.p, J.xg.p, J.xo.p, buf, import);
  SYZ_LAUNCHED();
}

__global__ __launch_bounds__(256) void k_sel_flags(const uint32_t* selbits, const uint32_t* ent_of_rank, size_t n,
                                                   const uint16_t* prog_len, const uint32_t* group,
                                                   const uint8_t* count_hist, int32_t C, uint8_t* selected,
                                                   int64_t* hist, int* err) {
  extern __shared__ unsigned long long lh[];
  const bool do_hist = hist != nullptr;
  if (do_hist) {
    for (int32_t i = threadIdx.x; i <= C; i += blockDim.x) lh[i] = 0;
    __syncthreads();
  }
  for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (size_t)gridDim.x * blockDim.x) {
    const uint32_t e = ent_of_rank[r];
    const uint32_t s = sel_bit(selbits, r);
    if (selected) selected[e] = (uint8_t)s;
    if (do_hist && s && (!count_hist || count_hist[group[e]])) {
      const uint32_t L = prog_len[e];
      if ((int32_t)L > C)
        atomicOr(err, 2);
      else
        atomicAdd(&lh[L], 1ull);
    }
  }
  if (do_hist) {
    __syncthreads();
    for (int32_t i = threadIdx.x; i <= C; i += blockDim.x)
      if (lh[i]) atomicAdd((unsigned long long*)&hist[i], lh[i]);
  }
}

// selbits: the rank bitmap, n / 32 + 1 words at least, zero past n
void sel_compact_dev(const uint32_t* selbits, const uint32_t* ent_of_rank, const uint64_t* gstart, size_t n, uint32_t G,
                     int64_t* out_idx, uint64_t* group_out_off, hipStream_t s) {
  Scratch& sc = ctx().scratch;
  const size_t nw = (n + 31) / 32;
  uint64_t* wpos = sc.get<uint64_t>("pm_wpos", nw + 2);
  scan_f<1>(SelWordsFn{selbits}, nw, wpos, nullptr, s, "sel");
  if (out_idx && n) {
    k_sel_compact<<<grid_for(n, 256, 8192), 256, 0, s>>>(selbits, wpos, ent_of_rank, n, out_idx);
    SYZ_LAUNCHED();
  }
  if (group_out_off) {
    k_sel_goff<<<grid_for(G + 1, 256, 64), 256, 0, s>>>(selbits, wpos, gstart, G, group_out_off);
    SYZ_LAUNCHED();
  }
}

void minimize_raw_end(MinJob& J, const RawEndArgs& e) {
  if (!J.begun) fail(SYZGPU_EINVAL, "minimize job: begin first");
  if (e.len_hist && (e.C <= 0 || !J.prog_len)) fail(SYZGPU_EINVAL, "len_hist needs prog_len and C > 0");
  Context& c = ctx();
  Scratch& sc = c.scratch;
  const size_t n = J.n;
  const uint32_t G = J.G;
  hipStream_t s = e.s;
  // (err holds no bit here: begin fails or redoes the job on any of its own)
  int* err = sc.get<int>("mz_err", 2);
  SYZ_HIP(hipStreamWaitEvent(s, J.done, 0));
  const uint8_t* dcount = nullptr;
  if (e.count_hist) {
    J.count_hist.ensure(G);
    SYZ_HIP(hipMemcpyAsync(J.count_hist.p, e.count_hist, G, hipMemcpyHostToDevice, s));
    dcount = J.count_hist.p;
  }
  ProfScope ps("select_out", s, (uint64_t)n * 8);
  if (e.len_hist) SYZ_HIP(hipMemsetAsync(e.len_hist, 0, (size_t)(e.C + 1) * 8, s));
  if (n) {
    k_sel_flags<<<grid_for(n, 256, 512), 256, e.len_hist ? (size_t)(e.C + 1) * 8 : 0, s>>>(
        J.selbits.p, J.ent_of_rank.p, n, e.len_hist ? J.prog_len : nullptr, J.group, dcount, e.C, e.selected,
        e.len_hist, err);
    SYZ_LAUNCHED();
  }
  if (e.out_idx || e.group_out_off)
    sel_compact_dev(J.selbits.p, J.ent_of_rank.p, J.gstart.p, n, G, e.out_idx, e.group_out_off, s);
  if (e.len_hist && !e.defer_check) {  // len(p.Calls) > C is Go's index-out-of-range panic (prio.go:148)
    int* herr = c.pinned.get<int>(4);
    SYZ_HIP(hipMemcpyAsync(herr, err, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    minimize_raw_end_check(herr[0]);
  }
}

void minimize_raw_end_check(int err) {
  if (err & 2) fail(SYZGPU_EINVAL, "len(p.Calls) > C (prog/prio.go:148 would panic)");
}

// host copies of the group-major kept list (the syzgpu_minimize_grouped outputs)
void minimize_raw_fetch(MinJob& J, int64_t* out_idx, uint64_t* group_out_off) {
  if (!J.begun) fail(SYZGPU_EINVAL, "no matching minimize result");
  Context& c = ctx();
  hipStream_t s = c.stream;
  int64_t* dout = c.scratch.get<int64_t>("mz_out", J.n + 1);
  uint64_t* dgoff = c.scratch.get<uint64_t>("mz_goff", J.G + 1);
  RawEndArgs e{};
  e.out_idx = dout;
  e.group_out_off = dgoff;
  e.s = s;
  minimize_raw_end(J, e);
  SYZ_HIP(hipMemcpyAsync(group_out_off, dgoff, (J.G + 1) * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint64_t m = group_out_off[J.G];
  if (m && out_idx) SYZ_HIP(hipMemcpyAsync(out_idx, dout, m * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
}

}  // namespace syz

using namespace syz;

extern "C" {

#ifdef SYZ_SMIN_STATS
int syzgpu_debug_smin_stats(unsigned long long* out, int reset) {
  (void)hipDeviceSynchronize();
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sm_stats), sizeof(unsigned long long) * 16);
  (void)hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(g_sl_stats), sizeof(unsigned long long) * 8);
  if (reset) {
    unsigned long long z[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sm_stats), z, sizeof(z));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sl_stats), z, sizeof(unsigned long long) * 8);
  }
  return 0;
}
#endif

int syzgpu_mz_create(syzgpu_mz** out) {
  SYZ_API_BODY({
    if (!out) fail(SYZGPU_EINVAL, "null pointer");
    *out = reinterpret_cast<syzgpu_mz*>(new MinJob());
  })
}

int syzgpu_mz_destroy(syzgpu_mz* job) {
  SYZ_API_BODY({
    if (job) {
      MinJob* J = reinterpret_cast<MinJob*>(job);
      { std::lock_guard<std::recursive_mutex> hl_(J->mu); }
      delete J;
    }
  })
}

int syzgpu_mz_begin_dev(syzgpu_mz* job, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                        const uint16_t* prog_len, size_t n, uint32_t ngroups, const uint32_t* key_lo,
                        const uint32_t* key_hi, void* stream) {
  SYZ_API_BODY({
    if (!job) fail(SYZGPU_EINVAL, "null job");
    if ((key_lo == nullptr) != (key_hi == nullptr)) fail(SYZGPU_EINVAL, "key_lo and key_hi go together");
    MinJob& J = *reinterpret_cast<MinJob*>(job);
    std::lock_guard<std::recursive_mutex> hl_(J.mu);
    RawMinArgs a{pcs, off, group, prog_len, n, ngroups};
    a.key_lo = key_lo;
    a.key_hi = key_hi;
    a.s = (hipStream_t)stream;
    minimize_raw_begin(J, a);
  })
}

int syzgpu_mz_export_sel_dev(syzgpu_mz* job, const uint32_t* groups, const uint64_t* offsets, uint32_t ngroups,
                             uint8_t* buf, void* stream) {
  SYZ_API_BODY({
    if (!job) fail(SYZGPU_EINVAL, "null job");
    MinJob& J = *reinterpret_cast<MinJob*>(job);
    std::lock_guard<std::recursive_mutex> hl_(J.mu);
    minimize_raw_xchg(J, groups, offsets, ngroups, buf, 0, (hipStream_t)stream);
  })
}

int syzgpu_mz_import_sel_dev(syzgpu_mz* job, const uint32_t* groups, const uint64_t* offsets, uint32_t ngroups,
                             const uint8_t* buf, void* stream) {
  SYZ_API_BODY({
    if (!job) fail(SYZGPU_EINVAL, "null job");
    MinJob& J = *reinterpret_cast<MinJob*>(job);
    std::lock_guard<std::recursive_mutex> hl_(J.mu);
    minimize_raw_xchg(J, groups, offsets, ngroups, const_cast<uint8_t*>(buf), 1, (hipStream_t)stream);
  })
}

int syzgpu_mz_end_dev(syzgpu_mz* job, int32_t C, const uint8_t* count_hist, uint8_t* selected, int64_t* len_hist,
                      int64_t* out_idx, uint64_t* group_out_off, void* stream) {
  SYZ_API_BODY({
    if (!job) fail(SYZGPU_EINVAL, "null job");
    MinJob& J = *reinterpret_cast<MinJob*>(job);
    std::lock_guard<std::recursive_mutex> hl_(J.mu);
    RawEndArgs e;
    e.C = C;
    e.count_hist = count_hist;
    e.selected = selected;
    e.len_hist = len_hist;
    e.out_idx = out_idx;
    e.group_out_off = group_out_off;
    e.s = (hipStream_t)stream;
    minimize_raw_end(J, e);
  })
}

// minimizeCorpus's tail in one call (manager.go:523-536): the kept flags, list and length histogram of
// the job (syzgpu_mz_end_dev), calcStaticPriorities of the usage matrix on a second stream beside
// them, then CalculatePriorities + BuildChoiceTable from the histogram (syzgpu_prio_choice_dev); the
// error checks of all three after one wait.
int syzgpu_mz_end_prio_dev(syzgpu_mz* job, int32_t C, const uint8_t* count_hist, uint8_t* selected,
                           int64_t* len_hist, int64_t* out_idx, uint64_t* group_out_off, const float* uses,
                           size_t nkeys, float* static_prios, float* prios, int64_t* run, uint8_t* row_present,
                           void* stream) {
  SYZ_API_BODY({
    if (!job) fail(SYZGPU_EINVAL, "null job");
    if (!len_hist || !static_prios || !prios || !run) fail(SYZGPU_EINVAL, "null pointer");
    MinJob& J = *reinterpret_cast<MinJob*>(job);
    std::lock_guard<std::recursive_mutex> hl_(J.mu);
    Context& c = ctx();
    hipStream_t s = (hipStream_t)stream;
    // calcStaticPriorities depends on the usage matrix only: on the transpose's stream, which is idle
    // once P is done (the side stream would hold it behind the small groups' Minimize) and ordered
    // after the job's begin on `stream` (uses must be ready there by then), joined before
    // CalculatePriorities
    hipStream_t ss = J.begun && c.part ? c.part : s;
    const uint32_t* dserr = static_priorities_enqueue(uses, nkeys, C, static_prios, ss);
    RawEndArgs e;
    e.C = C;
    e.count_hist = count_hist;
    e.selected = selected;
    e.len_hist = len_hist;
    e.out_idx = out_idx;
    e.group_out_off = group_out_off;
    e.s = s;
    e.defer_check = true;
    minimize_raw_end(J, e);
    if (ss != s) {
      SYZ_HIP(hipEventRecord(c.ev_part1, ss));
      SYZ_HIP(hipStreamWaitEvent(s, c.ev_part1, 0));
    }
    prio_choice_dev(static_prios, len_hist, nullptr, C, nullptr, prios, run, row_present, s);
    uint32_t* h = c.pinned.get<uint32_t>(8);
    SYZ_HIP(hipMemcpyAsync(h, c.scratch.get<int>("mz_err", 2), 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(h + 1, dserr, 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    minimize_raw_end_check((int)h[0]);
    static_prio_check(h[1]);
  })
}

int syzgpu_mz_fetch(syzgpu_mz* job, int64_t* out_idx, uint64_t* group_out_off) {
  SYZ_API_BODY({
    if (!job || !group_out_off) fail(SYZGPU_EINVAL, "null pointer");
    MinJob& J = *reinterpret_cast<MinJob*>(job);
    std::lock_guard<std::recursive_mutex> hl_(J.mu);
    minimize_raw_fetch(J, out_idx, group_out_off);
  })
}

int syzgpu_mz_info(syzgpu_mz* job, uint64_t* info, size_t cap) {
  SYZ_API_BODY({
    if (!job || !info) fail(SYZGPU_EINVAL, "null pointer");
    MinJob& J = *reinterpret_cast<MinJob*>(job);
    std::lock_guard<std::recursive_mutex> hl_(J.mu);
    const uint64_t v[7] = {J.n, J.G, J.stats_total_pcs, J.stats_items_direct, J.stats_items_hash, J.spec_hits,
                           J.spec_misses};
    for (size_t i = 0; i < cap && i < 7; i++) info[i] = v[i];
  })
}

}  // extern "C"

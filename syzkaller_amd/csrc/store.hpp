// The resident corpus store (the device analog of syz-manager's mgr.corpus, manager.go:52-65),
// shared by Minimize (minimize.hip) and the manager's cover analytics (analytics.hip).
#pragma once
#include <atomic>
#include <map>
#include <vector>

#include "pipeline.hpp"

namespace syz {

#ifndef SYZ_WIN_BITS
#define SYZ_WIN_BITS 15
#endif
#ifndef SYZ_BM_WORDS
#define SYZ_BM_WORDS 6144
#endif
constexpr uint32_t WIN_BITS = SYZ_WIN_BITS;  // compile-time A/B knob (tools/gpu_libvariants.sh)
constexpr uint32_t WIN = 1u << WIN_BITS;  // ids per LDS window (u32 min-rank table = 128 KB)

constexpr uint32_t VEC = 8;                 // ids per 16-byte vector
constexpr uint64_t CHUNK_VECS_MIN = 1u << 14;  // vectors per work item: bounds of the per-store size
constexpr uint64_t CHUNK_VECS_MAX = 1u << 18;
constexpr uint32_t BM_WORDS = SYZ_BM_WORDS;  // LDS rank bitmap: 196608 ranks per pass at 6144
constexpr uint32_t RANK_NONE = 0xFFFFFFFFu;

struct VecWork {
  uint32_t g;     // call group
  uint32_t nids;  // ids in this window (<= WIN)
  uint64_t vbeg, vend;
  uint32_t gtab;  // RANK_NONE: sole chunk of its panel, emit directly; else index of a global table
  uint32_t win;   // id window of the panel (the unit of key-space sharding)
  uint64_t tbeg = 0, tend = 0;  // the panel's appended vectors (incremental index), walked after vbeg..vend
};

// the cover analytics of a store (analytics.hip), computed on first use and kept with it
struct CoverStats;
void corpus_stats_free(CoverStats*);

// Winning ranks of a window table (LDS or global) -> set bits of sel_bits (global rank bitmap).
// Ranks of call g lie in [gstart[g], gstart[g+1]). Winners are mostly early ranks (the longest covers
// come first in Go-sort order), so the first BM_WORDS*32 ranks of the call are deduplicated through
// an LDS bitmap (one bit-OR per kept input instead of one per id) and the rarer later ones go straight
// to sel_bits: one pass over the table whatever the call's size.
template <bool ATOMIC_READ = false, uint32_t BMW = BM_WORDS>
__device__ __forceinline__ void emit_winners(const uint32_t* tab, uint32_t nids, uint64_t gbase, uint64_t ng,
                                             uint32_t* bm, uint32_t* sel_bits) {
  const uint32_t span = (uint32_t)min<uint64_t>((uint64_t)BMW * 32, ng);
  const uint32_t words = (span + 31) / 32;
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) bm[i] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nids; i += blockDim.x) {
    const uint32_t r = ATOMIC_READ ? __hip_atomic_load(&tab[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tab[i];
    if (r == RANK_NONE) continue;
    const uint64_t lr = (uint64_t)r - gbase;
    if (lr < span)
      atomicOr(&bm[lr >> 5], 1u << (lr & 31));
    else
      atomicOr(&sel_bits[r >> 5], 1u << (r & 31));
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) {
    const uint32_t wv = bm[i];
    if (!wv) continue;
    const uint64_t gb = gbase + 32ull * i;
    const uint32_t sh = (uint32_t)(gb & 31);
    atomicOr(&sel_bits[gb >> 5], wv << sh);
    if (sh) {
      const uint32_t hi = wv >> (32 - sh);
      if (hi) atomicOr(&sel_bits[(gb >> 5) + 1], hi);
    }
  }
  __syncthreads();
}

template <class T>
struct DevArr {
  T* p = nullptr;
  size_t n = 0;
  void alloc(size_t count) {
    free();
    n = count;
    SYZ_HIP(hipMalloc(&p, (count ? count : 1) * sizeof(T)));
  }
  void ensure(size_t count) {  // at least count elements; the contents are not kept
    if (p && count <= n) return;
    alloc(count + count / 4 + 16);
  }
  void free() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

template <class T>
struct Grow {  // grow-only device buffer owned by a handle
  T* p = nullptr;
  size_t cap = 0;
  void ensure(size_t count) {
    if (count <= cap && p) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = count + count / 8 + 16;
    SYZ_HIP(hipMalloc(&p, want * sizeof(T)));
    cap = want;
  }
  ~Grow() {
    if (p) (void)hipFree(p);
  }
};

struct Corpus {
  std::recursive_mutex mu;  // one call on a store at a time (mgr.mu serialises them in the reference)
  Grow<uint32_t> sel_bits, rom, eor;  // the selection between minimize_begin and _end
  bool begun = false;
  size_t n = 0;
  uint32_t G = 0;
  uint64_t total_pcs = 0, total_ids = 0, total_vecs = 0;
  DevArr<uint64_t> off, gstart, gdict, el0;  // el0: the Go-sort keys, len(cov) << 32 | member
  DevArr<uint32_t> group, members, member_of, nwin, dict, gtabs, vmem;
  DevArr<uint32_t> gtchunks, gtdone;  // work items per shared window table, and their arrivals
  DevArr<uint16_t> prog_len, ids16;
  DevArr<VecWork> work;  // work items of the big call groups first, then those of the small ones
  std::vector<VecWork> hwork;
  size_t nbig_work = 0;                        // work items of the big call groups
  uint64_t big_entries = 0, big_pcs = 0;       // entries / PCs in call groups above GS_T_SEG
  std::vector<VecWork> hwork_all;              // every work item (hwork: those of this rank's key parts)
  uint64_t big_vecs_all = 0, big_vecs = 0;     // id vectors of the big groups: all / in hwork
  DevArr<uint8_t> count_hist;                  // groups counted in len_hist (set_parts); unset: all
  bool has_count_hist = false;
  DevArr<uint32_t> xg;                         // selection-exchange list (groups, byte offsets)
  DevArr<uint64_t> xo;
  std::vector<uint64_t> xkey;
  std::vector<uint64_t> hstart;
  GosortPlan gsplan;
  uint32_t max_prog_len = 0;
  uint32_t ngtabs = 0;
  CoverStats* stats = nullptr;
  // incremental maintenance (corpus_inc.hip): ids per call, the (call, PC) -> id lookup sorted by
  // call << 32 | PC, and whether appends/keeps have left dict/gdict behind (the analytics rebuild)
  std::vector<uint64_t> hnids;
  DevArr<uint64_t> sd_key, dl_key;  // main (sorted) and delta (sorted: the keys appended since the last
  DevArr<uint32_t> sd_id, dl_id;    // merge) dictionaries
  size_t sd_n = 0, dl_n = 0;
  bool part_stale = false;  // appends since the last group partition / work list (redone lazily)
  bool app_pending = false;  // entries [app_n0, the covers' n) appended, not yet indexed (next user)
  size_t app_n0 = 0;
  uint64_t app_L0 = 0;
  bool sd_built = false, incremental = false;
  std::vector<VecWork> hmain;  // the items over the panel-major body of the stream (no tails)
  std::map<std::pair<uint32_t, uint32_t>, std::pair<uint64_t, uint64_t>> ptail;  // panel -> appended range
  uint64_t tail0 = 0, chunk_vecs = 0;  // first appended vector (the tail), work-item size of the body
  DevArr<uint16_t> ids16b;             // relayout targets (swapped in)
  DevArr<uint32_t> vmemb;
  bool keep_pending = false;           // a keep not yet applied: mgr.corpus = the old entries keep_idx
  size_t keep_m = 0, keep_n0 = 0;
  DevArr<int64_t> keep_idx;
  ~Corpus() {
    corpus_stats_free(stats);
    off.free(); gstart.free(); gdict.free(); el0.free(); group.free(); members.free(); member_of.free(); nwin.free(); dict.free();
    gtchunks.free(); gtdone.free(); count_hist.free(); xg.free(); xo.free();
    gtabs.free(); vmem.free(); prog_len.free(); ids16.free(); work.free(); sd_key.free(); sd_id.free();
    dl_key.free(); dl_id.free();
    ids16b.free(); vmemb.free(); keep_idx.free();
  }
};

// ---- the index (minimize.hip) ----
Corpus* corpus_create_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, const uint16_t* prog_len,
                          size_t n, uint32_t G, hipStream_t s);
void corpus_set_parts(Corpus& K, const uint16_t* part, const uint16_t* nparts, const uint8_t* count_hist,
                      hipStream_t s);
void corpus_minimize_begin(Corpus& K, hipStream_t s);
void corpus_minimize_end(Corpus& K, int32_t C, uint8_t* selected, int64_t* len_hist, hipStream_t s);
void corpus_minimize_dev(Corpus& K, int32_t C, uint8_t* selected, int64_t* len_hist, hipStream_t s);
void corpus_sel_xchg(Corpus& K, const uint32_t* groups, const uint64_t* offsets, uint32_t ng, uint8_t* buf,
                     int import, hipStream_t s);
void corpus_partition(Corpus& K, std::vector<uint64_t>& hpcs, hipStream_t s);
void corpus_upload_work(Corpus& K, hipStream_t s);

// Device buffer that keeps its first `used` elements when it grows (appends); 1.5x headroom.
// test hook (syzgpu_debug_fail_grow): the k-th growth from now fails as an allocation failure would
// (atomic: lanes on other threads grow their buffers at the same time)
inline std::atomic<int>& grow_fail_countdown() {
  static std::atomic<int> k{0};
  return k;
}
template <class T>
void grow_keep(Grow<T>& g, size_t used, size_t need, hipStream_t s) {
  if (need <= g.cap && g.p) return;
  if (std::atomic<int>& k = grow_fail_countdown(); k.load(std::memory_order_relaxed) > 0) {
    int cur = k.load(std::memory_order_relaxed);
    while (cur > 0 && !k.compare_exchange_weak(cur, cur - 1)) {
    }
    if (cur == 1) fail(SYZGPU_ENOMEM, "forced growth failure (test hook)");
  }
  const size_t want = need + need / 2 + 16;
  T* p = nullptr;
  SYZ_HIP(hipMalloc(&p, want * sizeof(T)));
  if (used && g.p) SYZ_HIP(hipMemcpyAsync(p, g.p, used * sizeof(T), hipMemcpyDeviceToDevice, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (g.p) (void)hipFree(g.p);
  g.p = p;
  g.cap = want;
}

}  // namespace syz

// syz-fuzzer's new-coverage check over a batch (syz-fuzzer/fuzzer.go:446-470 execute; the same
// rule as syz-manager NewInput, manager.go:609-616):
//   for each cover k, in order:  diff := Difference(Difference(cov_k, maxCover[g_k]), flakes)
//                                if diff != {} { maxCover[g_k] = Union(maxCover[g_k], diff); new }
//
// Exact batch reformulation: a cover whose diff is empty adds nothing, so before
// cover k the table is maxCover0[g] u (every earlier cover of g minus flakes). Cover k is new iff one
// of its PCs - not 0xFFFFFFFF (foreach drops it, cover.go:81-102), not a flake, not in maxCover0[g]
// - occurs first, among the covers of g, in cover k. With items (g<<32|pc, rank) laid out in rank
// order (maxCover0 entries rank 0, cover k rank k+1) a STABLE sort by key puts every key's first
// occurrence at the head of its run, so one pass over run heads decides every key:
//   head rank 0         -> the PC was in maxCover0[g]: output
//   head rank k+1       -> unless pc is 0xFFFFFFFF or a flake: cover k is new, the PC is output
// The runs come out sorted by (g, pc), so the updated tables are an ordered compaction. A table that
// took at least one Union loses a 0xFFFFFFFF entry it had (Union also goes through foreach).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "pipeline.hpp"

namespace syz {


__global__ void k_nov_items_mc(const uint32_t* mc, const uint64_t* mc_off, uint32_t G, uint64_t total, uint64_t* keys,
                               uint32_t* vals, int* err) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = (uint32_t)upper_bound_dev<uint64_t>(mc_off, 0, G + 1, j) - 1;
    const uint32_t pc = mc[j];
    if (j > mc_off[g] && mc[j - 1] >= pc) atomicOr(err, 1);  // maxCover tables must be canonical
    keys[j] = ((uint64_t)g << 32) | pc;
    vals[j] = 0;
  }
}

// one wave per cover
__global__ __launch_bounds__(256) void k_nov_items_cov(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                       size_t n, uint32_t G, uint64_t base, uint64_t* keys,
                                                       uint32_t* vals, int* err) {
  const size_t k = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (k >= n) return;
  const uint32_t g = group[k];
  if (g >= G) {
    if (__lane_id() == 0) atomicOr(err, 2);
    return;
  }
  const uint64_t b = off[k], e = off[k + 1];
  for (uint64_t j = b + __lane_id(); j < e; j += 64) {
    const uint32_t pc = pcs[j];
    if (j > b && pcs[j - 1] >= pc) atomicOr(err, 4);  // covers must be canonical (executor.cc:572-585)
    keys[base + j] = ((uint64_t)g << 32) | pc;
    vals[base + j] = (uint32_t)(k + 1);
  }
}

__device__ __forceinline__ bool in_sorted(const uint32_t* a, uint64_t n, uint32_t v) {
  const uint64_t p = lower_bound_dev<uint32_t>(a, 0, n, v);
  return p < n && a[p] == v;
}

__global__ void k_nov_mark(const uint64_t* keys, const uint32_t* vals, uint64_t ni, const uint32_t* flakes,
                           uint64_t nflakes, uint8_t* is_new, uint8_t* updated, uint8_t* flag, uint64_t* sentpos,
                           uint32_t* nsent) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ni; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    uint8_t f = 0;
    if (i == 0 || keys[i - 1] != key) {
      const uint32_t r = vals[i];
      const uint32_t pc = (uint32_t)key;
      if (r == 0) {
        f = 1;
        if (pc == SENT) sentpos[atomicAdd(nsent, 1u)] = i;
      } else if (pc != SENT && !in_sorted(flakes, nflakes, pc)) {
        is_new[r - 1] = 1;
        updated[key >> 32] = 1;
        f = 1;
      }
    }
    flag[i] = f;
  }
}

__global__ void k_nov_sent(const uint64_t* keys, const uint64_t* sentpos, const uint32_t* nsent,
                           const uint8_t* updated, uint8_t* flag) {
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < *nsent; t += gridDim.x * blockDim.x) {
    const uint64_t i = sentpos[t];
    if (updated[keys[i] >> 32]) flag[i] = 0;
  }
}

__global__ void k_nov_out(const uint64_t* keys, const uint8_t* flag, const uint64_t* pos, uint64_t ni, uint32_t* out,
                          uint64_t cap, int* err) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ni; i += (uint64_t)gridDim.x * blockDim.x)
    if (flag[i]) {
      if (pos[i] < cap)
        out[pos[i]] = (uint32_t)keys[i];
      else
        atomicOr(err, 8);
    }
}

// flakes must be strictly increasing (binary-searched by k_nov_mark)
__global__ void k_nov_check_flakes(const uint32_t* fl, size_t n, int* err) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (fl[i - 1] >= fl[i]) atomicOr(err, 16);
}

// gfirst[g] = first sorted index whose group is >= g (ni if none), g in [0, G]
__global__ void k_group_first(const uint64_t* keys, uint64_t ni, uint32_t G, uint64_t* gfirst) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= ni; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t lo = i == 0 ? 0 : (keys[i - 1] >> 32) + 1;
    const uint64_t hi = i == ni ? G : (keys[i] >> 32);
    for (uint64_t g = lo; g <= hi && g <= G; g++) gfirst[g] = i;
  }
}

__global__ void k_gather_pos(const uint64_t* pos, const uint64_t* gfirst, uint32_t G, uint64_t* out_off) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g <= G; g += gridDim.x * blockDim.x)
    out_off[g] = pos[gfirst[g]];
}

static int key_bits(uint32_t G) {
  int b = 0;
  while (b < 32 && (1ull << b) < G) b++;
  return 32 + b;
}

// ---- keyed-table strategy -------------------------------------------------------------------
// Exact same rule, without sorting the ~ΣL items. Keys are (g, d) where d is the rank of the PC among
// every PC marked in the call (covers, tables, flakes) - order-preserving, so a table row scanned by d
// is the sorted maxCover. The ranks come from a bitmap over the whole u32 PC space (2^26 words,
// 512 MB) with a summary bit per 512-word page; per touched word DW[w] = {bits, rank of its bit 0} so
// one 16-B gather turns a PC into d. The first-occurrence table T has G rows of P+1 u32 columns
// (column P holds a table's 0xFFFFFFFF entry, which foreach never matches): EMPTY, OLD (the key is in
// maxCover0[g]), FLAKE, or KT_COVER + k (cover k is the first of g that holds the key); atomicMin
// never moves OLD or FLAKE. Bitmap, summary and T are
// kept EMPTY between calls: each call clears exactly what it touched.
constexpr uint64_t KT_WORDS = 1ull << 26;      // u64 words of the PC bitmap
constexpr uint32_t KT_PAGE_WORDS = 512;        // words per page (32768 PCs)
constexpr uint32_t KT_PAGES = 1u << 17;        // pages of the PC space
constexpr uint32_t KT_SUM_WORDS = KT_PAGES / 64;
constexpr uint32_t KT_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t KT_OLD = 0;    // the key is in maxCover0[g]
constexpr uint32_t KT_FLAKE = 1;  // a flake outside maxCover0[g]: never new, never output
constexpr uint32_t KT_COVER = 2;  // + k: cover k is the first of g with the key
constexpr int KT_BLOCK = 256;
constexpr int KT_ITEMS = 16;                   // table entries per thread in the scans
constexpr uint64_t KT_CHUNK = (uint64_t)KT_BLOCK * KT_ITEMS;

using u64a = unsigned long long;

__device__ __forceinline__ void kt_mark(u64a* bm, u64a* sum, uint32_t pc) {
  const uint32_t w = pc >> 6;
  const u64a bit = 1ull << (pc & 63);
  if (!(bm[w] & bit)) atomicOr(&bm[w], bit);  // a stale 0 only costs a redundant atomic
  const uint32_t p = w / KT_PAGE_WORDS;
  const u64a pb = 1ull << (p & 63);
  if (!(sum[p >> 6] & pb)) atomicOr(&sum[p >> 6], pb);
}

// DW[pc >> 5] = {the 32 bitmap bits, rank of its bit 0}: one 8-B gather per PC
__device__ __forceinline__ uint32_t kt_dense(const uint2* __restrict__ dw, uint32_t pc) {
  const uint2 q = dw[pc >> 5];
  return q.y + (uint32_t)__popc(q.x & ((1u << (pc & 31)) - 1));
}

// The two passes over the batch's PCs run on flat tiles of KT_TILE PCs (KT_TPC consecutive PCs per
// thread, 16-B loads) rather than one wave per cover, so every lane has KT_TPC independent gathers in
// flight whatever the cover lengths. tile_k0[b] = the cover holding PC b*KT_TILE; a tile stages the
// offsets of its covers in LDS and each thread walks its PCs' cover indices forward from a search.
constexpr int KT_TB = 256;
constexpr int KT_TPC = 16;
constexpr uint64_t KT_TILE = (uint64_t)KT_TB * KT_TPC;
constexpr uint32_t KT_TOFF = 1024;  // cover offsets staged per tile

// per cover: group check (err 2), and the tile starts that fall inside it
__global__ void k_kt_tiles(const uint64_t* __restrict__ off, const uint32_t* __restrict__ group, size_t n, uint32_t G,
                           uint64_t* tile_k0, int* err) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    if (group[k] >= G) atomicOr(err, 2);
    const uint64_t b = off[k], e = off[k + 1];
    for (uint64_t t = (b + KT_TILE - 1) / KT_TILE; t * KT_TILE < e; t++) tile_k0[t] = k;
  }
}

struct KtTile {
  uint64_t k0;
  uint32_t ns;
  const uint64_t* off;
  const uint64_t* soff;
  __device__ __forceinline__ uint64_t at(uint64_t k) const { return k - k0 < ns ? soff[k - k0] : off[k]; }
};

// Loads this thread's PCs [j0, j0 + KT_TPC) (clipped to L) and the cover index of each.
__device__ __forceinline__ int kt_tile_load(const uint32_t* __restrict__ pcs, uint64_t L, size_t n, const KtTile& T,
                                            uint64_t j0, uint32_t (&pc)[KT_TPC], uint32_t (&kk)[KT_TPC]) {
  if (j0 >= L) return 0;
  const int cnt = (int)(L - j0 < (uint64_t)KT_TPC ? L - j0 : KT_TPC);
  if (cnt == KT_TPC) {
    const uint4* p4 = reinterpret_cast<const uint4*>(pcs + j0);
#pragma unroll
    for (int q = 0; q < KT_TPC / 4; q++) {
      const uint4 x = p4[q];
      pc[4 * q] = x.x, pc[4 * q + 1] = x.y, pc[4 * q + 2] = x.z, pc[4 * q + 3] = x.w;
    }
  } else {
    for (int q = 0; q < KT_TPC; q++) pc[q] = q < cnt ? pcs[j0 + q] : 0;
  }
  // cover of j0: last k with off[k] <= j0
  uint64_t lo, hi;
  if (T.ns > 1 && T.soff[T.ns - 1] > j0)
    lo = T.k0 + upper_bound_dev<uint64_t>(T.soff, 0, T.ns, j0) - 1;
  else
    lo = upper_bound_dev<uint64_t>(T.off, T.k0 + (T.ns ? T.ns - 1 : 0), n + 1, j0) - 1;
  hi = T.at(lo + 1);
  uint64_t k = lo;
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    while (j0 + q >= hi && k + 1 < n) {
      k++;
      hi = T.at(k + 1);
    }
    kk[q] = (uint32_t)k;
  }
  return cnt;
}

__device__ __forceinline__ void kt_tile_stage(const uint64_t* off, size_t n, const uint64_t* tile_k0, uint64_t* soff,
                                              KtTile& T, uint64_t tile) {
  T.k0 = tile_k0[tile];
  T.off = off;
  T.soff = soff;
  const uint64_t avail = n + 1 - T.k0;
  T.ns = (uint32_t)(avail < KT_TOFF + 1 ? avail : KT_TOFF + 1);
  for (uint32_t i = threadIdx.x; i < T.ns; i += KT_TB) soff[i] = off[T.k0 + i];
  __syncthreads();
}

// pass 1: canonical check (err 4) and the PC bitmap
__global__ __launch_bounds__(KT_TB) void k_kt_mark_cov(const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off,
                                                       size_t n, uint64_t L, const uint64_t* __restrict__ tile_k0,
                                                       u64a* bm, u64a* sum, int* err) {
  __shared__ uint64_t soff[KT_TOFF + 1];
  KtTile T;
  kt_tile_stage(off, n, tile_k0, soff, T, blockIdx.x);
  const uint64_t j0 = blockIdx.x * KT_TILE + (uint64_t)threadIdx.x * KT_TPC;
  uint32_t pc[KT_TPC], kk[KT_TPC];
  const int cnt = kt_tile_load(pcs, L, n, T, j0, pc, kk);
  if (!cnt) return;
  uint32_t prev = j0 ? pcs[j0 - 1] : 0;
  bool bad = false;
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    if (q < cnt) {
      bad |= j0 + q > T.at(kk[q]) && prev >= pc[q];  // covers must be canonical (executor.cc:572-585)
      prev = pc[q];
    }
  }
  if (bad) atomicOr(err, 4);
  u64a word[KT_TPC];
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) word[q] = q < cnt && pc[q] != SENT ? bm[pc[q] >> 6] : ~0ull;
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    const u64a bit = 1ull << (pc[q] & 63);
    if (!(word[q] & bit)) {  // first sight (or a stale 0): set it and its page's summary bit
      atomicOr(&bm[pc[q] >> 6], bit);
      const uint32_t p = pc[q] >> 15;
      const u64a pb = 1ull << (p & 63);
      if (!(sum[p >> 6] & pb)) atomicOr(&sum[p >> 6], pb);  // one line for all pages: check first
    }
  }
}

// maxCover0 entries (err 1 when a table is not canonical) and flakes (err 16)
__global__ void k_kt_mark_tabs(const uint32_t* mc, const uint64_t* mc_off, uint32_t G, uint64_t M, const uint32_t* fl,
                               uint64_t nfl, u64a* bm, u64a* sum, int* err) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < M + nfl; j += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t pc;
    if (j < M) {
      const uint32_t g = (uint32_t)upper_bound_dev<uint64_t>(mc_off, 0, G + 1, j) - 1;
      pc = mc[j];
      if (j > mc_off[g] && mc[j - 1] >= pc) atomicOr(err, 1);
    } else {
      const uint64_t i = j - M;
      pc = fl[i];
      if (i > 0 && fl[i - 1] >= pc) atomicOr(err, 16);
    }
    if (pc != SENT) kt_mark(bm, sum, pc);
  }
}

// one block: the touched pages in order (plist), their number in ctl[0]
__global__ __launch_bounds__(1024) void k_kt_pages(const u64a* __restrict__ sum, uint32_t* plist, uint32_t* ctl) {
  __shared__ uint32_t lds[1024 / 64 + 1];
  const uint32_t t = threadIdx.x;
  const u64a a = sum[2 * t], b = sum[2 * t + 1];
  uint32_t tot;
  uint32_t pos = block_excl_scan<1024>((uint32_t)(__popcll(a) + __popcll(b)), lds, &tot);
  for (int h = 0; h < 2; h++) {
    u64a m = h ? b : a;
    while (m) {
      const int i = __ffsll((long long)m) - 1;
      m &= m - 1;
      plist[pos++] = (2 * t + h) * 64 + i;
    }
  }
  if (t == 0) ctl[0] = tot;
}

// block per touched page: its number of marked PCs
__global__ __launch_bounds__(KT_PAGE_WORDS) void k_kt_pcount(const u64a* __restrict__ bm, const uint32_t* plist,
                                                             uint32_t* pcnt) {
  __shared__ uint32_t lds[KT_PAGE_WORDS / 64 + 1];
  const uint64_t w = (uint64_t)plist[blockIdx.x] * KT_PAGE_WORDS + threadIdx.x;
  const uint32_t c = block_sum<KT_PAGE_WORDS>((uint32_t)__popcll(bm[w]), lds);
  if (threadIdx.x == 0) pcnt[blockIdx.x] = c;
}

// block per touched page: DW for each word, pc_of for each marked PC
__global__ __launch_bounds__(KT_PAGE_WORDS) void k_kt_dense(const u64a* __restrict__ bm, const uint32_t* plist,
                                                            const uint64_t* ppre, uint2* dw, uint32_t* pc_of) {
  __shared__ uint32_t lds[KT_PAGE_WORDS / 64 + 1];
  const uint64_t w = (uint64_t)plist[blockIdx.x] * KT_PAGE_WORDS + threadIdx.x;
  u64a m = bm[w];
  uint32_t tot;
  uint32_t d = (uint32_t)ppre[blockIdx.x] + block_excl_scan<KT_PAGE_WORDS>((uint32_t)__popcll(m), lds, &tot);
  dw[2 * w] = make_uint2((uint32_t)m, d);
  dw[2 * w + 1] = make_uint2((uint32_t)(m >> 32), d + (uint32_t)__popc((uint32_t)m));
  while (m) {
    const int i = __ffsll((long long)m) - 1;
    m &= m - 1;
    pc_of[d++] = (uint32_t)(w << 6) | (uint32_t)i;
  }
}

// flakes -> FLAKE in every row (run first), then maxCover0 keys -> OLD (a flake in a table stays in it)
__global__ void k_kt_init_flakes(const uint32_t* fl, uint64_t nfl, uint32_t G, const uint2* __restrict__ dw, uint64_t P,
                                 uint32_t* tab) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nfl * G; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t pc = fl[j % nfl];
    if (pc != SENT) tab[(j / nfl) * (P + 1) + kt_dense(dw, pc)] = KT_FLAKE;
  }
}

__global__ void k_kt_init_mc(const uint32_t* mc, const uint64_t* mc_off, uint32_t G, uint64_t M,
                             const uint2* __restrict__ dw, uint64_t P, uint32_t* tab) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < M; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = (uint32_t)upper_bound_dev<uint64_t>(mc_off, 0, G + 1, j) - 1;
    const uint32_t pc = mc[j];
    tab[(uint64_t)g * (P + 1) + (pc == SENT ? P : kt_dense(dw, pc))] = KT_OLD;
  }
}

// pass 2: T[g][d] = min(T[g][d], KT_COVER + k) over the keys that are not 0xFFFFFFFF (flakes hold
// FLAKE, which the min never moves). Cover order, not group order: measured faster (10.5 vs 11.3 ms
// at config 3), as resident waves then spread their atomics over many rows instead of racing on the
// hot keys of one row.
__global__ __launch_bounds__(KT_TB) void k_kt_first(const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off,
                                                    const uint32_t* __restrict__ group, size_t n, uint64_t L, uint32_t G,
                                                    const uint64_t* __restrict__ tile_k0, const uint2* __restrict__ dw,
                                                    uint64_t P, uint32_t* tab) {
  __shared__ uint64_t soff[KT_TOFF + 1];
  KtTile T;
  kt_tile_stage(off, n, tile_k0, soff, T, blockIdx.x);
  const uint64_t j0 = blockIdx.x * KT_TILE + (uint64_t)threadIdx.x * KT_TPC;
  uint32_t pc[KT_TPC], kk[KT_TPC];
  const int cnt = kt_tile_load(pcs, L, n, T, j0, pc, kk);
  if (!cnt) return;
  uint2 q2[KT_TPC];
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) q2[q] = dw[pc[q] >> 5];
  uint32_t gg[KT_TPC];
  uint32_t last_k = ~0u, last_g = 0;
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    if (kk[q] != last_k) last_k = kk[q], last_g = group[kk[q]];
    gg[q] = last_g;
  }
  uint64_t idx[KT_TPC];
  uint32_t cur[KT_TPC];
  bool ok[KT_TPC];
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    const uint32_t d = q2[q].y + (uint32_t)__popc(q2[q].x & ((1u << (pc[q] & 31)) - 1));
    ok[q] = q < cnt && pc[q] != SENT && gg[q] < G;
    idx[q] = ok[q] ? (uint64_t)gg[q] * (P + 1) + d : 0;
    cur[q] = ok[q] ? tab[idx[q]] : 0;
  }
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    const uint32_t me = kk[q] + KT_COVER;
    if (ok[q] && cur[q] > me) atomicMin(&tab[idx[q]], me);  // a stale larger value only costs an atomic
  }
}

// per chunk of KT_CHUNK table entries: kept keys (cnt), is_new of every winning cover, updated rows
__global__ __launch_bounds__(KT_BLOCK) void k_kt_count(const uint32_t* __restrict__ tab, uint64_t P,
                                                       uint8_t* is_new, uint8_t* upd, uint32_t* cnt) {
  __shared__ uint32_t lds[KT_BLOCK / 64 + 1];
  const uint64_t i0 = blockIdx.x * KT_CHUNK + (uint64_t)threadIdx.x * KT_ITEMS;
  const uint4* t4 = reinterpret_cast<const uint4*>(tab + i0);
  uint32_t v[KT_ITEMS];
#pragma unroll
  for (int q = 0; q < KT_ITEMS / 4; q++) {
    const uint4 x = t4[q];
    v[4 * q] = x.x, v[4 * q + 1] = x.y, v[4 * q + 2] = x.z, v[4 * q + 3] = x.w;
  }
  uint32_t c = 0;
  uint64_t g = i0 / (P + 1), col = i0 - g * (P + 1), gnew = ~0ull;
#pragma unroll
  for (int q = 0; q < KT_ITEMS; q++) {
    if (v[q] != KT_EMPTY && v[q] != KT_FLAKE) {
      c++;
      if (v[q] != KT_OLD) {
        is_new[v[q] - KT_COVER] = 1;
        if (g != gnew) {
          upd[g] = 1;
          gnew = g;
        }
      }
    }
    if (++col == P + 1) col = 0, g++;
  }
  const uint32_t tot = block_sum<KT_BLOCK>(c, lds);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// a table that took a Union loses its 0xFFFFFFFF entry (Union goes through foreach)
__global__ void k_kt_sentfix(uint32_t* tab, uint32_t G, uint64_t P, const uint8_t* upd, uint32_t* cnt) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    const uint64_t i = (uint64_t)g * (P + 1) + P;
    if (upd[g] && tab[i] == KT_OLD) {
      tab[i] = KT_EMPTY;
      atomicSub(&cnt[i / KT_CHUNK], 1u);
    }
  }
}

// per chunk: compact kept keys into out (sorted by (g, pc)), row starts into ooff, table back to EMPTY
__global__ __launch_bounds__(KT_BLOCK) void k_kt_emit(uint32_t* tab, uint64_t E, uint64_t P, uint32_t G,
                                                      const uint64_t* cpre, uint64_t nchunks,
                                                      const uint32_t* __restrict__ pc_of, uint32_t* out, uint64_t cap,
                                                      uint64_t* ooff, int* err) {
  __shared__ uint32_t lds[KT_BLOCK / 64 + 1];
  const uint64_t i0 = blockIdx.x * KT_CHUNK + (uint64_t)threadIdx.x * KT_ITEMS;
  uint4* t4 = reinterpret_cast<uint4*>(tab + i0);
  uint32_t v[KT_ITEMS];
#pragma unroll
  for (int q = 0; q < KT_ITEMS / 4; q++) {
    const uint4 x = t4[q];
    v[4 * q] = x.x, v[4 * q + 1] = x.y, v[4 * q + 2] = x.z, v[4 * q + 3] = x.w;
  }
  uint32_t c = 0;
  bool dirty = false;
#pragma unroll
  for (int q = 0; q < KT_ITEMS; q++) {
    c += v[q] != KT_EMPTY && v[q] != KT_FLAKE;
    dirty |= v[q] != KT_EMPTY;
  }
  uint32_t tot;
  uint64_t pos = cpre[blockIdx.x] + block_excl_scan<KT_BLOCK>(c, lds, &tot);
  uint64_t g = i0 / (P + 1), col = i0 - g * (P + 1);
  for (int q = 0; q < KT_ITEMS; q++) {
    if (col == 0 && i0 + q < E) ooff[g] = pos;
    if (v[q] != KT_EMPTY && v[q] != KT_FLAKE) {
      if (pos < cap)
        out[pos] = pc_of[col];
      else
        atomicOr(err, 8);
      pos++;
    }
    if (++col == P + 1) col = 0, g++;
  }
  if (dirty) {
    const uint4 e4 = make_uint4(KT_EMPTY, KT_EMPTY, KT_EMPTY, KT_EMPTY);
#pragma unroll
    for (int q = 0; q < KT_ITEMS / 4; q++) t4[q] = e4;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) ooff[G] = cpre[nchunks];
}

// block per touched page: the bitmap back to zero
__global__ __launch_bounds__(KT_PAGE_WORDS) void k_kt_clear(u64a* bm, const uint32_t* plist) {
  bm[(uint64_t)plist[blockIdx.x] * KT_PAGE_WORDS + threadIdx.x] = 0;
}

// ---- per-call keys (SYZGPU_NOVELTY=keys): T is indexed by the (call, PC) pairs that occur, not by
// G x (P+1) ------------------------------------------------------------------------------------------
// B[g] is a bitmap over the dense PC ids d (P+1 columns, column P = the table sentinel) marking the
// keys call g holds (in a cover or in maxCover0[g]); BR[g][w] = {bits, rank of bit 0 over every row}
// turns (g, d) into e, the key's index in T (E2 = every call's distinct keys, ≈ a tenth of G x (P+1)
// at config 3), and row order stays PC order, so the emit is still an ordered compaction.
struct Bw {  // one 64-key word of B with the rank of its first key
  u64a bits;
  uint64_t rank;
};

__device__ __forceinline__ uint64_t kb_key(const Bw* __restrict__ br, uint64_t wpr, uint32_t g, uint32_t d) {
  const Bw q = br[(uint64_t)g * wpr + (d >> 6)];
  return q.rank + (uint64_t)__popcll(q.bits & ((1ull << (d & 63)) - 1));
}

// B from the covers (PCs other than 0xFFFFFFFF) ...
__global__ __launch_bounds__(KT_TB) void k_kb_mark_cov(const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ group, size_t n, uint64_t L,
                                                       uint32_t G, const uint64_t* __restrict__ tile_k0,
                                                       const uint2* __restrict__ dw, uint64_t wpr, u64a* B) {
  __shared__ uint64_t soff[KT_TOFF + 1];
  KtTile T;
  kt_tile_stage(off, n, tile_k0, soff, T, blockIdx.x);
  const uint64_t j0 = blockIdx.x * KT_TILE + (uint64_t)threadIdx.x * KT_TPC;
  uint32_t pc[KT_TPC], kk[KT_TPC];
  const int cnt = kt_tile_load(pcs, L, n, T, j0, pc, kk);
  if (!cnt) return;
  uint2 q2[KT_TPC];
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) q2[q] = dw[pc[q] >> 5];
  uint32_t last_k = ~0u, last_g = 0;
  uint64_t w[KT_TPC];
  u64a bit[KT_TPC], cur[KT_TPC];
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    if (kk[q] != last_k) last_k = kk[q], last_g = group[kk[q]];
    const bool ok = q < cnt && pc[q] != SENT && last_g < G;
    const uint32_t d = q2[q].y + (uint32_t)__popc(q2[q].x & ((1u << (pc[q] & 31)) - 1));
    w[q] = ok ? (uint64_t)last_g * wpr + (d >> 6) : ~0ull;
    bit[q] = 1ull << (d & 63);
    cur[q] = ok ? B[w[q]] : ~0ull;
  }
#pragma unroll
  for (int q = 0; q < KT_TPC; q++)
    if (!(cur[q] & bit[q])) atomicOr(&B[w[q]], bit[q]);  // a stale 0 only costs a redundant atomic
}

// ... and from maxCover0 (its 0xFFFFFFFF in column P)
__global__ void k_kb_mark_mc(const uint32_t* mc, const uint64_t* mc_off, uint32_t G, uint64_t M,
                             const uint2* __restrict__ dw, uint64_t P, uint64_t wpr, u64a* B) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < M; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = (uint32_t)upper_bound_dev<uint64_t>(mc_off, 0, G + 1, j) - 1;
    const uint32_t pc = mc[j];
    const uint64_t d = pc == SENT ? P : kt_dense(dw, pc);
    atomicOr(&B[(uint64_t)g * wpr + (d >> 6)], 1ull << (d & 63));
  }
}

__global__ void k_kb_popc(const u64a* __restrict__ B, uint64_t nw, uint32_t* cnt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x)
    cnt[i] = (uint32_t)__popcll(B[i]);
}

__global__ void k_kb_words(const u64a* __restrict__ B, const uint64_t* __restrict__ pre, uint64_t nw, Bw* br) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x)
    br[i] = Bw{B[i], pre[i]};
}

// flakes -> FLAKE where the call holds the key (run first), then maxCover0 keys -> OLD
__global__ void k_kb_init_flakes(const uint32_t* fl, uint64_t nfl, uint32_t G, const uint2* __restrict__ dw,
                                 const Bw* __restrict__ br, uint64_t wpr, uint32_t* tab) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nfl * G; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t pc = fl[j % nfl];
    const uint32_t g = (uint32_t)(j / nfl);
    if (pc == SENT) continue;
    const uint32_t d = kt_dense(dw, pc);
    const Bw q = br[(uint64_t)g * wpr + (d >> 6)];
    if ((q.bits >> (d & 63)) & 1ull) tab[q.rank + (uint64_t)__popcll(q.bits & ((1ull << (d & 63)) - 1))] = KT_FLAKE;
  }
}

__global__ void k_kb_init_mc(const uint32_t* mc, const uint64_t* mc_off, uint32_t G, uint64_t M,
                             const uint2* __restrict__ dw, uint64_t P, const Bw* __restrict__ br, uint64_t wpr,
                             uint32_t* tab) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < M; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = (uint32_t)upper_bound_dev<uint64_t>(mc_off, 0, G + 1, j) - 1;
    const uint32_t pc = mc[j];
    tab[kb_key(br, wpr, g, pc == SENT ? (uint32_t)P : kt_dense(dw, pc))] = KT_OLD;
  }
}

// T[e(g, d)] = min(T, KT_COVER + k) over the covers' keys
__global__ __launch_bounds__(KT_TB) void k_kb_first(const uint32_t* __restrict__ pcs, const uint64_t* __restrict__ off,
                                                    const uint32_t* __restrict__ group, size_t n, uint64_t L, uint32_t G,
                                                    const uint64_t* __restrict__ tile_k0, const uint2* __restrict__ dw,
                                                    const Bw* __restrict__ br, uint64_t wpr, uint32_t* tab) {
  __shared__ uint64_t soff[KT_TOFF + 1];
  KtTile T;
  kt_tile_stage(off, n, tile_k0, soff, T, blockIdx.x);
  const uint64_t j0 = blockIdx.x * KT_TILE + (uint64_t)threadIdx.x * KT_TPC;
  uint32_t pc[KT_TPC], kk[KT_TPC];
  const int cnt = kt_tile_load(pcs, L, n, T, j0, pc, kk);
  if (!cnt) return;
  uint2 q2[KT_TPC];
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) q2[q] = dw[pc[q] >> 5];
  uint32_t last_k = ~0u, last_g = 0;
  Bw bq[KT_TPC];
  uint32_t dd[KT_TPC];
  bool ok[KT_TPC];
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    if (kk[q] != last_k) last_k = kk[q], last_g = group[kk[q]];
    ok[q] = q < cnt && pc[q] != SENT && last_g < G;
    dd[q] = q2[q].y + (uint32_t)__popc(q2[q].x & ((1u << (pc[q] & 31)) - 1));
    bq[q] = ok[q] ? br[(uint64_t)last_g * wpr + (dd[q] >> 6)] : Bw{0, 0};
  }
  uint64_t idx[KT_TPC];
  uint32_t cur[KT_TPC];
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    idx[q] = bq[q].rank + (uint64_t)__popcll(bq[q].bits & ((1ull << (dd[q] & 63)) - 1));
    cur[q] = ok[q] ? tab[idx[q]] : 0;
  }
#pragma unroll
  for (int q = 0; q < KT_TPC; q++) {
    const uint32_t me = kk[q] + KT_COVER;
    if (ok[q] && cur[q] > me) atomicMin(&tab[idx[q]], me);
  }
}

// per chunk of KB_WORDS words of B: kept keys, is_new of the winning covers, updated rows
constexpr int KB_ITEMS = 4;  // B words per thread
constexpr uint64_t KB_CHUNK = (uint64_t)KT_BLOCK * KB_ITEMS;
__global__ __launch_bounds__(KT_BLOCK) void k_kb_count(const Bw* __restrict__ br, uint64_t nw, uint64_t wpr,
                                                       const uint32_t* __restrict__ tab, uint8_t* is_new, uint8_t* upd,
                                                       uint32_t* cnt) {
  __shared__ uint32_t lds[KT_BLOCK / 64 + 1];
  const uint64_t w0 = blockIdx.x * KB_CHUNK + (uint64_t)threadIdx.x * KB_ITEMS;
  uint32_t c = 0;
  for (int q = 0; q < KB_ITEMS; q++) {
    const uint64_t w = w0 + q;
    if (w >= nw) break;
    const Bw b = br[w];
    const int nb = __popcll(b.bits);
    for (int i = 0; i < nb; i++) {
      const uint32_t v = tab[b.rank + i];
      if (v != KT_FLAKE && v != KT_EMPTY) {
        c++;
        if (v != KT_OLD) {
          is_new[v - KT_COVER] = 1;
          upd[w / wpr] = 1;
        }
      }
    }
  }
  const uint32_t tot = block_sum<KT_BLOCK>(c, lds);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// a table that took a Union loses its 0xFFFFFFFF entry (column P)
__global__ void k_kb_sentfix(const Bw* __restrict__ br, uint64_t wpr, uint64_t P, uint32_t G, const uint8_t* upd,
                             uint32_t* tab, uint32_t* cnt) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    const uint64_t w = (uint64_t)g * wpr + (P >> 6);
    const Bw b = br[w];
    if (!((b.bits >> (P & 63)) & 1ull)) continue;
    const uint64_t e = b.rank + (uint64_t)__popcll(b.bits & ((1ull << (P & 63)) - 1));
    if (upd[g] && tab[e] == KT_OLD) {
      tab[e] = KT_FLAKE;  // dropped like a flake
      atomicSub(&cnt[w / KB_CHUNK], 1u);
    }
  }
}

// per chunk: the kept keys in (g, pc) order, row starts into ooff
__global__ __launch_bounds__(KT_BLOCK) void k_kb_emit(const Bw* __restrict__ br, uint64_t nw, uint64_t wpr, uint32_t G,
                                                      const uint32_t* __restrict__ tab, const uint64_t* cpre,
                                                      uint64_t nchunks, const uint32_t* __restrict__ pc_of, uint32_t* out,
                                                      uint64_t cap, uint64_t* ooff, int* err) {
  __shared__ uint32_t lds[KT_BLOCK / 64 + 1];
  const uint64_t w0 = blockIdx.x * KB_CHUNK + (uint64_t)threadIdx.x * KB_ITEMS;
  uint32_t c = 0;
  for (int q = 0; q < KB_ITEMS; q++) {
    const uint64_t w = w0 + q;
    if (w >= nw) break;
    const Bw b = br[w];
    const int nb = __popcll(b.bits);
    for (int i = 0; i < nb; i++) c += tab[b.rank + i] < KT_EMPTY && tab[b.rank + i] != KT_FLAKE;
  }
  uint32_t tot;
  uint64_t pos = cpre[blockIdx.x] + block_excl_scan<KT_BLOCK>(c, lds, &tot);
  for (int q = 0; q < KB_ITEMS; q++) {
    const uint64_t w = w0 + q;
    if (w >= nw) break;
    if (w % wpr == 0) ooff[w / wpr] = pos;
    const Bw b = br[w];
    u64a m = b.bits;
    uint64_t e = b.rank;
    while (m) {
      const int i = __ffsll((long long)m) - 1;
      m &= m - 1;
      const uint32_t v = tab[e++];
      if (v != KT_FLAKE && v != KT_EMPTY) {
        if (pos < cap)
          out[pos] = pc_of[(w % wpr) * 64 + i];
        else
          atomicOr(err, 8);
        pos++;
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) ooff[G] = cpre[nchunks];
}

static int strategy();

static bool novelty_table(const uint32_t* d_pcs, const uint64_t* d_off, const uint32_t* d_grp, size_t n, uint64_t L,
                          uint32_t G,
                          const uint32_t* d_mc, const uint64_t* d_mco, uint64_t M, const uint32_t* d_fl,
                          size_t nflakes, uint8_t* d_new, uint32_t* d_out, size_t out_cap, uint64_t* d_ooff,
                          int* err, uint64_t table_budget, hipStream_t s) {
  Context& c = ctx();
  Scratch& sc = c.scratch;
  u64a* bm = sc.get_clean<u64a>("kt_bm", KT_WORDS, 0, s);
  u64a* sum = sc.get_clean<u64a>("kt_sum", KT_SUM_WORDS, 0, s);
  uint2* dw = sc.get<uint2>("kt_dw", 2 * KT_WORDS);
  uint32_t* plist = sc.get<uint32_t>("kt_plist", KT_PAGES);
  uint32_t* ctl = c.pinned.get<uint32_t>(4);
  uint32_t* d_ctl = sc.get<uint32_t>("kt_ctl", 4);
  const uint64_t ntiles = (L + KT_TILE - 1) / KT_TILE;
  uint64_t* tile_k0 = sc.get<uint64_t>("kt_tile_k0", ntiles + 1);
  {
    ProfScope ps("novelty_mark", s, L * 4 + n * 12 + 8 + (M + nflakes) * 4);
    if (n) {
      k_kt_tiles<<<grid_for(n, 256, 16384), 256, 0, s>>>(d_off, d_grp, n, G, tile_k0, err);
      SYZ_LAUNCHED();
    }
    if (ntiles) {
      k_kt_mark_cov<<<(unsigned)ntiles, KT_TB, 0, s>>>(d_pcs, d_off, n, L, tile_k0, bm, sum, err);
      SYZ_LAUNCHED();
    }
    if (M + nflakes) {
      k_kt_mark_tabs<<<grid_for(M + nflakes, 256, 16384), 256, 0, s>>>(d_mc, d_mco, G, M, d_fl, nflakes, bm, sum, err);
      SYZ_LAUNCHED();
    }
    k_kt_pages<<<1, 1024, 0, s>>>(sum, plist, d_ctl);
    SYZ_LAUNCHED();
  }
  SYZ_HIP(hipMemcpyAsync(ctl, d_ctl, 4, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint32_t npages = ctl[0];
  uint32_t* pcnt = sc.get<uint32_t>("kt_pcnt", npages + 1);
  uint64_t* ppre = sc.get<uint64_t>("kt_ppre", npages + 1);
  if (npages) {
    k_kt_pcount<<<npages, KT_PAGE_WORDS, 0, s>>>(bm, plist, pcnt);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(pcnt, ppre, npages, s);
  uint64_t* hP = c.pinned.get<uint64_t>(2);
  SYZ_HIP(hipMemcpyAsync(hP, ppre + npages, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint64_t P = hP[0];
  const uint64_t E = (uint64_t)G * (P + 1);
  const uint64_t nchunks = (E + KT_CHUNK - 1) / KT_CHUNK;
  const uint64_t wpr = (P + 1 + 63) / 64, nw = (uint64_t)G * wpr;  // per-call keys: B words
  const bool grid = strategy() != 3;  // SYZGPU_NOVELTY=keys: per-call keys
  auto release = [&]() {  // the bitmap and its summary back to zero
    if (npages) {
      k_kt_clear<<<npages, KT_PAGE_WORDS, 0, s>>>(bm, plist);
      SYZ_LAUNCHED();
    }
    SYZ_HIP(hipMemsetAsync(sum, 0, KT_SUM_WORDS * 8, s));
    SYZ_HIP(hipStreamSynchronize(s));
    sc.put_clean("kt_bm");
    sc.put_clean("kt_sum");
  };
  if (grid ? nchunks * KT_CHUNK * 4 > table_budget : nw * 36 > table_budget) {  // too big: sort instead
    release();
    return false;
  }
  if (!grid) {
    uint32_t* pc_of = sc.get<uint32_t>("kt_pcof", P + 1);
    u64a* B = sc.get<u64a>("kb_b", nw + 1);
    Bw* br = sc.get<Bw>("kb_br", nw + 1);
    uint32_t* wc = sc.get<uint32_t>("kb_wc", nw + 1);
    uint64_t* wpre = sc.get<uint64_t>("kb_wpre", nw + 1);
    uint8_t* upd = sc.get<uint8_t>("kt_upd", G + 1);
    const uint64_t nch = (nw + KB_CHUNK - 1) / KB_CHUNK;
    uint32_t* cnt = sc.get<uint32_t>("kt_cnt", nch + 1);
    uint64_t* cpre = sc.get<uint64_t>("kt_cpre", nch + 1);
    SYZ_HIP(hipMemsetAsync(upd, 0, G + 1, s));
    SYZ_HIP(hipMemsetAsync(B, 0, nw * 8, s));
    {
      ProfScope ps("novelty_dense", s, (M + nflakes) * 4 + nw * 40);
      if (npages) {
        k_kt_dense<<<npages, KT_PAGE_WORDS, 0, s>>>(bm, plist, ppre, dw, pc_of);
        SYZ_LAUNCHED();
      }
      SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)(pc_of + P), (int)SENT, 1, s));
    }
    {
      ProfScope ps("novelty_keys", s, L * 4 + n * 12 + 8 + M * 4);
      if (ntiles) {
        k_kb_mark_cov<<<(unsigned)ntiles, KT_TB, 0, s>>>(d_pcs, d_off, d_grp, n, L, G, tile_k0, dw, wpr, B);
        SYZ_LAUNCHED();
      }
      if (M) {
        k_kb_mark_mc<<<grid_for(M, 256, 16384), 256, 0, s>>>(d_mc, d_mco, G, M, dw, P, wpr, B);
        SYZ_LAUNCHED();
      }
      k_kb_popc<<<grid_for(nw, 256, 16384), 256, 0, s>>>(B, nw, wc);
      SYZ_LAUNCHED();
      exclusive_scan_u32(wc, wpre, nw, s);
      k_kb_words<<<grid_for(nw, 256, 16384), 256, 0, s>>>(B, wpre, nw, br);
      SYZ_LAUNCHED();
    }
    SYZ_HIP(hipMemcpyAsync(hP, wpre + nw, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    const uint64_t E2 = hP[0];
    if (E2 * 4 > table_budget) {
      release();
      return false;
    }
    uint32_t* tab = sc.get<uint32_t>("kb_tab", E2 + 1);
    SYZ_HIP(hipMemsetAsync(tab, 0xFF, (E2 + 1) * 4, s));
    {
      ProfScope ps("novelty_first", s, L * 4 + n * 12 + 8);
      if (nflakes) {
        k_kb_init_flakes<<<grid_for(nflakes * G, 256, 16384), 256, 0, s>>>(d_fl, nflakes, G, dw, br, wpr, tab);
        SYZ_LAUNCHED();
      }
      if (M) {
        k_kb_init_mc<<<grid_for(M, 256, 16384), 256, 0, s>>>(d_mc, d_mco, G, M, dw, P, br, wpr, tab);
        SYZ_LAUNCHED();
      }
      if (ntiles) {
        k_kb_first<<<(unsigned)ntiles, KT_TB, 0, s>>>(d_pcs, d_off, d_grp, n, L, G, tile_k0, dw, br, wpr, tab);
        SYZ_LAUNCHED();
      }
    }
    {
      ProfScope ps("novelty_emit", s, nw * 16 + E2 * 8);
      k_kb_count<<<(unsigned)nch, KT_BLOCK, 0, s>>>(br, nw, wpr, tab, d_new, upd, cnt);
      SYZ_LAUNCHED();
      k_kb_sentfix<<<grid_for(G, 256, 64), 256, 0, s>>>(br, wpr, P, G, upd, tab, cnt);
      SYZ_LAUNCHED();
      exclusive_scan_u32(cnt, cpre, nch, s);
      k_kb_emit<<<(unsigned)nch, KT_BLOCK, 0, s>>>(br, nw, wpr, G, tab, cpre, nch, pc_of, d_out, out_cap, d_ooff, err);
      SYZ_LAUNCHED();
    }
    release();
    return true;
  }
  uint32_t* pc_of = sc.get<uint32_t>("kt_pcof", P + 1);
  uint32_t* tab = sc.get_clean<uint32_t>("kt_tab", nchunks * KT_CHUNK, 0xFF, s);
  uint8_t* upd = sc.get<uint8_t>("kt_upd", G + 1);
  uint32_t* cnt = sc.get<uint32_t>("kt_cnt", nchunks + 1);
  uint64_t* cpre = sc.get<uint64_t>("kt_cpre", nchunks + 1);
  SYZ_HIP(hipMemsetAsync(upd, 0, G + 1, s));
  {
    ProfScope ps("novelty_dense", s, (M + nflakes) * 4);
    if (npages) {
      k_kt_dense<<<npages, KT_PAGE_WORDS, 0, s>>>(bm, plist, ppre, dw, pc_of);
      SYZ_LAUNCHED();
    }
    SYZ_HIP(hipMemsetD32Async((hipDeviceptr_t)(pc_of + P), (int)SENT, 1, s));
    if (nflakes) {
      k_kt_init_flakes<<<grid_for(nflakes * G, 256, 16384), 256, 0, s>>>(d_fl, nflakes, G, dw, P, tab);
      SYZ_LAUNCHED();
    }
    if (M) {
      k_kt_init_mc<<<grid_for(M, 256, 16384), 256, 0, s>>>(d_mc, d_mco, G, M, dw, P, tab);
      SYZ_LAUNCHED();
    }
  }
  {
    ProfScope ps("novelty_first", s, L * 4 + n * 12 + 8);
    if (ntiles) {
      k_kt_first<<<(unsigned)ntiles, KT_TB, 0, s>>>(d_pcs, d_off, d_grp, n, L, G, tile_k0, dw, P, tab);
      SYZ_LAUNCHED();
    }
  }
  {
    ProfScope ps("novelty_emit", s, E * 8);
    k_kt_count<<<(unsigned)nchunks, KT_BLOCK, 0, s>>>(tab, P, d_new, upd, cnt);
    SYZ_LAUNCHED();
    k_kt_sentfix<<<grid_for(G, 256, 64), 256, 0, s>>>(tab, G, P, upd, cnt);
    SYZ_LAUNCHED();
    exclusive_scan_u32(cnt, cpre, nchunks, s);
    k_kt_emit<<<(unsigned)nchunks, KT_BLOCK, 0, s>>>(tab, E, P, G, cpre, nchunks, pc_of, d_out, out_cap, d_ooff, err);
    SYZ_LAUNCHED();
  }
  release();
  sc.put_clean("kt_tab");
  return true;
}

// Default: PC windows (novelty_win.hip) when the span fits them, else the keyed table over G x (P+1),
// else the radix sort. SYZGPU_NOVELTY=windows|table|sort|keys forces one (keys: the keyed table over
// per-call keys, measured 31.3 vs 14.6 ms for the G x (P+1) table at config 3). Tests run every one.
static int strategy() {
  const char* e = getenv("SYZGPU_NOVELTY");
  if (e && !strcmp(e, "sort")) return 1;
  if (e && !strcmp(e, "table")) return 2;
  if (e && !strcmp(e, "keys")) return 3;
  if (e && !strcmp(e, "windows")) return 4;
  if (e && !strcmp(e, "hwindows")) return 5;  // the windows, hashed whatever the span
  return 0;
}

// The keyed table is used while it stays under a quarter of free device memory (and 64 GB).
static uint64_t table_budget() {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
  const uint64_t b = fr / 4;
  return strategy() >= 2 ? ~0ull : std::min<uint64_t>(b, 64ull << 30);
}

static void check_errors(int* err, hipStream_t s);

bool novelty_windows(const uint32_t* d_pcs, const uint64_t* d_off, const uint32_t* d_grp, size_t n, uint32_t G,
                     const uint32_t* d_mc, const uint64_t* d_mco, const uint32_t* d_fl, size_t nfl, uint8_t* d_new,
                     uint32_t* d_out, size_t out_cap, uint64_t* d_ooff, int* err, bool force_hash, hipStream_t s);

// The batch on device-resident inputs: L = off[n] PCs in the covers, M = mc_off[G] in the tables.
// Writes is_new[n], out_mc[<= out_cap] and out_mc_off[G+1] on the device; the call returns after the
// stream has drained (it reports input errors and capacity).
void novelty_dev(const uint32_t* d_pcs, const uint64_t* d_off, const uint32_t* d_grp, size_t n, uint32_t G,
                 const uint32_t* d_mc, const uint64_t* d_mco, uint64_t M, const uint32_t* d_fl, size_t nflakes,
                 uint64_t L, uint8_t* d_new, uint32_t* d_out, size_t out_cap, uint64_t* d_ooff, hipStream_t s) {
  Context& c = ctx();
  Scratch& sc = c.scratch;
  if (G == 0) fail(SYZGPU_EINVAL, "ngroups must be > 0");
  if (n >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "too many covers in one batch");
  const uint64_t ni = L + M;
  int* err = sc.get<int>("nv_err", 2);
  SYZ_HIP(hipMemsetAsync(err, 0, 8, s));
  if (strategy() == 0 || strategy() >= 4) {  // (writes every is_new flag itself)
    if (nflakes > 1) {
      k_nov_check_flakes<<<grid_for(nflakes, 256, 1024), 256, 0, s>>>(d_fl, nflakes, err);
      SYZ_LAUNCHED();
    }
    if (novelty_windows(d_pcs, d_off, d_grp, n, G, d_mc, d_mco, d_fl, nflakes, d_new, d_out, out_cap, d_ooff, err,
                        strategy() == 5, s)) {
      check_errors(err, s);
      return;
    }
    // forced: no silent change of strategy
    if (strategy() >= 4) fail(SYZGPU_EINVAL, "novelty: the windows strategy cannot take this batch (ngroups > 4096)");
  }
  if (n) SYZ_HIP(hipMemsetAsync(d_new, 0, n, s));
  if (strategy() != 1 && novelty_table(d_pcs, d_off, d_grp, n, L, G, d_mc, d_mco, M, d_fl, nflakes, d_new, d_out, out_cap,
                                       d_ooff, err, table_budget(), s)) {
    check_errors(err, s);
    return;
  }
  uint64_t* keys = sc.get<uint64_t>("nv_keys", ni + 1);
  uint32_t* vals = sc.get<uint32_t>("nv_vals", ni + 1);
  uint64_t* ktmp = sc.get<uint64_t>("nv_ktmp", ni + 1);
  uint32_t* vtmp = sc.get<uint32_t>("nv_vtmp", ni + 1);
  uint8_t* upd = sc.get<uint8_t>("nv_upd", G + 1);
  uint8_t* flag = sc.get<uint8_t>("nv_flag", ni + 1);
  uint64_t* pos = sc.get<uint64_t>("nv_pos", ni + 1);
  uint64_t* sentpos = sc.get<uint64_t>("nv_sentpos", G + 1);
  uint32_t* nsent = sc.get<uint32_t>("nv_nsent", 1);
  uint64_t* gfirst = sc.get<uint64_t>("nv_gfirst", G + 1);
  SYZ_HIP(hipMemsetAsync(upd, 0, G + 1, s));
  SYZ_HIP(hipMemsetAsync(nsent, 0, 4, s));
  if (nflakes > 1) {
    k_nov_check_flakes<<<grid_for(nflakes, 256, 1024), 256, 0, s>>>(d_fl, nflakes, err);
    SYZ_LAUNCHED();
  }
  {
    ProfScope ps("novelty_items", s, ni * 16);
    if (M) {
      k_nov_items_mc<<<grid_for(M, 256, 16384), 256, 0, s>>>(d_mc, d_mco, G, M, keys, vals, err);
      SYZ_LAUNCHED();
    }
    if (n) {
      k_nov_items_cov<<<(unsigned)((n * 64 + 255) / 256), 256, 0, s>>>(d_pcs, d_off, d_grp, n, G, M, keys, vals, err);
      SYZ_LAUNCHED();
    }
  }
  {
    ProfScope ps("novelty_sort", s, ni * 12 * 2 * (uint64_t)((key_bits(G) + RADIX_BITS - 1) / RADIX_BITS));
    radix_sort_pairs(keys, vals, ktmp, vtmp, ni, key_bits(G), s);
  }
  {
    ProfScope ps("novelty_mark", s, ni * 13);
    if (ni) {
      k_nov_mark<<<grid_for(ni, 256, 65536), 256, 0, s>>>(keys, vals, ni, d_fl, nflakes, d_new, upd, flag, sentpos,
                                                        nsent);
      SYZ_LAUNCHED();
      k_nov_sent<<<grid_for(G, 256, 64), 256, 0, s>>>(keys, sentpos, nsent, upd, flag);
      SYZ_LAUNCHED();
    }
  }
  exclusive_scan_u8(flag, pos, ni, s);
  if (ni) {
    k_nov_out<<<grid_for(ni, 256, 65536), 256, 0, s>>>(keys, flag, pos, ni, d_out, out_cap, err);
    SYZ_LAUNCHED();
  }
  k_group_first<<<grid_for(ni + 1, 256, 65536), 256, 0, s>>>(keys, ni, G, gfirst);
  SYZ_LAUNCHED();
  k_gather_pos<<<grid_for(G + 1, 256, 1024), 256, 0, s>>>(pos, gfirst, G, d_ooff);
  SYZ_LAUNCHED();
  check_errors(err, s);
}

static void check_errors(int* err, hipStream_t s) {
  int herr[2];
  SYZ_HIP(hipMemcpyAsync(herr, err, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (herr[0] & 1) fail(SYZGPU_EINVAL, "maxCover tables must be canonical (strictly increasing)");
  if (herr[0] & 2) fail(SYZGPU_EINVAL, "group id >= ngroups");
  if (herr[0] & 4) fail(SYZGPU_EINVAL, "covers must be canonical (strictly increasing)");
  if (herr[0] & 16) fail(SYZGPU_EINVAL, "flakes must be canonical (strictly increasing)");
  if (herr[0] & 8) fail(SYZGPU_ECAPACITY, "out_mc capacity too small");
  if (herr[0] & 32) fail(SYZGPU_EINTERNAL, "novelty: a hashed window's table overflowed at one address per round");
}

void novelty_batch(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n, uint32_t G,
                   const uint32_t* mc, const uint64_t* mc_off, const uint32_t* flakes, size_t nflakes,
                   uint8_t* is_new, uint32_t* out_mc, size_t out_cap, uint64_t* out_mc_off) {
  Context& c = ctx();
  Scratch& sc = c.scratch;
  hipStream_t s = c.stream;
  if (G == 0) fail(SYZGPU_EINVAL, "ngroups must be > 0");
  if (!off || !mc_off || !out_mc_off || (n && (!group || !is_new))) fail(SYZGPU_EINVAL, "null pointer");
  if (off[0] != 0 || mc_off[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
  for (size_t i = 1; i < nflakes; i++)
    if (flakes[i - 1] >= flakes[i]) fail(SYZGPU_EINVAL, "flakes must be canonical (strictly increasing)");
  const uint64_t L = off[n], M = mc_off[G], ni = L + M;
  uint32_t* d_pcs = sc.get<uint32_t>("nv_pcs", L + 1);
  uint64_t* d_off = sc.get<uint64_t>("nv_off", n + 1);
  uint32_t* d_grp = sc.get<uint32_t>("nv_grp", n + 1);
  uint32_t* d_mc = sc.get<uint32_t>("nv_mc", M + 1);
  uint64_t* d_mco = sc.get<uint64_t>("nv_mco", G + 1);
  uint32_t* d_fl = sc.get<uint32_t>("nv_fl", nflakes + 1);
  uint8_t* d_new = sc.get<uint8_t>("nv_new", n + 1);
  uint64_t* d_ooff = sc.get<uint64_t>("nv_ooff", G + 1);
  uint32_t* d_out = sc.get<uint32_t>("nv_out", ni + 1);
  if (L) SYZ_HIP(hipMemcpyAsync(d_pcs, pcs, L * 4, hipMemcpyHostToDevice, s));
  SYZ_HIP(hipMemcpyAsync(d_off, off, (n + 1) * 8, hipMemcpyHostToDevice, s));
  if (n) SYZ_HIP(hipMemcpyAsync(d_grp, group, n * 4, hipMemcpyHostToDevice, s));
  if (M) SYZ_HIP(hipMemcpyAsync(d_mc, mc, M * 4, hipMemcpyHostToDevice, s));
  SYZ_HIP(hipMemcpyAsync(d_mco, mc_off, (G + 1) * 8, hipMemcpyHostToDevice, s));
  if (nflakes) SYZ_HIP(hipMemcpyAsync(d_fl, flakes, nflakes * 4, hipMemcpyHostToDevice, s));
  novelty_dev(d_pcs, d_off, d_grp, n, G, d_mc, d_mco, M, d_fl, nflakes, L, d_new, d_out, ni + 1, d_ooff, s);
  SYZ_HIP(hipMemcpyAsync(out_mc_off, d_ooff, (G + 1) * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint64_t total = out_mc_off[G];
  if (total > out_cap) fail(SYZGPU_ECAPACITY, "out_mc capacity too small");
  if (total) SYZ_HIP(hipMemcpyAsync(out_mc, d_out, total * 4, hipMemcpyDeviceToHost, s));
  if (n) SYZ_HIP(hipMemcpyAsync(is_new, d_new, n, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
}

}  // namespace syz

extern "C" int syzgpu_novelty_batch_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                                        uint32_t ngroups, const uint32_t* mc, const uint64_t* mc_off, size_t mc_total,
                                        const uint32_t* flakes, size_t nflakes, size_t total_pcs, uint8_t* is_new,
                                        uint32_t* out_mc, size_t out_cap, uint64_t* out_mc_off, void* stream) {
  SYZ_API_BODY({
    if (!off || !mc_off || !out_mc_off || (n && (!group || !is_new)) || (nflakes && !flakes))
      syz::fail(SYZGPU_EINVAL, "null pointer");
    syz::novelty_dev(pcs, off, group, n, ngroups, mc, mc_off, mc_total, flakes, nflakes, total_pcs, is_new, out_mc,
                     out_cap, out_mc_off, (hipStream_t)stream);
  })
}

extern "C" int syzgpu_novelty_batch(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                                    uint32_t ngroups, const uint32_t* mc, const uint64_t* mc_off,
                                    const uint32_t* flakes, size_t nflakes, uint8_t* is_new, uint32_t* out_mc,
                                    size_t out_cap, uint64_t* out_mc_off) {
  SYZ_API_BODY({
    syz::novelty_batch(pcs, off, group, n, ngroups, mc, mc_off, flakes, nflakes, is_new, out_mc, out_cap,
                       out_mc_off);
  })
}

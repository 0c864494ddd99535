// The manager's cover analytics (syz-manager/html.go) on the resident corpus store:
//   httpSummary  html.go:67-97   per call: inputs, len(Union of its covers), len(Intersection(that,
//                                uniqueCover(true))); the total cover len(Union over calls)
//   uniqueCover  html.go:213-237 PCs counted once over calls (perCall) or over inputs, Canonicalized
//   httpCorpus   html.go:158-170 per input: len(Intersection(inp.Cover, uniqueCover(false)))
//   httpCover    html.go:184-211 the PC lists themselves
// The store already holds every call's distinct PCs as dense ids (dict) and every cover as a
// panel-major id stream, so:
//   1. k_vec_uniq streams the panels once (like k_vec_min) and keeps, per (call, id), the only input
//      holding it or MULTI: an LDS table per work item, merged through the global table when a panel
//      spans several items;
//   2. the dictionary (one entry per (call, pc)) is radix-sorted by pc: a run of length 1 is a PC of
//      exactly one call (uniqueCover(true)), and such a PC held by one input is in exactly one input
//      overall (uniqueCover(false));
//   3. k_cs_runs walks the sorted dictionary once (coalesced): the totals, each call's and each
//      input's unique PCs, a flag per sorted entry; lists are ordered compactions of it.
// Union and Intersection go through foreach (cover.go:81-102) and never emit 0xFFFFFFFF; uniqueCover
// keeps it unless it is the only element (Canonicalize's `last := sent`, cover.go:28-40).
#include <algorithm>
#include <cstring>

#include "corpus.hpp"

namespace syz {

constexpr uint32_t UQ_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t UQ_MULTI = 0xFFFFFFFEu;
constexpr uint8_t CS_ONE_CALL = 1;   // the PC is in exactly one call's covers
constexpr uint8_t CS_ONE_INPUT = 2;  // ... and in exactly one input's cover

struct CoverStats {
  DevArr<VecWork> work;             // every panel's work items (all key parts), largest first
  DevArr<uint32_t> uq;              // per dict entry: the only member holding it, or UQ_MULTI
  DevArr<uint32_t> keys, ktmp;      // dictionary pcs, radix-sorted
  DevArr<uint32_t> vals, vtmp;      // ... and their dict index
  uint32_t* skeys = nullptr;        // the sorted halves (after the pointer swaps of the sort)
  uint32_t* svals = nullptr;
  DevArr<uint8_t> sflag;            // per sorted entry: CS_ONE_CALL | CS_ONE_INPUT
  DevArr<uint64_t> tot;             // [0] distinct pcs but 0xFFFFFFFF, [1] one-call pcs, [2] one-input pcs,
                                    // [3] 0xFFFFFFFF is one-call, [4] 0xFFFFFFFF is one-input
  DevArr<uint8_t> sentg;            // per call: its covers hold 0xFFFFFFFF
  DevArr<uint64_t> call_unique;     // per call
  DevArr<uint32_t> input_unique;    // per entry (corpus order)
  bool valid = false;
};

void corpus_stats_free(CoverStats* st) {
  if (!st) return;
  st->work.free(); st->uq.free(); st->keys.free(); st->ktmp.free(); st->vals.free(); st->vtmp.free();
  st->sflag.free(); st->tot.free(); st->sentg.free(); st->call_unique.free(); st->input_unique.free();
  delete st;
}

__device__ __forceinline__ void uq_apply(uint32_t* t, uint32_t id, uint32_t m) {
  uint32_t cur = t[id];
  if (cur == m || cur == UQ_MULTI) return;
  if (cur == UQ_EMPTY) {
    cur = atomicCAS(&t[id], UQ_EMPTY, m);
    if (cur == UQ_EMPTY || cur == m) return;
  }
  t[id] = UQ_MULTI;  // a second member: no CAS from EMPTY can follow, racing stores write the same
}

__device__ __forceinline__ void uq_vec(uint32_t* t, const uint4 q, uint32_t m) {
  uq_apply(t, q.x & 0xFFFF, m);
  uq_apply(t, q.x >> 16, m);
  uq_apply(t, q.y & 0xFFFF, m);
  uq_apply(t, q.y >> 16, m);
  uq_apply(t, q.z & 0xFFFF, m);
  uq_apply(t, q.z >> 16, m);
  uq_apply(t, q.w & 0xFFFF, m);
  uq_apply(t, q.w >> 16, m);
}

constexpr int UQ_BLOCK = 1024;
constexpr int UQ_DEPTH = 4;

// One workgroup per work item (grid-stride): the holder of every id of one window over a chunk of its
// stream. A sole chunk writes its table; a chunk of a split panel merges it with the same rule.
__global__ __launch_bounds__(UQ_BLOCK) void k_vec_uniq(const VecWork* __restrict__ work, uint32_t nitems,
                                                       const uint4* __restrict__ ids16,
                                                       const uint32_t* __restrict__ vmem,
                                                       const uint64_t* __restrict__ gdict, uint32_t* uq) {
  __shared__ uint32_t tab[WIN];
  for (uint32_t wi = blockIdx.x; wi < nitems; wi += gridDim.x) {
    const VecWork w = work[wi];
    for (uint32_t i = threadIdx.x; i < w.nids; i += UQ_BLOCK) tab[i] = UQ_EMPTY;
    __syncthreads();
    uint64_t v = w.vbeg + threadIdx.x;
    constexpr uint64_t STEP = (uint64_t)UQ_DEPTH * UQ_BLOCK;
    for (; v + (UQ_DEPTH - 1) * UQ_BLOCK < w.vend; v += STEP) {
      uint4 q[UQ_DEPTH];
      uint32_t m[UQ_DEPTH];
#pragma unroll
      for (int j = 0; j < UQ_DEPTH; j++) {
        q[j] = ids16[v + j * UQ_BLOCK];
        m[j] = vmem[v + j * UQ_BLOCK];
      }
#pragma unroll
      for (int j = 0; j < UQ_DEPTH; j++) uq_vec(tab, q[j], m[j]);
    }
    for (; v < w.vend; v += UQ_BLOCK) uq_vec(tab, ids16[v], vmem[v]);
    __syncthreads();
    uint32_t* dst = uq + gdict[w.g] + ((uint64_t)w.win << WIN_BITS);
    if (w.gtab == RANK_NONE) {
      for (uint32_t i = threadIdx.x; i < w.nids; i += UQ_BLOCK) dst[i] = tab[i];
    } else {
      for (uint32_t i = threadIdx.x; i < w.nids; i += UQ_BLOCK) {
        const uint32_t t = tab[i];
        if (t == UQ_EMPTY) continue;
        uint32_t cur = t == UQ_MULTI ? 0 : __hip_atomic_load(&dst[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t != UQ_MULTI) {
          if (cur == t || cur == UQ_MULTI) continue;
          if (cur == UQ_EMPTY) {
            cur = atomicCAS(&dst[i], UQ_EMPTY, t);
            if (cur == UQ_EMPTY || cur == t) continue;
          }
        }
        __hip_atomic_store(&dst[i], UQ_MULTI, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
  }
}

__global__ void k_cs_keys(const uint32_t* dict, uint64_t T, uint32_t* keys, uint32_t* vals) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < T; j += (uint64_t)gridDim.x * blockDim.x) {
    keys[j] = dict[j];
    vals[j] = (uint32_t)j;
  }
}

__device__ __forceinline__ uint32_t dict_group(const uint64_t* gdict, uint32_t G, uint64_t j) {
  return (uint32_t)upper_bound_dev<uint64_t>(gdict, 0, G + 1, j) - 1;
}

constexpr int CS_BLOCK = 256;
constexpr uint32_t CS_LDS_G = 8192;  // calls counted in LDS per block (more: global atomics)

// Over the sorted dictionary, coalesced: the flags of every sorted entry, the totals, each call's
// one-call PCs (per-block LDS counts) and each input's one-input PCs. Only the one-call entries
// look up their call (binary search of gdict) and their holder (uq).
__global__ __launch_bounds__(CS_BLOCK) void k_cs_runs(const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ vals, uint64_t T,
                                                      const uint32_t* __restrict__ uq,
                                                      const uint32_t* __restrict__ members,
                                                      const uint64_t* __restrict__ gdict, uint32_t G, uint8_t* sflag,
                                                      uint64_t* tot, uint8_t* sentg, uint64_t* call_unique,
                                                      uint32_t* input_unique) {
  extern __shared__ uint32_t ghist[];
  __shared__ uint64_t lds[CS_BLOCK / 64 + 1];
  const bool lds_g = G <= CS_LDS_G;
  if (lds_g)
    for (uint32_t g = threadIdx.x; g < G; g += CS_BLOCK) ghist[g] = 0;
  __syncthreads();
  uint64_t c0 = 0, c1 = 0, c2 = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * CS_BLOCK + threadIdx.x; i < T; i += (uint64_t)gridDim.x * CS_BLOCK) {
    const uint32_t k = keys[i];
    const bool head = i == 0 || keys[i - 1] != k;
    const bool single = head && (i + 1 == T || keys[i + 1] != k);
    const bool sent = k == SENT;
    uint8_t f = 0;
    c0 += head && !sent;
    if (single || sent) {
      const uint32_t j = vals[i];
      const uint32_t g = dict_group(gdict, G, j);
      if (sent) sentg[g] = 1;
      if (single) {
        const uint32_t u = uq[j];
        const bool one_input = u != UQ_MULTI;
        f = CS_ONE_CALL | (one_input ? CS_ONE_INPUT : 0);
        c1++;
        c2 += one_input;
        if (sent) {
          tot[3] = 1;
          if (one_input) tot[4] = 1;
        } else {
          if (lds_g)
            atomicAdd(&ghist[g], 1u);
          else
            atomicAdd((unsigned long long*)&call_unique[g], 1ull);
          if (one_input) atomicAdd(&input_unique[u], 1u);  // (the index's vectors name entries)
        }
      }
    }
    sflag[i] = f;
  }
  const uint64_t s0 = block_sum<CS_BLOCK>(c0, lds);
  const uint64_t s1 = block_sum<CS_BLOCK>(c1, lds);
  const uint64_t s2 = block_sum<CS_BLOCK>(c2, lds);
  if (threadIdx.x == 0) {
    if (s0) atomicAdd((unsigned long long*)&tot[0], (unsigned long long)s0);
    if (s1) atomicAdd((unsigned long long*)&tot[1], (unsigned long long)s1);
    if (s2) atomicAdd((unsigned long long*)&tot[2], (unsigned long long)s2);
  }
  if (lds_g)
    for (uint32_t g = threadIdx.x; g < G; g += CS_BLOCK)
      if (ghist[g]) atomicAdd((unsigned long long*)&call_unique[g], (unsigned long long)ghist[g]);
}

// list predicate over the sorted dictionary (see corpus_cover)
__global__ void k_cs_flag(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, uint64_t T,
                          const uint8_t* __restrict__ sflag, const uint64_t* __restrict__ gdict, int64_t call,
                          int unique, uint8_t* flag) {
  const uint8_t want = unique == 0 ? 0 : unique == 1 ? CS_ONE_CALL : CS_ONE_INPUT;
  const uint64_t jb = call >= 0 ? gdict[call] : 0, je = call >= 0 ? gdict[call + 1] : 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = keys[i];
    bool f;
    if (call < 0) {
      if (unique == 0)
        f = (i == 0 || keys[i - 1] != k) && k != SENT;
      else
        f = sflag[i] & want;
    } else {
      const uint32_t j = vals[i];
      f = j >= jb && j < je && k != SENT && (unique == 0 || (sflag[i] & want));
    }
    flag[i] = f;
  }
}

__global__ void k_cs_emit(const uint32_t* keys, const uint8_t* flag, const uint64_t* pos, uint64_t T, uint32_t* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += (uint64_t)gridDim.x * blockDim.x)
    if (flag[i]) out[pos[i]] = keys[i];
}

// Computes (or recomputes) the store's analytics on stream s.
static CoverStats& corpus_analyze(Corpus& K, hipStream_t s) {
  if (!K.stats) K.stats = new CoverStats();
  CoverStats& S = *K.stats;
  const uint64_t T = K.total_ids;
  const size_t n = K.n;
  if (!S.work.p) {
    std::vector<VecWork> hw = K.hwork_all;
    std::stable_sort(hw.begin(), hw.end(),
                     [](const VecWork& x, const VecWork& y) { return x.vend - x.vbeg > y.vend - y.vbeg; });
    S.work.alloc(hw.size());
    if (!hw.empty())
      SYZ_HIP(hipMemcpyAsync(S.work.p, hw.data(), hw.size() * sizeof(VecWork), hipMemcpyHostToDevice, s));
    S.uq.alloc(T);
    S.keys.alloc(T);
    S.ktmp.alloc(T);
    S.vals.alloc(T);
    S.vtmp.alloc(T);
    S.sflag.alloc(T);
    S.tot.alloc(5);
    S.sentg.alloc(K.G);
    S.call_unique.alloc(K.G);
    S.input_unique.alloc(n);
    SYZ_HIP(hipStreamSynchronize(s));  // hw is a host temporary
  }
  SYZ_HIP(hipMemsetAsync(S.tot.p, 0, 5 * 8, s));
  if (K.G) SYZ_HIP(hipMemsetAsync(S.sentg.p, 0, K.G, s));
  if (K.G) SYZ_HIP(hipMemsetAsync(S.call_unique.p, 0, K.G * 8, s));
  if (n) SYZ_HIP(hipMemsetAsync(S.input_unique.p, 0, n * 4, s));
  if (T) {
    SYZ_HIP(hipMemsetAsync(S.uq.p, 0xFF, T * 4, s));
    {
      ProfScope ps("cs_uniq", s, K.total_pcs * 4 + (uint64_t)n * 10);
      if (S.work.n && K.total_vecs) {
        const unsigned grid = (unsigned)std::min<size_t>(S.work.n, 1u << 20);
        k_vec_uniq<<<grid, UQ_BLOCK, 0, s>>>(S.work.p, (uint32_t)S.work.n, reinterpret_cast<const uint4*>(K.ids16.p),
                                             K.vmem.p, K.gdict.p, S.uq.p);
        SYZ_LAUNCHED();
      }
    }
    {
      ProfScope ps("cs_sort", s, T * 8 * 2 * 4);
      k_cs_keys<<<grid_for(T, 256, 8192), 256, 0, s>>>(K.dict.p, T, S.keys.p, S.vals.p);
      SYZ_LAUNCHED();
      uint32_t *k = S.keys.p, *kt = S.ktmp.p;
      uint32_t *v = S.vals.p, *vt = S.vtmp.p;
      radix_sort_pairs(k, v, kt, vt, T, 32, s);
      S.skeys = k;
      S.svals = v;
    }
    {
      ProfScope ps("cs_runs", s, T * 9);
      const size_t lds = K.G <= CS_LDS_G ? (size_t)K.G * 4 : 0;
      // few blocks: each flushes G call counts and 3 totals with atomics (same-address atomics serialize)
      k_cs_runs<<<grid_for(T, CS_BLOCK, 512), CS_BLOCK, lds, s>>>(S.skeys, S.svals, T, S.uq.p, nullptr,
                                                                  K.gdict.p, K.G, S.sflag.p, S.tot.p, S.sentg.p,
                                                                  S.call_unique.p, S.input_unique.p);
      SYZ_LAUNCHED();
    }
  }
  S.valid = true;
  return S;
}

__global__ void k_cs_percall(const uint64_t* gstart, const uint64_t* gdict, const uint8_t* sentg, uint32_t G,
                             uint64_t* call_inputs, uint64_t* call_cover) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    if (call_inputs) call_inputs[g] = gstart[g + 1] - gstart[g];
    if (call_cover) call_cover[g] = gdict[g + 1] - gdict[g] - sentg[g];
  }
}

// input_unique in entry order: the counts were added per entry already
__global__ void k_cs_totals(const uint64_t* tot, uint64_t* totals) {
  if (threadIdx.x == 0) {
    totals[0] = tot[0];
    totals[1] = tot[1] - (tot[1] == 1 && tot[3]);  // Canonicalize drops a lone 0xFFFFFFFF
    totals[2] = tot[2] - (tot[2] == 1 && tot[4]);
  }
}

static void corpus_cover_stats_dev(Corpus& K, uint64_t* call_inputs, uint64_t* call_cover, uint64_t* call_unique,
                                   uint64_t* totals, uint32_t* input_unique, hipStream_t s) {
  CoverStats& S = corpus_analyze(K, s);
  if (K.G && (call_inputs || call_cover)) {
    k_cs_percall<<<grid_for(K.G, 256, 64), 256, 0, s>>>(K.gstart.p, K.gdict.p, S.sentg.p, K.G, call_inputs,
                                                       call_cover);
    SYZ_LAUNCHED();
  }
  if (call_unique && K.G)
    SYZ_HIP(hipMemcpyAsync(call_unique, S.call_unique.p, K.G * 8, hipMemcpyDeviceToDevice, s));
  if (totals) {
    k_cs_totals<<<1, 64, 0, s>>>(S.tot.p, totals);
    SYZ_LAUNCHED();
  }
  if (input_unique && K.n)
    SYZ_HIP(hipMemcpyAsync(input_unique, S.input_unique.p, K.n * 4, hipMemcpyDeviceToDevice, s));
}

// httpCover's lists (html.go:186-211): call >= 0: that call's union, intersected with
// uniqueCover(unique == 1) when unique; call < 0: the union of all calls (unique == 0) or
// uniqueCover(unique == 1) itself. Returns the length; writes min(len, cap) PCs.
static uint64_t corpus_cover(Corpus& K, int64_t call, int unique, uint32_t* out_dev, uint64_t cap, hipStream_t s) {
  if (call >= (int64_t)K.G) fail(SYZGPU_EINVAL, "call group out of range");
  if (unique < 0 || unique > 2) fail(SYZGPU_EINVAL, "unique must be 0, 1 (per call) or 2 (per input)");
  if (!K.stats || !K.stats->valid) corpus_analyze(K, s);
  CoverStats& S = *K.stats;
  const uint64_t T = K.total_ids;
  if (!T) return 0;
  Scratch& sc = ctx().scratch;
  uint8_t* flag = sc.get<uint8_t>("cs_flag", T + 1);
  uint64_t* pos = sc.get<uint64_t>("cs_pos", T + 1);
  k_cs_flag<<<grid_for(T, 256, 8192), 256, 0, s>>>(S.skeys, S.svals, T, S.sflag.p, K.gdict.p, call, unique, flag);
  SYZ_LAUNCHED();
  exclusive_scan_u8(flag, pos, T, s);
  uint64_t len = 0, tot[5];
  SYZ_HIP(hipMemcpyAsync(&len, pos + T, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(tot, S.tot.p, 40, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (len > cap) return len;
  k_cs_emit<<<grid_for(T, 256, 8192), 256, 0, s>>>(S.skeys, flag, pos, T, out_dev);
  SYZ_LAUNCHED();
  if (call < 0 && unique && len == 1 && tot[unique == 1 ? 3 : 4]) len = 0;  // a lone 0xFFFFFFFF
  return len;
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzgpu_corpus_cover_stats_dev(syzgpu_corpus* cp, uint64_t* call_inputs, uint64_t* call_cover,
                                  uint64_t* call_unique, uint64_t* totals, uint32_t* input_unique, void* stream) {
  SYZ_API_BODY({
    if (!cp) fail(SYZGPU_EINVAL, "null corpus");
    CorpusHandle& H = *reinterpret_cast<CorpusHandle*>(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    corpus_cover_stats_dev(corpus_index_full(H, (hipStream_t)stream), call_inputs, call_cover, call_unique, totals,
                           input_unique, (hipStream_t)stream);
  })
}

int syzgpu_corpus_cover_stats(syzgpu_corpus* cp, uint64_t* call_inputs, uint64_t* call_cover, uint64_t* call_unique,
                              uint64_t* totals, uint32_t* input_unique) {
  SYZ_API_BODY({
    if (!cp) fail(SYZGPU_EINVAL, "null corpus");
    CorpusHandle& H = *reinterpret_cast<CorpusHandle*>(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    hipStream_t s = C_.stream;
    Corpus& K = corpus_index_full(H, s);
    const uint32_t G = K.G;
    const size_t n = K.n;
    uint64_t* d = C_.scratch.get<uint64_t>("cs_out", 3ull * G + 4);
    uint32_t* du = C_.scratch.get<uint32_t>("cs_out_u", n + 1);
    corpus_cover_stats_dev(K, d, d + G, d + 2ull * G, d + 3ull * G, du, s);
    std::vector<uint64_t> h(3ull * G + 3);
    SYZ_HIP(hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, s));
    if (input_unique && n) SYZ_HIP(hipMemcpyAsync(input_unique, du, n * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (call_inputs) memcpy(call_inputs, h.data(), G * 8);
    if (call_cover) memcpy(call_cover, h.data() + G, G * 8);
    if (call_unique) memcpy(call_unique, h.data() + 2ull * G, G * 8);
    if (totals) memcpy(totals, h.data() + 3ull * G, 3 * 8);
  })
}

int syzgpu_corpus_cover(syzgpu_corpus* cp, int64_t call, int unique, uint32_t* out, size_t cap, size_t* out_n) {
  SYZ_API_BODY({
    if (!cp || !out_n) fail(SYZGPU_EINVAL, "null pointer");
    CorpusHandle& H = *reinterpret_cast<CorpusHandle*>(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    hipStream_t s = C_.stream;
    Corpus& K = corpus_index_full(H, s);
    uint32_t* d = C_.scratch.get<uint32_t>("cs_list", K.total_ids + 1);
    const uint64_t len = corpus_cover(K, call, unique, d, K.total_ids + 1, s);
    *out_n = len;
    if (len > cap) fail(SYZGPU_ECAPACITY, "output capacity too small");
    if (len) SYZ_HIP(hipMemcpyAsync(out, d, len * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

}  // extern "C"

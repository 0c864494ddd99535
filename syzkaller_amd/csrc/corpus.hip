// syzgpu_corpus: syz-manager's mgr.corpus resident on the device (corpus.hpp).
//
//   create          mgr.corpus loaded (manager.go:52-65, 160-188): covers copied in, index built
//   append          NewInput: mgr.corpus = append(mgr.corpus, inp) (manager.go:609-616): the new covers
//                   are appended in place, O(new); the index goes stale
//   minimize        minimizeCorpus's per-call Minimize (manager.go:507-527): on the index when it is
//                   current (or key parts are set), else on the raw pipeline (panels.hip)
//   keep            mgr.corpus = newCorpus (manager.go:529): the kept entries, in the order given
//                   (minimizeCorpus's: call groups in order, each in Minimize's selection order),
//                   gathered into a fresh CSR; the index goes stale
//   minimize_keep   the two above as one call, the manager's whole minimizeCorpus
#include <algorithm>

#include "corpus.hpp"

namespace syz {

__global__ void k_shift_off(const uint64_t* off, size_t m, uint64_t base, uint64_t* out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i <= m; i += (size_t)gridDim.x * blockDim.x)
    out[i] = off[i] + base;
}

// bad[0] |= 1 for a call id >= G; bad[1] = max(bad[1], prog_len) (prog_len may be null)
__global__ void k_check_groups(const uint32_t* group, const uint16_t* prog_len, size_t m, uint32_t G,
                               uint32_t* bad) {
  uint32_t mx = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x) {
    if (group[i] >= G) atomicOr(bad, 1u);
    if (prog_len) mx = max(mx, (uint32_t)prog_len[i]);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t o = __shfl_xor(mx, d, 64);
    mx = o > mx ? o : mx;
  }
  if (__lane_id() == 0 && mx) atomicMax(&bad[1], mx);
}

// keep, metadata: the kept entries' cover lengths, call ids and program lengths, in output order
__global__ void k_keep_meta(const int64_t* idx, size_t m, size_t n, const uint64_t* off, const uint32_t* group,
                            const uint16_t* prog_len, uint32_t* len, uint32_t* group2, uint16_t* prog_len2,
                            uint32_t* info) {
  uint32_t mx = 0;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < m; t += (size_t)gridDim.x * blockDim.x) {
    const int64_t e = idx[t];
    if (e < 0 || (uint64_t)e >= n) {
      atomicOr(&info[0], 1u);
      len[t] = 0;
      group2[t] = 0;
      prog_len2[t] = 0;
      continue;
    }
    len[t] = (uint32_t)(off[e + 1] - off[e]);
    group2[t] = group[e];
    prog_len2[t] = prog_len[e];
    mx = max(mx, (uint32_t)prog_len[e]);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t o = __shfl_xor(mx, d, 64);
    mx = o > mx ? o : mx;
  }
  if (__lane_id() == 0 && mx) atomicMax(&info[1], mx);
}

// keep, covers: one wave per kept entry, 64 PCs per step (coalesced reads and writes)
__global__ __launch_bounds__(256) void k_keep_pcs(const int64_t* idx, size_t m, size_t n, const uint32_t* pcs,
                                                  const uint64_t* off, const uint64_t* off2, uint32_t* pcs2) {
  const unsigned lane = __lane_id();
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < m; t += waves) {
    const int64_t e = idx[t];
    if (e < 0 || (uint64_t)e >= n) continue;
    const uint64_t a = off[e], len = off[e + 1] - a, b = off2[t];
    for (uint64_t i = lane; i < len; i += 64) pcs2[b + i] = pcs[a + i];
  }
}

template <class T>
static void swap_grow(Grow<T>& a, Grow<T>& b) {
  std::swap(a.p, b.p);
  std::swap(a.cap, b.cap);
}

Corpus& corpus_index(CorpusHandle& H, hipStream_t s) {
  if (H.index && (H.index->keep_pending || H.index->app_pending || H.index->part_stale)) {
    try {
      corpus_index_sync(*H.index, H, s);
    } catch (...) {
      H.index.reset();
    }
  }
  if (!H.index) {
    H.index.reset(corpus_create_dev(H.pcs.p, H.off.p, H.group.p, H.prog_len.p, H.n, H.G, s));
    if (H.parts_set)
      corpus_set_parts(*H.index, H.part.data(), H.nparts.data(), H.has_count_hist ? H.count_hist.data() : nullptr, s);
  }
  return *H.index;
}

Corpus& corpus_index_full(CorpusHandle& H, hipStream_t s) {
  if (H.index && (H.index->incremental || H.index->app_pending)) H.index.reset();
  return corpus_index(H, s);
}

// the index (if any) follows a change of H's covers, or is dropped
template <class F>
static void index_follow(CorpusHandle& H, F f) {
  if (!H.index) return;
  if (H.parts_set || getenv("SYZGPU_NO_INC_INDEX")) {
    H.index.reset();
    return;
  }
  try {
    f(*H.index);
  } catch (...) {
    H.index.reset();
  }
}

void append_reserve(CorpusHandle& H, size_t m, uint64_t Lm, hipStream_t s) {
  const size_t n = H.n, nt = n + m;
  if (nt >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "too many corpus entries");
  grow_keep(H.pcs, H.L, H.L + Lm + 1, s);
  grow_keep(H.off, n + 1, nt + 1, s);
  grow_keep(H.group, n, nt + 1, s);
  grow_keep(H.prog_len, n, nt + 1, s);
}

// covers (device pointers) appended after H's current ones; prog_len may be null (zeros)
void append_covers(CorpusHandle& H, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                   const uint16_t* prog_len, size_t m, hipStream_t s, bool cc_update) {
  if (!off || (m && !group)) fail(SYZGPU_EINVAL, "null pointer");
  uint64_t* h = ctx().pinned.get<uint64_t>(3);
  uint32_t* bad = ctx().scratch.get<uint32_t>("co_bad", 2);
  SYZ_HIP(hipMemsetAsync(bad, 0, 8, s));
  if (m) {  // checked before anything changes, so a rejected append leaves the corpus as it was
    k_check_groups<<<grid_for(m, 256, 1024), 256, 0, s>>>(group, prog_len, m, H.G, bad);
    SYZ_LAUNCHED();
  }
  SYZ_HIP(hipMemcpyAsync(&h[0], off, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(&h[1], off + m, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(&h[2], bad, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));  // the append's one wait
  if (h[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
  const uint32_t* hb = reinterpret_cast<const uint32_t*>(&h[2]);
  if (hb[0]) fail(SYZGPU_EINVAL, "group id >= ngroups");
  const uint32_t maxlen = hb[1];
  const uint64_t Lm = h[1];
  if (Lm && !pcs) fail(SYZGPU_EINVAL, "null pointer");
  const size_t n = H.n, nt = n + m;
  const uint64_t L0 = H.L;
  append_reserve(H, m, Lm, s);  // (before corpusCover changes: a failed growth leaves everything as it was)
  if (cc_update) cc_add(H, pcs, off, group, m, Lm, s);  // corpusCover follows every append
  index_follow(H, [&](Corpus& K) {  // a recorded keep first (the appends before it are applied by it)
    if (K.keep_pending) corpus_index_sync(K, H, s);
  });
  if (Lm) SYZ_HIP(hipMemcpyAsync(H.pcs.p + H.L, pcs, Lm * 4, hipMemcpyDeviceToDevice, s));
  k_shift_off<<<grid_for(m + 1, 256, 4096), 256, 0, s>>>(off, m, H.L, H.off.p + n);
  SYZ_LAUNCHED();
  if (m) SYZ_HIP(hipMemcpyAsync(H.group.p + n, group, m * 4, hipMemcpyDeviceToDevice, s));
  if (m && prog_len) SYZ_HIP(hipMemcpyAsync(H.prog_len.p + n, prog_len, m * 2, hipMemcpyDeviceToDevice, s));
  if (m && !prog_len) SYZ_HIP(hipMemsetAsync(H.prog_len.p + n, 0, m * 2, s));
  H.max_prog_len = std::max(H.max_prog_len, maxlen);
  H.n = nt;
  H.L += Lm;
  H.path = 0;
  index_follow(H, [&](Corpus& K) { corpus_index_note_append(K, n, L0); });
}

static CorpusHandle* handle_create_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                       const uint16_t* prog_len, size_t n, uint32_t G, hipStream_t s) {
  if (G == 0 || G > 4096) fail(SYZGPU_EINVAL, "ngroups out of range (1..4096)");
  std::unique_ptr<CorpusHandle> H(new CorpusHandle());
  H->G = G;
  append_covers(*H, pcs, off, group, prog_len, n, s);  // (no index yet: nothing to follow)
  corpus_index(*H, s);  // validates the covers (canonical, group ids) and serves minimize at once
  SYZ_HIP(hipStreamSynchronize(s));
  return H.release();
}

// mgr.corpus = the entries idx[0..m) (device int64), in that order
// distinct: idx is minimize's kept list (in range, no entry twice), so the kept PCs fit the old
// count and the gather goes out before the one wait
static void keep_entries(CorpusHandle& H, const int64_t* idx, size_t m, hipStream_t s, bool distinct = false) {
  if (m && !idx) fail(SYZGPU_EINVAL, "null pointer");
  // corpusCover holds every cover the store has held: taken before a keep that may drop a call's PCs
  // (minimizeCorpus's keep without key parts cannot: Minimize keeps a first holder of every PC). The
  // distinct form comes only from minimize_keep, whose begin and end run back to back on this store
  // alone, so its selection covers every holder of every PC here; a multi-rank minimize (selections
  // exchanged between begin_dev and end_dev, where a rank may drop all its local holders of a PC) keeps
  // through syzgpu_corpus_keep[_dev], which is not distinct and builds corpusCover first.
  // Deliberate difference from manager.go:121 (corpusCover starts empty there): the store seeds it from
  // the covers it was created with, as if each had come through NewInput (manager.go:609-616), which is
  // how the manager's corpus entries get there.
  if (!distinct || H.parts_set) cc_ensure(H, s);
  index_follow(H, [&](Corpus& K) { corpus_index_sync(K, H, s); });  // a recorded keep first
  Scratch& sc = ctx().scratch;
  uint32_t* len = sc.get<uint32_t>("co_len", m + 1);
  uint32_t* info = sc.get<uint32_t>("co_info", 2);
  H.off2.ensure(m + 1);
  H.group2.ensure(m + 1);
  H.prog_len2.ensure(m + 1);
  SYZ_HIP(hipMemsetAsync(info, 0, 8, s));
  if (m) {
    k_keep_meta<<<grid_for(m, 256, 4096), 256, 0, s>>>(idx, m, H.n, H.off.p, H.group.p, H.prog_len.p, len,
                                                      H.group2.p, H.prog_len2.p, info);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(len, H.off2.p, m, s);
  uint64_t* h = ctx().pinned.get<uint64_t>(2);
  if (distinct) {
    H.pcs2.ensure(H.L + 1);
    if (m) {
      k_keep_pcs<<<grid_for(m * 64, 256, 65536), 256, 0, s>>>(idx, m, H.n, H.pcs.p, H.off.p, H.off2.p, H.pcs2.p);
      SYZ_LAUNCHED();
    }
  }
  SYZ_HIP(hipMemcpyAsync(&h[0], H.off2.p + m, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(&h[1], info, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint32_t* hi = reinterpret_cast<const uint32_t*>(&h[1]);
  if (hi[0]) fail(SYZGPU_EINVAL, "kept entry index out of range");
  const uint64_t L2 = m ? h[0] : 0;
  if (!distinct) {
    H.pcs2.ensure(L2 + 1);
    if (m && L2) {
      k_keep_pcs<<<grid_for(m * 64, 256, 65536), 256, 0, s>>>(idx, m, H.n, H.pcs.p, H.off.p, H.off2.p, H.pcs2.p);
      SYZ_LAUNCHED();
    }
    SYZ_HIP(hipStreamSynchronize(s));  // the old covers are the next keep's target
  }
  swap_grow(H.pcs, H.pcs2);
  swap_grow(H.off, H.off2);
  swap_grow(H.group, H.group2);
  swap_grow(H.prog_len, H.prog_len2);
  const size_t n0 = H.n;
  H.n = m;
  H.L = L2;
  H.max_prog_len = hi[1];
  H.path = 0;
  index_follow(H, [&](Corpus& K) { corpus_index_keep(K, H, idx, m, n0, s); });
}

static void handle_begin(CorpusHandle& H, hipStream_t s) {
  if (H.parts_set || H.index) {
    corpus_minimize_begin(corpus_index(H, s), s);
    H.path = 1;
  } else {
    RawMinArgs a{H.pcs.p, H.off.p, H.group.p, H.prog_len.p, H.n, H.G};
    a.s = s;
    minimize_raw_begin(H.job, a);
    H.path = 2;
  }
}

static void handle_xchg(CorpusHandle& H, const uint32_t* groups, const uint64_t* offsets, uint32_t ng, uint8_t* buf,
                        int import, hipStream_t s) {
  if (H.path == 1)
    corpus_sel_xchg(*H.index, groups, offsets, ng, buf, import, s);
  else if (H.path == 2)
    minimize_raw_xchg(H.job, groups, offsets, ng, buf, import, s);
  else
    fail(SYZGPU_EINVAL, "corpus: minimize_begin first");
}

static void handle_end(CorpusHandle& H, int32_t C, uint8_t* selected, int64_t* len_hist, int64_t* out_idx,
                       uint64_t* group_out_off, hipStream_t s) {
  if (len_hist && C <= 0) fail(SYZGPU_EINVAL, "len_hist needs C > 0");
  if (H.path == 1) {
    Corpus& K = *H.index;
    corpus_minimize_end(K, C, selected, len_hist, s);
    if (out_idx || group_out_off) {
      sel_compact_dev(K.sel_bits.p, K.eor.p, K.gstart.p, K.n, K.G, out_idx, group_out_off, s);
    }
  } else if (H.path == 2) {
    RawEndArgs e;
    e.C = C;
    e.selected = selected;
    e.len_hist = len_hist;
    e.out_idx = out_idx;
    e.group_out_off = group_out_off;
    e.s = s;
    minimize_raw_end(H.job, e);
  } else {
    fail(SYZGPU_EINVAL, "corpus: minimize_begin first");
  }
}

// minimizeCorpus + mgr.corpus = newCorpus; returns the kept count
static uint64_t minimize_keep(CorpusHandle& H, int32_t C, uint8_t* selected, int64_t* len_hist, int64_t* out_idx,
                              uint64_t* group_out_off, hipStream_t s) {
  Scratch& sc = ctx().scratch;
  PhaseTimer pt("minimize_keep");
  int64_t* out = out_idx ? out_idx : sc.get<int64_t>("co_out", H.n + 1);
  uint64_t* goff = group_out_off ? group_out_off : sc.get<uint64_t>("co_goff", H.G + 1);
  handle_begin(H, s);
  pt.mark(H.path == 1 ? "begin_index" : "begin_raw", s);
  handle_end(H, C, selected, len_hist, out, goff, s);
  pt.mark("end", s);
  uint64_t* h = ctx().pinned.get<uint64_t>(1);
  SYZ_HIP(hipMemcpyAsync(h, goff + H.G, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint64_t m = *h;
  keep_entries(H, out, m, s, true);
  pt.mark("keep", s);
  return m;
}

}  // namespace syz

using namespace syz;

namespace {
CorpusHandle& H_of(syzgpu_corpus* c) {
  if (!c) fail(SYZGPU_EINVAL, "null corpus");
  return *reinterpret_cast<CorpusHandle*>(c);
}
}  // namespace

extern "C" {

int syzgpu_corpus_create_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                             const uint16_t* prog_len, size_t n, uint32_t ngroups, void* stream,
                             syzgpu_corpus** out) {
  SYZ_API_BODY({
    if (!out || !off) fail(SYZGPU_EINVAL, "null pointer");
    *out = reinterpret_cast<syzgpu_corpus*>(
        handle_create_dev(pcs, off, group, prog_len, n, ngroups, (hipStream_t)stream));
  })
}

int syzgpu_corpus_create(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, const uint16_t* prog_len,
                         size_t n, uint32_t ngroups, syzgpu_corpus** out) {
  SYZ_API_BODY({
    if (!out || !off || (n && !group)) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    const uint64_t tot = off[n];
    uint32_t* dp = C_.scratch.get<uint32_t>("cc_pcs", tot + 1);
    uint64_t* doff = C_.scratch.get<uint64_t>("cc_off", n + 1);
    uint32_t* dg = C_.scratch.get<uint32_t>("cc_grp", n + 1);
    uint16_t* dl = prog_len ? C_.scratch.get<uint16_t>("cc_len", n + 1) : nullptr;
    if (tot) SYZ_HIP(hipMemcpyAsync(dp, pcs, tot * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(doff, off, (n + 1) * 8, hipMemcpyHostToDevice, s));
    if (n) SYZ_HIP(hipMemcpyAsync(dg, group, n * 4, hipMemcpyHostToDevice, s));
    if (dl && n) SYZ_HIP(hipMemcpyAsync(dl, prog_len, n * 2, hipMemcpyHostToDevice, s));
    *out = reinterpret_cast<syzgpu_corpus*>(handle_create_dev(dp, doff, dg, dl, n, ngroups, s));
  })
}

int syzgpu_corpus_destroy(syzgpu_corpus* cp) {
  SYZ_API_BODY({
    if (cp) {
      CorpusHandle* H = reinterpret_cast<CorpusHandle*>(cp);
      { std::lock_guard<std::recursive_mutex> hl_(H->mu); }
      delete H;
    }
  })
}

int syzgpu_corpus_append_dev(syzgpu_corpus* cp, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                             const uint16_t* prog_len, size_t n, void* stream, syzgpu_corpus** out) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    append_covers(H, pcs, off, group, prog_len, n, (hipStream_t)stream);
    if (out) *out = cp;
  })
}

int syzgpu_corpus_append(syzgpu_corpus* cp, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                         const uint16_t* prog_len, size_t n, syzgpu_corpus** out) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    if (!off || (n && !group)) fail(SYZGPU_EINVAL, "null pointer");
    if (off[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
    hipStream_t s = C_.stream;
    const uint64_t tot = off[n];
    uint32_t* dp = C_.scratch.get<uint32_t>("cc_pcs", tot + 1);
    uint64_t* doff = C_.scratch.get<uint64_t>("cc_off", n + 1);
    uint32_t* dg = C_.scratch.get<uint32_t>("cc_grp", n + 1);
    uint16_t* dl = prog_len ? C_.scratch.get<uint16_t>("cc_len", n + 1) : nullptr;
    if (tot) SYZ_HIP(hipMemcpyAsync(dp, pcs, tot * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(doff, off, (n + 1) * 8, hipMemcpyHostToDevice, s));
    if (n) SYZ_HIP(hipMemcpyAsync(dg, group, n * 4, hipMemcpyHostToDevice, s));
    if (dl && n) SYZ_HIP(hipMemcpyAsync(dl, prog_len, n * 2, hipMemcpyHostToDevice, s));
    append_covers(H, dp, doff, dg, dl, n, s);
    SYZ_HIP(hipStreamSynchronize(s));
    if (out) *out = cp;
  })
}

int syzgpu_corpus_new_inputs_dev(syzgpu_corpus* cp, const uint32_t* pcs, const uint64_t* off,
                                 const uint32_t* group, const uint16_t* prog_len, size_t n, uint8_t* is_new,
                                 void* stream, uint64_t* accepted) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    const uint64_t na = corpus_new_inputs(H, pcs, off, group, prog_len, n, is_new, (hipStream_t)stream);
    if (accepted) *accepted = na;
  })
}

int syzgpu_corpus_new_inputs(syzgpu_corpus* cp, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                             const uint16_t* prog_len, size_t n, uint8_t* is_new, uint64_t* accepted) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    if (!off || (n && !group)) fail(SYZGPU_EINVAL, "null pointer");
    if (off[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
    hipStream_t s = C_.stream;
    const uint64_t tot = off[n];
    uint32_t* dp = C_.scratch.get<uint32_t>("cc_hpcs", tot + 1);
    uint64_t* doff = C_.scratch.get<uint64_t>("cc_hoff", n + 1);
    uint32_t* dg = C_.scratch.get<uint32_t>("cc_hgrp", n + 1);
    uint16_t* dl = prog_len ? C_.scratch.get<uint16_t>("cc_hlen", n + 1) : nullptr;
    uint8_t* dn = C_.scratch.get<uint8_t>("cc_hnew", n + 1);
    if (tot) SYZ_HIP(hipMemcpyAsync(dp, pcs, tot * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(doff, off, (n + 1) * 8, hipMemcpyHostToDevice, s));
    if (n) SYZ_HIP(hipMemcpyAsync(dg, group, n * 4, hipMemcpyHostToDevice, s));
    if (dl && n) SYZ_HIP(hipMemcpyAsync(dl, prog_len, n * 2, hipMemcpyHostToDevice, s));
    const uint64_t na = corpus_new_inputs(H, dp, doff, dg, dl, n, dn, s);
    if (is_new && n) SYZ_HIP(hipMemcpyAsync(is_new, dn, n, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (accepted) *accepted = na;
  })
}

int syzgpu_corpus_cover_union(syzgpu_corpus* cp, uint32_t* out, uint64_t* out_off, size_t cap, uint64_t* total) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    if (!total || !out_off) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    uint32_t* d = C_.scratch.get<uint32_t>("cc_xout", cap + 1);
    uint64_t* doff = C_.scratch.get<uint64_t>("cc_xoff", H.G + 1);
    const uint64_t nt = cc_export(H, d, doff, cap, s);
    *total = nt;
    if (nt > cap) fail(SYZGPU_ECAPACITY, "corpusCover larger than the output");
    if (nt && out) SYZ_HIP(hipMemcpyAsync(out, d, nt * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(out_off, doff, (H.G + 1) * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_corpus_keep_dev(syzgpu_corpus* cp, const int64_t* idx, size_t m, void* stream) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    keep_entries(H, idx, m, (hipStream_t)stream);
  })
}

int syzgpu_corpus_keep(syzgpu_corpus* cp, const int64_t* idx, size_t m) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    if (m && !idx) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    int64_t* d = C_.scratch.get<int64_t>("co_kidx", m + 1);
    if (m) SYZ_HIP(hipMemcpyAsync(d, idx, m * 8, hipMemcpyHostToDevice, s));
    keep_entries(H, d, m, s);
  })
}

int syzgpu_corpus_minimize_keep_dev(syzgpu_corpus* cp, int32_t C, uint8_t* selected, int64_t* len_hist,
                                    int64_t* out_idx, uint64_t* group_out_off, void* stream, uint64_t* kept) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    const uint64_t m = minimize_keep(H, C, selected, len_hist, out_idx, group_out_off, (hipStream_t)stream);
    if (kept) *kept = m;
  })
}

int syzgpu_corpus_reindex(syzgpu_corpus* cp, void* stream) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    corpus_index(H, (hipStream_t)stream);
  })
}

int syzgpu_corpus_minimize_dev(syzgpu_corpus* cp, int32_t C, uint8_t* selected, int64_t* len_hist, void* stream) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    if (len_hist && C <= 0) fail(SYZGPU_EINVAL, "len_hist needs C > 0");
    if (len_hist && (int64_t)H.max_prog_len > (int64_t)C)
      fail(SYZGPU_EINVAL, "len(p.Calls) > C (prog/prio.go:148 would panic)");
    handle_begin(H, (hipStream_t)stream);
    handle_end(H, C, selected, len_hist, nullptr, nullptr, (hipStream_t)stream);
  })
}

int syzgpu_corpus_minimize_ordered_dev(syzgpu_corpus* cp, int32_t C, uint8_t* selected, int64_t* len_hist,
                                       int64_t* out_idx, uint64_t* group_out_off, void* stream) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    if (len_hist && (int64_t)H.max_prog_len > (int64_t)C)
      fail(SYZGPU_EINVAL, "len(p.Calls) > C (prog/prio.go:148 would panic)");
    handle_begin(H, (hipStream_t)stream);
    handle_end(H, C, selected, len_hist, out_idx, group_out_off, (hipStream_t)stream);
  })
}

int syzgpu_corpus_minimize(syzgpu_corpus* cp, int64_t* out_idx, uint64_t* group_out_off) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    if (!group_out_off) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    int64_t* dout = C_.scratch.get<int64_t>("mz_out", H.n + 1);
    uint64_t* dgoff = C_.scratch.get<uint64_t>("mz_goff", H.G + 1);
    handle_begin(H, s);
    handle_end(H, 0, nullptr, nullptr, dout, dgoff, s);
    SYZ_HIP(hipMemcpyAsync(group_out_off, dgoff, (H.G + 1) * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (group_out_off[H.G] && out_idx)
      SYZ_HIP(hipMemcpyAsync(out_idx, dout, group_out_off[H.G] * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_corpus_info(const syzgpu_corpus* cp, uint64_t* info, size_t cap) {
  SYZ_API_BODY({
    if (!info) fail(SYZGPU_EINVAL, "null pointer");
    CorpusHandle& H = H_of(const_cast<syzgpu_corpus*>(cp));
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    if (H.index && (H.index->keep_pending || H.index->app_pending)) corpus_index(H, C_.stream);  // recorded changes applied
    uint64_t v[12] = {H.n, H.G, H.L, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (H.index) {
      const Corpus& K = *H.index;
      const uint64_t w[12] = {K.n,          K.G,           K.total_pcs, K.total_ids, K.hwork.size(), K.ngtabs,
                              K.total_vecs, K.big_entries, K.big_pcs,   K.big_vecs,  K.big_vecs_all, 1};
      std::copy(w, w + 12, v);
    }
    for (size_t i = 0; i < cap && i < 12; i++) info[i] = v[i];
  })
}

int syzgpu_corpus_set_parts(syzgpu_corpus* cp, const uint16_t* part, const uint16_t* nparts,
                            const uint8_t* count_hist) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    const uint32_t G = H.G;
    bool split = false;
    for (uint32_t g = 0; g < G && nparts; g++) {
      if (nparts[g] > 1) {
        split = true;
        if (!part || part[g] >= nparts[g]) fail(SYZGPU_EINVAL, "part[g] must be < nparts[g]");
      }
    }
    H.parts_set = split || count_hist;
    H.part.assign(G, 0);
    H.nparts.assign(G, 1);
    if (nparts) {
      H.nparts.assign(nparts, nparts + G);
      if (part) H.part.assign(part, part + G);
    }
    H.has_count_hist = count_hist != nullptr;
    H.count_hist.assign(count_hist ? count_hist : nullptr, count_hist ? count_hist + G : nullptr);
    corpus_set_parts(corpus_index(H, C_.stream), H.part.data(), H.nparts.data(), count_hist, C_.stream);
  })
}

int syzgpu_corpus_minimize_begin_dev(syzgpu_corpus* cp, void* stream) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    handle_begin(H, (hipStream_t)stream);
  })
}

int syzgpu_corpus_export_sel_dev(syzgpu_corpus* cp, const uint32_t* groups, const uint64_t* offsets,
                                 uint32_t ngroups, uint8_t* buf, void* stream) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    handle_xchg(H, groups, offsets, ngroups, buf, 0, (hipStream_t)stream);
  })
}

int syzgpu_corpus_import_sel_dev(syzgpu_corpus* cp, const uint32_t* groups, const uint64_t* offsets,
                                 uint32_t ngroups, const uint8_t* buf, void* stream) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    handle_xchg(H, groups, offsets, ngroups, const_cast<uint8_t*>(buf), 1, (hipStream_t)stream);
  })
}

int syzgpu_corpus_minimize_end_dev(syzgpu_corpus* cp, int32_t C, uint8_t* selected, int64_t* len_hist,
                                   void* stream) {
  SYZ_API_BODY({
    CorpusHandle& H = H_of(cp);
    std::lock_guard<std::recursive_mutex> hl_(H.mu);
    if (len_hist && (int64_t)H.max_prog_len > (int64_t)C)
      fail(SYZGPU_EINVAL, "len(p.Calls) > C (prog/prio.go:148 would panic)");
    handle_end(H, C, selected, len_hist, nullptr, nullptr, (hipStream_t)stream);
  })
}

}  // extern "C"

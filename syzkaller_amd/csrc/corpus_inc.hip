// The corpus index kept current across NewInput appends and mgr.corpus = newCorpus keeps
// (syz-manager/manager.go:609-616 and :523-529), so minimizeCorpus after them stays on the index's
// id-stream walk (k_vec_min) instead of falling back to the raw pipeline.
//
//   append  the new covers' PCs looked up in the per-call dictionary (sorted (call << 32 | PC) keys,
//           binary search); unseen pairs get the next dense ids of their call; each new cover's ids
//           sorted and cut at the id windows. Their vectors join the stream's TAIL (everything
//           appended since the last relayout, itself panel-major: each append rebuilds only the
//           tail), and each panel's tail range is walked by the workgroup of the panel's last work
//           item after its body range (VecWork tbeg/tend): no extra items, no extra merges. A vector
//           names its ENTRY (appends never renumber entries), the unseen keys join a small sorted
//           DELTA dictionary (merged into the main one only when it grows past a fraction of it), and
//           the group partition and work list are redone lazily by the next user (a minimize): an
//           append costs O(its covers + delta + tail), not O(index).
//   keep    recorded, and applied by the next user of the index (an append, a minimize): one
//           relayout of the whole stream, panel-major again with the tails folded in, dropping the
//           vectors of dropped entries (flags, a scan, one copy) and renumbering the entries; the
//           work items are cut afresh as a build cuts them.
//
// The dictionary's id -> PC table (dict/gdict) is not extended: the cover analytics rebuild the
// index from the covers when it is behind (corpus_index_full). Any failure drops the index (the
// corpus then minimizes on the raw pipeline until the next build), never the covers.
#include <algorithm>
#include <map>

#include "corpus.hpp"

namespace syz {

__global__ void k_splits(const uint32_t* ids, const uint64_t* off, const uint32_t* group, size_t n,
                         const uint32_t* nwin, const uint64_t* sbase, uint32_t* splits);

namespace {

constexpr uint32_t NONE32 = 0xFFFFFFFFu;

template <class T>
void dev_grow_keep(DevArr<T>& a, size_t used, size_t need, hipStream_t s) {
  if (need <= a.n && a.p) return;
  const size_t want = need + need / 2 + 1024;
  T* p = nullptr;
  SYZ_HIP(hipMalloc(&p, want * sizeof(T)));
  if (used && a.p) SYZ_HIP(hipMemcpyAsync(p, a.p, used * sizeof(T), hipMemcpyDeviceToDevice, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (a.p) (void)hipFree(a.p);
  a.p = p;
  a.n = want;
}

// sd_key[gdict[g] + id] = g << 32 | dict[gdict[g] + id], sd_id = id (then sorted by key)
__global__ void k_sd_init(const uint32_t* dict, const uint64_t* gdict, uint32_t G, uint64_t T, uint64_t* key,
                          uint32_t* id) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = (uint32_t)upper_bound_dev<uint64_t>(gdict, 0, G + 1, i) - 1;
    key[i] = ((uint64_t)g << 32) | dict[i];
    id[i] = (uint32_t)(i - gdict[g]);
  }
}

// one wave per new entry: each PC's id from the sorted dictionary, or a miss
__global__ __launch_bounds__(256) void k_ci_lookup(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                   size_t e0, size_t m, const uint64_t* sd_key,
                                                   const uint32_t* sd_id, uint64_t sd_n, const uint64_t* dl_key,
                                                   const uint32_t* dl_id, uint64_t dl_n, uint64_t pbase,
                                                   uint32_t* ids, uint32_t* miss) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < m; t += waves) {
    const size_t e = e0 + t;
    const uint64_t g = group[e];
    for (uint64_t p = off[e] + __lane_id(); p < off[e + 1]; p += 64) {
      const uint64_t key = (g << 32) | pcs[p];
      const uint64_t x = lower_bound_dev<uint64_t>(sd_key, 0, sd_n, key);
      bool hit = x < sd_n && sd_key[x] == key;
      uint32_t id = hit ? sd_id[x] : NONE32;
      if (!hit && dl_n) {  // the keys appended since the last merge
        const uint64_t y = lower_bound_dev<uint64_t>(dl_key, 0, dl_n, key);
        hit = y < dl_n && dl_key[y] == key;
        if (hit) id = dl_id[y];
      }
      ids[p - pbase] = id;
      miss[p - pbase] = hit ? 0u : 1u;
    }
  }
}

// the missed (call, PC) keys, compacted
__global__ void k_ci_misskeys(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t e0, size_t m,
                              uint64_t pbase, const uint32_t* miss, const uint64_t* mpos, uint64_t* mkey) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < m; t += waves) {
    const size_t e = e0 + t;
    const uint64_t g = group[e];
    for (uint64_t p = off[e] + __lane_id(); p < off[e + 1]; p += 64)
      if (miss[p - pbase]) mkey[mpos[p - pbase]] = (g << 32) | pcs[p];
  }
}

// first-of-run flags of the sorted missed keys
__global__ void k_ci_uflag(const uint64_t* k, uint64_t n, uint32_t* f) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    f[i] = (i == 0 || k[i] != k[i - 1]) ? 1u : 0u;
}

__global__ void k_ci_ucompact(const uint64_t* k, uint64_t n, const uint32_t* f, const uint64_t* pos, uint64_t* u) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (f[i]) u[pos[i]] = k[i];
}

// ids of the missed PCs: the next ids of their call, in PC order among the call's new keys
__global__ __launch_bounds__(256) void k_ci_missid(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                   size_t e0, size_t m, uint64_t pbase, const uint64_t* u,
                                                   uint64_t nu, const uint64_t* ubeg, const uint64_t* nids0,
                                                   uint32_t* ids) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < m; t += waves) {
    const size_t e = e0 + t;
    const uint64_t g = group[e];
    for (uint64_t p = off[e] + __lane_id(); p < off[e + 1]; p += 64)
      if (ids[p - pbase] == NONE32) {
        const uint64_t key = (g << 32) | pcs[p];
        const uint64_t j = lower_bound_dev<uint64_t>(u, 0, nu, key);
        ids[p - pbase] = (uint32_t)(nids0[g] + (j - ubeg[g]));
      }
  }
}

// merge of the sorted dictionary (a) and the sorted new keys (b, ids from ubeg / nids0): a key's
// place = its index + the other list's keys below it (the lists share no key)
__global__ void k_ci_merge(const uint64_t* a, const uint32_t* aid, uint64_t na, const uint64_t* b, uint64_t nb,
                           const uint64_t* ubeg, const uint64_t* nids0, uint64_t* out, uint32_t* oid) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb;
       i += (uint64_t)gridDim.x * blockDim.x) {
    if (i < na) {
      const uint64_t k = a[i];
      const uint64_t q = i + lower_bound_dev<uint64_t>(b, 0, nb, k);
      out[q] = k;
      oid[q] = aid[i];
    } else {
      const uint64_t j = i - na, k = b[j], g = k >> 32;
      const uint64_t q = j + lower_bound_dev<uint64_t>(a, 0, na, k);
      out[q] = k;
      oid[q] = (uint32_t)(nids0[g] + (j - ubeg[g]));
    }
  }
}

// merge of two sorted (key, id) lists that share no key
__global__ void k_ci_merge2(const uint64_t* a, const uint32_t* aid, uint64_t na, const uint64_t* b,
                            const uint32_t* bid, uint64_t nb, uint64_t* out, uint32_t* oid) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb;
       i += (uint64_t)gridDim.x * blockDim.x) {
    if (i < na) {
      const uint64_t q = i + lower_bound_dev<uint64_t>(b, 0, nb, a[i]);
      out[q] = a[i];
      oid[q] = aid[i];
    } else {
      const uint64_t j = i - na;
      const uint64_t q = j + lower_bound_dev<uint64_t>(a, 0, na, b[j]);
      out[q] = b[j];
      oid[q] = bid[j];
    }
  }
}

// ubeg[g] = first new key of call g
__global__ void k_ci_ubeg(const uint64_t* u, uint64_t nu, uint32_t G, uint64_t* ubeg) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g <= G; g += gridDim.x * blockDim.x)
    ubeg[g] = lower_bound_dev<uint64_t>(u, 0, nu, (uint64_t)g << 32);
}

__global__ void k_ci_reloff(const uint64_t* off, size_t e0, size_t m, uint64_t* rel) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i <= m; i += (size_t)gridDim.x * blockDim.x)
    rel[i] = off[e0 + i] - off[e0];
}

struct Slice {  // one new cover's ids in one window -> vectors [vout, vout + ceil(len / VEC))
  uint32_t e, w, s0, len;
  uint64_t vout;
};

// one wave per slice: window-relative u16 ids (padded with the last id) and the entry per vector
__global__ __launch_bounds__(256) void k_ci_vfill(const Slice* sl, size_t ns, const uint32_t* ids,
                                                  const uint64_t* rel, size_t e0, uint16_t* ids16, uint32_t* vmem) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < ns; t += waves) {
    const Slice x = sl[t];
    const uint32_t* src = ids + rel[x.e] + x.s0;
    const uint32_t padded = (x.len + VEC - 1) / VEC * VEC, wb = x.w << WIN_BITS;
    for (uint32_t k = __lane_id(); k < padded; k += 64) ids16[x.vout * VEC + k] = (uint16_t)(src[min(k, x.len - 1)] - wb);
    const uint32_t e = (uint32_t)(e0 + x.e);
    for (uint32_t k = __lane_id(); k < padded / VEC; k += 64) vmem[x.vout + k] = e;
  }
}

// keep: new id of every old entry (NONE: dropped)
__global__ void k_ci_inv(const int64_t* idx, size_t m, uint32_t* inv) {
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < m; t += (size_t)gridDim.x * blockDim.x)
    inv[idx[t]] = (uint32_t)t;
}

// an entry kept twice has one id in inv: the index cannot follow such a keep (the covers can)
__global__ void k_ci_invcheck(const int64_t* idx, size_t m, const uint32_t* inv, uint32_t* bad) {
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < m; t += (size_t)gridDim.x * blockDim.x)
    if (inv[idx[t]] != (uint32_t)t) atomicOr(bad, 1u);
}

__global__ void k_ci_vflag(const uint32_t* vmem, uint64_t nv, const uint32_t* inv, uint32_t* f) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * blockDim.x)
    f[v] = inv[vmem[v]] != NONE32 ? 1u : 0u;
}

__global__ void k_ci_gather(const uint64_t* pos, const uint64_t* at, size_t n, uint64_t* out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = pos[at[i]];
}

// K's per-entry copies of the handle's (current) covers metadata
void take_entries(Corpus& K, const CorpusHandle& H, hipStream_t s) {
  K.n = H.n;
  K.total_pcs = H.L;
  K.off.ensure(H.n + 1);
  K.group.ensure(H.n + 1);
  K.prog_len.ensure(H.n + 1);
  SYZ_HIP(hipMemcpyAsync(K.off.p, H.off.p, (H.n + 1) * 8, hipMemcpyDeviceToDevice, s));
  if (H.n) {
    SYZ_HIP(hipMemcpyAsync(K.group.p, H.group.p, H.n * 4, hipMemcpyDeviceToDevice, s));
    SYZ_HIP(hipMemcpyAsync(K.prog_len.p, H.prog_len.p, H.n * 2, hipMemcpyDeviceToDevice, s));
  }
  K.max_prog_len = H.max_prog_len;
  K.incremental = true;
  corpus_stats_free(K.stats);
  K.stats = nullptr;
}

// the sorted (call, PC) -> id lookup, built once from the dictionary
void ensure_sorted_dict(Corpus& K, hipStream_t s) {
  if (K.sd_built) return;
  Scratch& sc = ctx().scratch;
  const uint64_t T = K.total_ids;
  K.sd_key.alloc(T + 1);
  K.sd_id.alloc(T + 1);
  uint64_t* kt = sc.get<uint64_t>("ci_ktmp", T + 1);
  uint32_t* vt = sc.get<uint32_t>("ci_vtmp", T + 1);
  if (T) {
    k_sd_init<<<grid_for(T, 256, 8192), 256, 0, s>>>(K.dict.p, K.gdict.p, K.G, T, K.sd_key.p, K.sd_id.p);
    SYZ_LAUNCHED();
    uint64_t* k = K.sd_key.p;
    uint32_t* v = K.sd_id.p;
    radix_sort_pairs(k, v, kt, vt, T, 44, s);
    if (k != K.sd_key.p) {  // the sort's result landed in the scratch pair
      SYZ_HIP(hipMemcpyAsync(K.sd_key.p, k, T * 8, hipMemcpyDeviceToDevice, s));
      SYZ_HIP(hipMemcpyAsync(K.sd_id.p, v, T * 4, hipMemcpyDeviceToDevice, s));
    }
  }
  K.sd_n = T;
  K.sd_built = true;
}


// one wave per copy: ids16 / vmem vectors [src, src + len) -> [dst, dst + len) of the target
struct VCopy {
  uint64_t src, dst, len;
};
__global__ __launch_bounds__(256) void k_ci_copy(const VCopy* cp, size_t nc, const uint4* ids16, const uint32_t* vmem,
                                                 uint4* ids16b, uint32_t* vmemb) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < nc; t += waves) {
    const VCopy c = cp[t];
    for (uint64_t k = __lane_id(); k < c.len; k += 64) {
      ids16b[c.dst + k] = ids16[c.src + k];
      vmemb[c.dst + k] = vmem[c.src + k];
    }
  }
}

// relayout: vector v of segment j (segments sorted by start) goes to segbase[j] + its rank among the
// segment's kept vectors; kept = its entry survives (inv), entry renumbered
__global__ void k_ci_relayout(const uint4* ids16, const uint32_t* vmem, uint64_t nv, const uint64_t* segstart,
                              uint32_t nseg, const uint64_t* segbase, const uint64_t* pos, const uint32_t* inv,
                              uint4* ids16b, uint32_t* vmemb) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t e = inv[vmem[v]];
    if (e == NONE32) continue;
    const uint32_t j = (uint32_t)upper_bound_dev<uint64_t>(segstart, 0, nseg, v) - 1;
    const uint64_t q = segbase[j] + (pos[v] - pos[segstart[j]]);
    ids16b[q] = ids16[v];
    vmemb[q] = e;
  }
}

// the work list the kernels run: the body's items, each panel's tail on its last body item (or on
// an item of its own when the panel has no body yet); table sizes from the calls' id counts
void compose_work(Corpus& K, hipStream_t s) {
  std::vector<VecWork> w = K.hmain;
  std::map<std::pair<uint32_t, uint32_t>, size_t> last;  // panel -> its last body item
  for (size_t i = 0; i < w.size(); i++) {
    w[i].tbeg = w[i].tend = 0;
    auto k = std::make_pair(w[i].g, w[i].win);
    auto it = last.find(k);
    if (it == last.end() || w[it->second].vbeg < w[i].vbeg) last[k] = i;
  }
  for (const auto& kv : K.ptail) {
    auto it = last.find(kv.first);
    if (it != last.end()) {
      w[it->second].tbeg = kv.second.first;
      w[it->second].tend = kv.second.second;
    } else {
      VecWork x{kv.first.first, 0, 0, 0, RANK_NONE, kv.first.second};
      x.tbeg = kv.second.first;
      x.tend = kv.second.second;
      w.push_back(x);
    }
  }
  for (VecWork& x : w) x.nids = (uint32_t)std::min<uint64_t>(WIN, K.hnids[x.g] - (uint64_t)x.win * WIN);
  K.big_vecs_all = 0;
  for (const VecWork& x : w)
    if (K.hstart[x.g + 1] - K.hstart[x.g] > GS_T_SEG) K.big_vecs_all += (x.vend - x.vbeg) + (x.tend - x.tbeg);
  K.hwork_all = w;
  K.hwork = w;
  corpus_upload_work(K, s);
}

// the pending keep (K.keep_idx of K.keep_n0 old entries), applied: partition, relayout, fresh items
void apply_keep(Corpus& K, const CorpusHandle& H, hipStream_t s) {
  Scratch& sc = ctx().scratch;
  PhaseTimer pt("index_keep");
  const size_t m = K.keep_m, n0 = K.keep_n0;
  const int64_t* idx = K.keep_idx.p;
  if (n0 != K.n || m != H.n) fail(SYZGPU_EINTERNAL, "corpus index out of step with the covers");
  uint32_t* inv = sc.get<uint32_t>("ci_inv", n0 + 1);
  uint32_t* bad = sc.get<uint32_t>("ci_bad", 1);
  SYZ_HIP(hipMemsetAsync(inv, 0xFF, (n0 + 1) * 4, s));
  SYZ_HIP(hipMemsetAsync(bad, 0, 4, s));
  if (m) {
    k_ci_inv<<<grid_for(m, 256, 4096), 256, 0, s>>>(idx, m, inv);
    SYZ_LAUNCHED();
    k_ci_invcheck<<<grid_for(m, 256, 4096), 256, 0, s>>>(idx, m, inv, bad);
    SYZ_LAUNCHED();
  }
  // segments of the stream: body items and tails, each with its panel
  struct Seg {
    uint64_t a, b;
    uint32_t g, w;
  };
  std::vector<Seg> seg;
  for (const VecWork& x : K.hmain)
    if (x.vend > x.vbeg) seg.push_back(Seg{x.vbeg, x.vend, x.g, x.win});
  for (const auto& kv : K.ptail)
    if (kv.second.second > kv.second.first) seg.push_back(Seg{kv.second.first, kv.second.second, kv.first.first, kv.first.second});
  std::sort(seg.begin(), seg.end(), [](const Seg& x, const Seg& y) { return x.a < y.a; });
  const uint64_t nv = K.total_vecs;
  uint32_t* f = sc.get<uint32_t>("ci_vflag", nv + 1);
  uint64_t* pos = sc.get<uint64_t>("ci_vpos", nv + 1);
  if (nv) {
    k_ci_vflag<<<grid_for(nv, 256, 16384), 256, 0, s>>>(K.vmem.p, nv, inv, f);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(f, pos, nv, s);
  std::vector<uint64_t> hat;
  for (const Seg& x : seg) {
    hat.push_back(x.a);
    hat.push_back(x.b);
  }
  hat.push_back(nv);
  uint64_t* dat = sc.get<uint64_t>("ci_at", hat.size());
  uint64_t* dnew = sc.get<uint64_t>("ci_atnew", hat.size());
  std::vector<uint64_t> hnew(hat.size());
  uint32_t hbad = 0;
  SYZ_HIP(hipMemcpyAsync(dat, hat.data(), hat.size() * 8, hipMemcpyHostToDevice, s));
  k_ci_gather<<<grid_for(hat.size(), 256, 1024), 256, 0, s>>>(pos, dat, hat.size(), dnew);
  SYZ_LAUNCHED();
  SYZ_HIP(hipMemcpyAsync(hnew.data(), dnew, hat.size() * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (hbad) fail(SYZGPU_EINVAL, "corpus index: an entry kept twice");
  pt.mark("flags", s);
  // panels in (call, window) order; inside a panel its segments in stream order
  std::vector<size_t> ord(seg.size());
  for (size_t j = 0; j < seg.size(); j++) ord[j] = j;
  std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) {
    return seg[x].g != seg[y].g ? seg[x].g < seg[y].g : seg[x].w < seg[y].w;
  });
  std::vector<uint64_t> segstart(seg.size()), segbase(seg.size());
  std::vector<VecWork> items;
  uint64_t run = 0;
  for (size_t k = 0; k < ord.size();) {
    const uint32_t g = seg[ord[k]].g, w = seg[ord[k]].w;
    const uint64_t pb = run;
    for (; k < ord.size() && seg[ord[k]].g == g && seg[ord[k]].w == w; k++) {
      const size_t j = ord[k];
      segbase[j] = run;
      run += hnew[2 * j + 1] - hnew[2 * j];
    }
    if (run == pb) continue;
    const uint64_t nch = (run - pb + K.chunk_vecs - 1) / K.chunk_vecs;
    const uint32_t gt = nch > 1 ? (uint32_t)0 : RANK_NONE;  // numbered below
    const uint64_t per = (run - pb + nch - 1) / nch;
    for (uint64_t v = pb; v < run; v += per) items.push_back(VecWork{g, 0, v, std::min(run, v + per), gt, w});
  }
  for (size_t j = 0; j < seg.size(); j++) segstart[j] = seg[j].a;
  // shared tables: one per panel cut into several items
  K.ngtabs = 0;
  for (size_t i = 0; i < items.size(); i++) {
    if (items[i].gtab == RANK_NONE) continue;
    if (i > 0 && items[i - 1].gtab != RANK_NONE && items[i - 1].g == items[i].g && items[i - 1].win == items[i].win)
      items[i].gtab = items[i - 1].gtab;
    else
      items[i].gtab = K.ngtabs++;
  }
  take_entries(K, H, s);
  std::vector<uint64_t> hpcs;
  corpus_partition(K, hpcs, s);
  pt.mark("partition", s);
  K.ids16b.ensure((run + 1) * VEC);
  K.vmemb.ensure(run + 1);
  if (nv && !seg.empty()) {
    uint64_t* dss = sc.get<uint64_t>("ci_segstart", seg.size());
    uint64_t* dsb = sc.get<uint64_t>("ci_segbase", seg.size());
    SYZ_HIP(hipMemcpyAsync(dss, segstart.data(), seg.size() * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(dsb, segbase.data(), seg.size() * 8, hipMemcpyHostToDevice, s));
    k_ci_relayout<<<grid_for(nv, 256, 16384), 256, 0, s>>>(reinterpret_cast<const uint4*>(K.ids16.p), K.vmem.p, nv,
                                                          dss, (uint32_t)seg.size(), dsb, pos, inv,
                                                          reinterpret_cast<uint4*>(K.ids16b.p), K.vmemb.p);
    SYZ_LAUNCHED();
  }
  std::swap(K.ids16.p, K.ids16b.p);
  std::swap(K.ids16.n, K.ids16b.n);
  std::swap(K.vmem.p, K.vmemb.p);
  std::swap(K.vmem.n, K.vmemb.n);
  K.total_vecs = run;
  K.tail0 = run;
  K.ptail.clear();
  K.hmain = items;
  K.gtabs.ensure((size_t)K.ngtabs * WIN + 1);
  K.gtchunks.ensure(K.ngtabs + 1);
  K.gtdone.ensure(K.ngtabs + 1);
  compose_work(K, s);
  K.keep_pending = false;
  K.part_stale = false;
  pt.mark("relayout_work", s);
}

// the keys of the delta dictionary folded into the main one (when the delta has grown)
void merge_delta(Corpus& K, hipStream_t s) {
  if (!K.dl_n) return;
  Scratch& sc = ctx().scratch;
  const uint64_t nt = K.sd_n + K.dl_n;
  uint64_t* k2 = sc.get<uint64_t>("ci_sdk2", nt + 1);
  uint32_t* i2 = sc.get<uint32_t>("ci_sdi2", nt + 1);
  k_ci_merge2<<<grid_for(nt, 256, 16384), 256, 0, s>>>(K.sd_key.p, K.sd_id.p, K.sd_n, K.dl_key.p, K.dl_id.p, K.dl_n,
                                                        k2, i2);
  SYZ_LAUNCHED();
  dev_grow_keep(K.sd_key, 0, nt + 1, s);
  dev_grow_keep(K.sd_id, 0, nt + 1, s);
  SYZ_HIP(hipMemcpyAsync(K.sd_key.p, k2, nt * 8, hipMemcpyDeviceToDevice, s));
  SYZ_HIP(hipMemcpyAsync(K.sd_id.p, i2, nt * 4, hipMemcpyDeviceToDevice, s));
  K.sd_n = nt;
  K.dl_n = 0;
}

}  // namespace

void corpus_index_sync(Corpus& K, const CorpusHandle& H, hipStream_t s) {
  if (K.keep_pending) apply_keep(K, H, s);  // (partitions and composes the work itself)
  if (K.app_pending) {  // the appends since the last user, as one batch
    K.app_pending = false;
    corpus_index_append(K, H, K.app_n0, K.app_L0, s);
  }
  if (K.part_stale) {  // appends since the last partition: the group partition and the work list
    PhaseTimer pt("index_sync");
    std::vector<uint64_t> hpcs;
    corpus_partition(K, hpcs, s);
    compose_work(K, s);
    K.part_stale = false;
    pt.mark("partition_work", s);
  }
}

// H has just taken m = H.n - n0 new entries (their PCs from L0). Brings K up to H's covers.
void corpus_index_append(Corpus& K, const CorpusHandle& H, size_t n0, uint64_t L0, hipStream_t s) {
  Scratch& sc = ctx().scratch;
  const uint32_t G = K.G;
  if (K.keep_pending) fail(SYZGPU_EINTERNAL, "corpus index: keep pending at append");
  const size_t m = H.n - n0;
  const uint64_t Lm = H.L - L0;
  if (n0 != K.n) fail(SYZGPU_EINTERNAL, "corpus index out of step with the covers");
  PhaseTimer pt("index_append");
  if (!K.incremental) {  // the first change: the build's items are the body
    K.hmain = K.hwork_all;
    K.ptail.clear();
    K.tail0 = K.total_vecs;
  }
  ensure_sorted_dict(K, s);
  const uint64_t* off = H.off.p;
  // 1. ids of the new PCs: dictionary hits, then the missed keys -> next ids of their call
  uint32_t* ids = sc.get<uint32_t>("ci_ids", Lm + 1);
  uint32_t* miss = sc.get<uint32_t>("ci_miss", Lm + 1);
  uint64_t* mpos = sc.get<uint64_t>("ci_mpos", Lm + 1);
  const unsigned wgrid = (unsigned)std::min<size_t>((m * 64 + 255) / 256 + 1, 65536);
  if (m) {
    k_ci_lookup<<<wgrid, 256, 0, s>>>(H.pcs.p, off, H.group.p, n0, m, K.sd_key.p, K.sd_id.p, K.sd_n, K.dl_key.p,
                                      K.dl_id.p, K.dl_n, L0, ids, miss);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(miss, mpos, Lm, s);
  uint64_t* rel = sc.get<uint64_t>("ci_rel", m + 1);
  k_ci_reloff<<<grid_for(m + 1, 256, 1024), 256, 0, s>>>(off, n0, m, rel);
  SYZ_LAUNCHED();
  uint64_t* hb = ctx().pinned.get<uint64_t>(2 * m + 8);  // [nmiss, rel[0..m], groups (u32)]
  SYZ_HIP(hipMemcpyAsync(hb, mpos + Lm, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hb + 1, rel, (m + 1) * 8, hipMemcpyDeviceToHost, s));
  if (m) SYZ_HIP(hipMemcpyAsync(hb + m + 2, H.group.p + n0, m * 4, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint64_t nmiss = hb[0];
  const std::vector<uint64_t> hrel(hb + 1, hb + m + 2);
  const uint32_t* hg32 = reinterpret_cast<const uint32_t*>(hb + m + 2);
  const std::vector<uint32_t> hgrp(hg32, hg32 + m);
  std::vector<uint64_t> nids0 = K.hnids;
  uint64_t* d_nids0 = sc.get<uint64_t>("ci_nids0", G + 1);
  uint64_t* ubeg = sc.get<uint64_t>("ci_ubeg", G + 1);
  if (nmiss) {
    SYZ_HIP(hipMemcpyAsync(d_nids0, nids0.data(), G * 8, hipMemcpyHostToDevice, s));
    uint64_t* mk = sc.get<uint64_t>("ci_mkey", nmiss + 1);
    uint32_t* mv = sc.get<uint32_t>("ci_mval", nmiss + 1);
    uint64_t* mkt = sc.get<uint64_t>("ci_mkt", nmiss + 1);
    uint32_t* mvt = sc.get<uint32_t>("ci_mvt", nmiss + 1);
    k_ci_misskeys<<<wgrid, 256, 0, s>>>(H.pcs.p, off, H.group.p, n0, m, L0, miss, mpos, mk);
    SYZ_LAUNCHED();
    SYZ_HIP(hipMemsetAsync(mv, 0, nmiss * 4, s));
    radix_sort_pairs(mk, mv, mkt, mvt, nmiss, 44, s);
    uint32_t* uf = sc.get<uint32_t>("ci_uflag", nmiss + 1);
    uint64_t* upos = sc.get<uint64_t>("ci_upos", nmiss + 1);
    k_ci_uflag<<<grid_for(nmiss, 256, 4096), 256, 0, s>>>(mk, nmiss, uf);
    SYZ_LAUNCHED();
    exclusive_scan_u32(uf, upos, nmiss, s);
    uint64_t* u = sc.get<uint64_t>("ci_u", nmiss + 1);
    k_ci_ucompact<<<grid_for(nmiss, 256, 4096), 256, 0, s>>>(mk, nmiss, uf, upos, u);
    SYZ_LAUNCHED();
    uint64_t nu = 0;
    SYZ_HIP(hipMemcpyAsync(&nu, upos + nmiss, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    k_ci_ubeg<<<grid_for(G + 1, 256, 64), 256, 0, s>>>(u, nu, G, ubeg);
    SYZ_LAUNCHED();
    k_ci_missid<<<wgrid, 256, 0, s>>>(H.pcs.p, off, H.group.p, n0, m, L0, u, nu, ubeg, d_nids0, ids);
    SYZ_LAUNCHED();
    // the DELTA dictionary takes the new keys (merged, still sorted: O(delta + new), not O(dictionary));
    // it is folded into the main one once it outgrows a fraction of it
    const uint64_t nt = K.dl_n + nu;
    uint64_t* k2 = sc.get<uint64_t>("ci_dlk2", nt + 1);
    uint32_t* i2 = sc.get<uint32_t>("ci_dli2", nt + 1);
    k_ci_merge<<<grid_for(nt, 256, 16384), 256, 0, s>>>(K.dl_key.p, K.dl_id.p, K.dl_n, u, nu, ubeg, d_nids0, k2, i2);
    SYZ_LAUNCHED();
    dev_grow_keep(K.dl_key, 0, nt + 1, s);
    dev_grow_keep(K.dl_id, 0, nt + 1, s);
    SYZ_HIP(hipMemcpyAsync(K.dl_key.p, k2, nt * 8, hipMemcpyDeviceToDevice, s));
    SYZ_HIP(hipMemcpyAsync(K.dl_id.p, i2, nt * 4, hipMemcpyDeviceToDevice, s));
    K.dl_n = nt;
    if (K.dl_n > std::max<uint64_t>(1ull << 20, K.sd_n / 8)) merge_delta(K, s);
    // the new ids per call: ubeg's differences (G + 1 words back, not the nu keys)
    uint64_t* hub = ctx().pinned.get<uint64_t>(G + 1);
    SYZ_HIP(hipMemcpyAsync(hub, ubeg, (G + 1) * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    for (uint32_t g = 0; g < G; g++) K.hnids[g] += hub[g + 1] - hub[g];
    K.total_ids += nu;
  }
  pt.mark("ids", s);
  // 2. each new cover's ids sorted (a cover's ids are distinct iff its PCs are), cut at the windows
  std::vector<uint32_t> nwin(G);
  for (uint32_t g = 0; g < G; g++) nwin[g] = (uint32_t)std::max<uint64_t>(1, (K.hnids[g] + WIN - 1) / WIN);
  std::vector<uint64_t> hsb(m + 1, 0);
  for (size_t e = 0; e < m; e++) hsb[e + 1] = hsb[e] + nwin[hgrp[e]] + 1;
  uint64_t* clen = sc.get<uint64_t>("ci_clen", m + 1);
  uint64_t* sbase = sc.get<uint64_t>("ci_sbase", m + 1);
  uint32_t* splits = sc.get<uint32_t>("ci_splits", hsb[m] + 1);
  SYZ_HIP(hipMemcpyAsync(K.nwin.p, nwin.data(), G * 4, hipMemcpyHostToDevice, s));
  SYZ_HIP(hipMemcpyAsync(sbase, hsb.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
  std::vector<uint64_t> hclen(m);
  std::vector<uint32_t> hsp(hsb[m] + 1);
  if (m) {
    canonicalize_batch_dev2(ids, rel, m, clen, s);
    k_splits<<<grid_for(m, 256, 4096), 256, 0, s>>>(ids, rel, H.group.p + n0, m, K.nwin.p, sbase, splits);
    SYZ_LAUNCHED();
    SYZ_HIP(hipMemcpyAsync(hclen.data(), clen, m * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(hsp.data(), splits, hsb[m] * 4, hipMemcpyDeviceToHost, s));
  }
  // 3. the entries taken; the group partition (and the work list) are redone by the next user: the
  // old vectors keep their entry ids
  take_entries(K, H, s);
  SYZ_HIP(hipStreamSynchronize(s));  // hclen / hsp are in
  for (size_t e = 0; e < m; e++)
    if (hclen[e] != hrel[e + 1] - hrel[e]) fail(SYZGPU_EINVAL, "corpus index needs canonical covers");
  pt.mark("canon_splits", s);
  const uint64_t nv0 = K.total_vecs;
  // 4. the tail rebuilt panel-major: per panel its old tail range, then its new slices
  std::vector<Slice> hsl;
  for (size_t e = 0; e < m; e++) {
    const uint32_t g = hgrp[e];
    const uint32_t* sp = hsp.data() + hsb[e];
    for (uint32_t w = 0; w < nwin[g]; w++)
      if (sp[w + 1] > sp[w]) hsl.push_back(Slice{(uint32_t)e, w, sp[w], sp[w + 1] - sp[w], 0});
  }
  std::stable_sort(hsl.begin(), hsl.end(), [&](const Slice& a, const Slice& b) {
    const uint32_t ga = hgrp[a.e], gb = hgrp[b.e];
    return ga != gb ? ga < gb : a.w < b.w;
  });
  std::map<std::pair<uint32_t, uint32_t>, std::pair<uint64_t, uint64_t>> nt;  // panel -> new tail range
  std::vector<VCopy> cps;
  uint64_t q = K.tail0;
  size_t si = 0;
  auto take_slices = [&](uint32_t g, uint32_t w) {
    for (; si < hsl.size() && hgrp[hsl[si].e] == g && hsl[si].w == w; si++) {
      hsl[si].vout = q;
      q += (hsl[si].len + VEC - 1) / VEC;
    }
  };
  auto it = K.ptail.begin();
  while (it != K.ptail.end() || si < hsl.size()) {
    std::pair<uint32_t, uint32_t> pk;
    if (it != K.ptail.end() &&
        (si >= hsl.size() || it->first <= std::make_pair(hgrp[hsl[si].e], hsl[si].w)))
      pk = it->first;
    else
      pk = {hgrp[hsl[si].e], hsl[si].w};
    const uint64_t a = q;
    if (it != K.ptail.end() && it->first == pk) {
      const uint64_t len = it->second.second - it->second.first;
      if (len) cps.push_back(VCopy{it->second.first, q, len});
      q += len;
      ++it;
    }
    if (si < hsl.size() && hgrp[hsl[si].e] == pk.first && hsl[si].w == pk.second) take_slices(pk.first, pk.second);
    nt[pk] = {a, q};
  }
  const uint64_t nv = q;
  dev_grow_keep(K.ids16, nv0 * VEC, nv * VEC + VEC, s);
  dev_grow_keep(K.vmem, nv0, nv + 1, s);
  const uint64_t ntail = nv - K.tail0;
  if (!cps.empty()) {  // the old tail moves: through a scratch copy of itself
    const uint64_t ot = nv0 - K.tail0;
    uint16_t* t16 = sc.get<uint16_t>("ci_t16", (ot + 1) * VEC);
    uint32_t* tvm = sc.get<uint32_t>("ci_tvm", ot + 1);
    SYZ_HIP(hipMemcpyAsync(t16, K.ids16.p + K.tail0 * VEC, ot * VEC * 2, hipMemcpyDeviceToDevice, s));
    SYZ_HIP(hipMemcpyAsync(tvm, K.vmem.p + K.tail0, ot * 4, hipMemcpyDeviceToDevice, s));
    for (VCopy& c : cps) c.src -= K.tail0;
    VCopy* dcp = sc.get<VCopy>("ci_copies", cps.size());
    SYZ_HIP(hipMemcpyAsync(dcp, cps.data(), cps.size() * sizeof(VCopy), hipMemcpyHostToDevice, s));
    k_ci_copy<<<(unsigned)std::min<size_t>((cps.size() * 64 + 255) / 256, 65536), 256, 0, s>>>(
        dcp, cps.size(), reinterpret_cast<const uint4*>(t16), tvm, reinterpret_cast<uint4*>(K.ids16.p), K.vmem.p);
    SYZ_LAUNCHED();
  }
  if (!hsl.empty()) {
    Slice* dsl = sc.get<Slice>("ci_slices", hsl.size());
    SYZ_HIP(hipMemcpyAsync(dsl, hsl.data(), hsl.size() * sizeof(Slice), hipMemcpyHostToDevice, s));
    k_ci_vfill<<<(unsigned)std::min<size_t>((hsl.size() * 64 + 255) / 256, 65536), 256, 0, s>>>(
        dsl, hsl.size(), ids, rel, n0, K.ids16.p, K.vmem.p);
    SYZ_LAUNCHED();
  }
  (void)ntail;
  K.total_vecs = nv;
  K.ptail = nt;
  K.part_stale = true;  // 5. the work list (body items + each panel's tail) with the next partition
  pt.mark("vectors", s);
}

// H has just taken the entries from n0 (PCs from L0): recorded, indexed by the index's next user
// (corpus_index_sync) together with any later appends, so a NewInput costs the covers' copy only
void corpus_index_note_append(Corpus& K, size_t n0, uint64_t L0) {
  if (K.app_pending) return;  // the pending range already starts earlier
  K.app_pending = true;
  K.app_n0 = n0;
  K.app_L0 = L0;
}

// H has just become the entries idx[0..m) (device, old ids) of a corpus of n0 entries: recorded, and
// applied by the index's next user (corpus_index_sync)
void corpus_index_keep(Corpus& K, const CorpusHandle& H, const int64_t* idx, size_t m, size_t n0, hipStream_t s) {
  if (K.keep_pending) apply_keep(K, H, s);  // (not reached: the corpus keeps the index in step)
  if (n0 != K.n) fail(SYZGPU_EINTERNAL, "corpus index out of step with the covers");
  if (!K.incremental) {
    K.hmain = K.hwork_all;
    K.ptail.clear();
    K.tail0 = K.total_vecs;
  }
  K.keep_idx.ensure(m + 1);
  if (m) SYZ_HIP(hipMemcpyAsync(K.keep_idx.p, idx, m * 8, hipMemcpyDeviceToDevice, s));
  K.keep_m = m;
  K.keep_n0 = n0;
  K.keep_pending = true;
  K.incremental = true;
  (void)H;
}

}  // namespace syz

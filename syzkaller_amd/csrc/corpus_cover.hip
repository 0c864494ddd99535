// corpusCover on the resident store: syz-manager's per-call union of every accepted cover
// (manager.go:65, :121) and NewInput's gate on it (manager.go:609-616):
//
//     if len(cover.Difference(a.Cover, mgr.corpusCover[call])) == 0 { return }
//     mgr.corpusCover[call] = cover.Union(mgr.corpusCover[call], a.Cover)
//     mgr.corpus = append(mgr.corpus, a.RpcInput)
//
// The set is the store's: sorted (call << 32 | PC) keys, a main array plus a small sorted DELTA of the
// keys added since the last fold (the index dictionary's scheme, corpus_inc.hip), so an update costs
// O(batch + delta), not O(set). It holds every cover the store has held (the manager's corpus only
// grows through NewInput), built from the store's covers on first use — the first gate, or a keep that
// could drop a call's PCs (minimizeCorpus's own keep cannot: Minimize keeps a first holder of every PC)
// — and kept current by every append. PC 0xFFFFFFFF (cover.go's sentinel) is never in it: foreach
// drops it from every Difference and Union.
//
// The gate over a batch without the sequential loop: a key x missing from corpusCover is brought in by
// the FIRST input of the batch holding it (at that input x is still missing, so the input is accepted
// and unions x in; every later holder sees x covered). So input k is accepted iff it is the first
// holder of some missing key: one binary search per PC, one sort of the missing (key, input) pairs,
// first-of-run flags (the first-occurrence form of the fuzzer's maxCover update, without flakes).
#include <algorithm>

#include "corpus.hpp"
#include "pipeline.hpp"

namespace syz {

namespace {

constexpr uint32_t CC_SENT = 0xFFFFFFFFu;
constexpr int CC_SMALL = 4096;  // missing pairs sorted in one workgroup's LDS (composite keys)
constexpr int CC_SMALL_BLOCK = 1024;

__device__ __forceinline__ bool cc_has(const uint64_t* a, uint64_t n, uint64_t key) {
  const uint64_t x = lower_bound_dev<uint64_t>(a, 0, n, key);
  return x < n && a[x] == key;
}

// one wave per cover: miss[p] = its (call, PC) key is in neither the main set nor the delta;
// err |= 1 for a call id >= G, |= 2 for a cover that is not strictly increasing
__global__ __launch_bounds__(256) void k_cc_lookup(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                   size_t m, uint32_t G, const uint64_t* key, uint64_t nk,
                                                   const uint64_t* dkey, uint64_t ndk, int strict,
                                                   uint32_t* miss, uint32_t* err) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  const uint64_t base = off[0];
  for (size_t e = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < m; e += waves) {
    const uint32_t g = group[e];
    const uint64_t a = off[e], b = off[e + 1];
    if (g >= G) {
      if (__lane_id() == 0) atomicOr(err, 1u);
      for (uint64_t p = a + __lane_id(); p < b; p += 64) miss[p - base] = 0;
      continue;
    }
    for (uint64_t p = a + __lane_id(); p < b; p += 64) {
      const uint32_t pc = pcs[p];
      if (strict && p > a && pcs[p - 1] >= pc) atomicOr(err, 2u);
      const uint64_t k = ((uint64_t)g << 32) | pc;
      miss[p - base] = (pc != CC_SENT && !cc_has(key, nk, k) && !(ndk && cc_has(dkey, ndk, k))) ? 1u : 0u;
    }
  }
}

// the missing pairs, compacted in (input, PC) order: key and input
__global__ __launch_bounds__(256) void k_cc_pairs(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                  size_t m, const uint32_t* miss, const uint64_t* mpos,
                                                  uint64_t* mk, uint32_t* mv) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  const uint64_t base = off[0];
  for (size_t e = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < m; e += waves) {
    const uint64_t g = group[e];
    for (uint64_t p = off[e] + __lane_id(); p < off[e + 1]; p += 64)
      if (miss[p - base]) {
        const uint64_t q = mpos[p - base];
        mk[q] = (g << 32) | pcs[p];
        mv[q] = (uint32_t)e;
      }
  }
}

// small batches (n <= CC_SMALL pairs, inputs < 2^20): one workgroup sorts key << 20 | input in LDS
// (bitonic), flags the first holder of every key (acc) and writes the distinct keys (u, *nu)
__global__ __launch_bounds__(CC_SMALL_BLOCK) void k_cc_small(const uint64_t* mk, const uint32_t* mv, uint32_t n,
                                                             uint32_t np2, uint8_t* acc, uint64_t* u,
                                                             uint64_t* nu) {
  __shared__ uint64_t s[CC_SMALL];
  __shared__ uint32_t wsum[CC_SMALL_BLOCK / 64];
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < np2; i += CC_SMALL_BLOCK) s[i] = i < n ? (mk[i] << 20) | mv[i] : ~0ull;
  __syncthreads();
  for (uint32_t k = 2; k <= np2; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = t; i < np2 / 2; i += CC_SMALL_BLOCK) {
        const uint32_t lo = 2 * j * (i / j) + (i % j), hi = lo + j;
        const uint64_t a = s[lo], b = s[hi];
        if ((a > b) == ((lo & k) == 0)) {
          s[lo] = b;
          s[hi] = a;
        }
      }
      __syncthreads();
    }
  // each thread owns CC_SMALL / CC_SMALL_BLOCK consecutive slots
  constexpr uint32_t PER = CC_SMALL / CC_SMALL_BLOCK;
  uint32_t f = 0, cnt = 0;
  for (uint32_t r = 0; r < PER; r++) {
    const uint32_t i = t * PER + r;
    const bool first = i < n && (i == 0 || (s[i] >> 20) != (s[i - 1] >> 20));
    f |= (first ? 1u : 0u) << r;
    cnt += first;
    if (first) acc[(uint32_t)(s[i] & 0xFFFFFu)] = 1;
  }
  uint32_t x = cnt;  // block exclusive scan of cnt
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if ((int)__lane_id() >= d) x += y;
  }
  if (__lane_id() == 63) wsum[t >> 6] = x;
  __syncthreads();
  uint32_t wbase = 0;
  for (uint32_t w = 0; w < (t >> 6); w++) wbase += wsum[w];
  uint32_t pos = wbase + x - cnt;
  for (uint32_t r = 0; r < PER; r++)
    if ((f >> r) & 1u) u[pos++] = s[t * PER + r] >> 20;
  if (t == CC_SMALL_BLOCK - 1) *nu = wbase + x;
}

// large batches, after a stable sort of the pairs by key: first-of-run flags and the first holders
__global__ void k_cc_first(const uint64_t* k, const uint32_t* v, uint64_t n, uint8_t* acc, uint32_t* f) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const bool first = i == 0 || k[i] != k[i - 1];
    f[i] = first ? 1u : 0u;
    if (first) acc[v[i]] = 1;
  }
}

__global__ void k_cc_ucompact(const uint64_t* k, uint64_t n, const uint32_t* f, const uint64_t* pos, uint64_t* u) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (f[i]) u[pos[i]] = k[i];
}

// merge of two sorted key lists that share no key: each key's place = its index + the other list's
// keys below it
__global__ void k_cc_merge(const uint64_t* a, uint64_t na, const uint64_t* b, uint64_t nb, uint64_t* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb;
       i += (uint64_t)gridDim.x * blockDim.x) {
    if (i < na)
      out[i + lower_bound_dev<uint64_t>(b, 0, nb, a[i])] = a[i];
    else
      out[i - na + lower_bound_dev<uint64_t>(a, 0, na, b[i - na])] = b[i - na];
  }
}

// one wave per entry: its cover's keys (the sentinel PC as ~0: sorted last, dropped by the unique pass)
__global__ __launch_bounds__(256) void k_cc_keys(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                 size_t n, uint64_t* key, uint32_t* val) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t e = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < n; e += waves) {
    const uint64_t g = group[e];
    for (uint64_t p = off[e] + __lane_id(); p < off[e + 1]; p += 64) {
      const uint32_t pc = pcs[p];
      key[p] = pc == CC_SENT ? ~0ull : (g << 32) | pc;
      val[p] = 0;
    }
  }
}

__global__ void k_cc_uflag(const uint64_t* k, uint64_t n, uint32_t* f) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    f[i] = (k[i] != ~0ull && (i == 0 || k[i] != k[i - 1])) ? 1u : 0u;
}

// the accepted inputs' cover lengths (0 for the others)
__global__ void k_cc_lens(const uint64_t* off, const uint8_t* acc, size_t m, uint32_t* len) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x)
    len[i] = acc[i] ? (uint32_t)(off[i + 1] - off[i]) : 0u;
}

// the compacted offsets: off2[apos[e]] = lpos[e] for accepted e, off2[na] = the accepted PCs
__global__ void k_cc_offs(const uint8_t* acc, const uint64_t* apos, const uint64_t* lpos, size_t m, uint64_t* off2) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i <= m; i += (size_t)gridDim.x * blockDim.x)
    if (i == m)
      off2[apos[m]] = lpos[m];
    else if (acc[i])
      off2[apos[i]] = lpos[i];
}

// one wave per input: accepted ones gathered to their compacted place (covers, call, length)
__global__ __launch_bounds__(256) void k_cc_gather(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                   const uint16_t* prog_len, const uint8_t* acc, const uint64_t* apos,
                                                   size_t m, const uint64_t* off2, uint32_t* pcs2, uint32_t* group2,
                                                   uint16_t* prog_len2) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t e = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < m; e += waves) {
    if (!acc[e]) continue;
    const uint64_t j = apos[e], a = off[e], len = off[e + 1] - a, b = off2[j];
    for (uint64_t i = __lane_id(); i < len; i += 64) pcs2[b + i] = pcs[a + i];
    if (__lane_id() == 0) {
      group2[j] = group[e];
      if (prog_len2) prog_len2[j] = prog_len[e];
    }
  }
}

// corpusCover's keys as PCs, and each call's first place
__global__ void k_cc_export(const uint64_t* k, uint64_t n, uint32_t G, uint32_t* out, uint64_t* out_off) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n + G + 1;
       i += (uint64_t)gridDim.x * blockDim.x) {
    if (i < n)
      out[i] = (uint32_t)k[i];
    else
      out_off[i - n] = lower_bound_dev<uint64_t>(k, 0, n, (uint64_t)(i - n) << 32);
  }
}

unsigned wave_grid(size_t m) { return (unsigned)std::min<size_t>((m * 64 + 255) / 256 + 1, 65536); }

void swap_arr(DevArr<uint64_t>& a, DevArr<uint64_t>& b) {
  std::swap(a.p, b.p);
  std::swap(a.n, b.n);
}

// the delta's keys folded into the main array
void cc_fold(CoverSet& S, hipStream_t s) {
  if (!S.dn) return;
  const uint64_t nt = S.n + S.dn;
  S.tmp.ensure(nt + 1);
  k_cc_merge<<<grid_for(nt, 256, 16384), 256, 0, s>>>(S.key.p, S.n, S.dkey.p, S.dn, S.tmp.p);
  SYZ_LAUNCHED();
  swap_arr(S.key, S.tmp);
  S.n = nt;
  S.dn = 0;
}

// The batch's missing keys: acc[e] = 1 for the first holder of each (acc may be null: an unconditional
// append, whose covers need not be canonical), the distinct keys left in the scratch "cc_u" (count
// returned). Throws on bad input before anything changes.
uint64_t cc_classify(CoverSet& S, const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t m,
                     uint64_t Lm, uint32_t G, uint8_t* acc, hipStream_t s) {
  Scratch& sc = ctx().scratch;
  uint32_t* miss = sc.get<uint32_t>("cc_miss", Lm + 1);
  uint64_t* mpos = sc.get<uint64_t>("cc_mpos", Lm + 1);
  uint32_t* err = sc.get<uint32_t>("cc_err", 1);
  uint64_t* dnu = sc.get<uint64_t>("cc_nu", 1);
  SYZ_HIP(hipMemsetAsync(err, 0, 4, s));
  if (m) {
    k_cc_lookup<<<wave_grid(m), 256, 0, s>>>(pcs, off, group, m, G, S.key.p, S.n, S.dkey.p, S.dn, acc != nullptr,
                                             miss, err);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(miss, mpos, Lm, s);
  uint64_t* h = ctx().pinned.get<uint64_t>(2);
  SYZ_HIP(hipMemcpyAsync(&h[0], mpos + Lm, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(&h[1], err, 4, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint64_t nmiss = h[0];
  const uint32_t e = (uint32_t)h[1];
  if (e & 1) fail(SYZGPU_EINVAL, "group id >= ngroups");
  if (e & 2) fail(SYZGPU_EINVAL, "NewInput covers must be canonical (strictly increasing)");
  if (!nmiss) return 0;
  uint64_t* mk = sc.get<uint64_t>("cc_mk", nmiss + 1);
  uint32_t* mv = sc.get<uint32_t>("cc_mv", nmiss + 1);
  uint64_t* u = sc.get<uint64_t>("cc_u", nmiss + 1);
  uint8_t* a8 = acc ? acc : sc.get<uint8_t>("cc_acc0", m + 1);
  k_cc_pairs<<<wave_grid(m), 256, 0, s>>>(pcs, off, group, m, miss, mpos, mk, mv);
  SYZ_LAUNCHED();
  if (nmiss <= (uint64_t)CC_SMALL && m < (1u << 20)) {
    uint32_t np2 = 64;
    while (np2 < nmiss) np2 <<= 1;
    k_cc_small<<<1, CC_SMALL_BLOCK, 0, s>>>(mk, mv, (uint32_t)nmiss, np2, a8, u, dnu);
    SYZ_LAUNCHED();
  } else {
    uint64_t* mkt = sc.get<uint64_t>("cc_mkt", nmiss + 1);
    uint32_t* mvt = sc.get<uint32_t>("cc_mvt", nmiss + 1);
    radix_sort_pairs(mk, mv, mkt, mvt, nmiss, 44, s);  // stable: each key's pairs stay in input order
    uint32_t* f = sc.get<uint32_t>("cc_f", nmiss + 1);
    uint64_t* fpos = sc.get<uint64_t>("cc_fpos", nmiss + 1);
    k_cc_first<<<grid_for(nmiss, 256, 8192), 256, 0, s>>>(mk, mv, nmiss, a8, f);
    SYZ_LAUNCHED();
    exclusive_scan_u32(f, fpos, nmiss, s);
    k_cc_ucompact<<<grid_for(nmiss, 256, 8192), 256, 0, s>>>(mk, nmiss, f, fpos, u);
    SYZ_LAUNCHED();
    SYZ_HIP(hipMemcpyAsync(dnu, fpos + nmiss, 8, hipMemcpyDeviceToDevice, s));
  }
  SYZ_HIP(hipMemcpyAsync(&h[0], dnu, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  return h[0];
}

// the distinct missing keys of the last classify (scratch "cc_u") merged into the delta
void cc_commit(CoverSet& S, uint64_t nu, hipStream_t s) {
  if (!nu) return;
  const uint64_t* u = ctx().scratch.get<uint64_t>("cc_u", nu + 1);
  const uint64_t nt = S.dn + nu;
  S.tmp.ensure(nt + 1);
  k_cc_merge<<<grid_for(nt, 256, 16384), 256, 0, s>>>(S.dkey.p, S.dn, u, nu, S.tmp.p);
  SYZ_LAUNCHED();
  swap_arr(S.dkey, S.tmp);
  S.dn = nt;
  if (S.dn > std::max<uint64_t>(1ull << 20, S.n / 8)) cc_fold(S, s);
}

}  // namespace

void cc_ensure(CorpusHandle& H, hipStream_t s) {
  CoverSet& S = H.cc;
  if (S.built) return;
  PhaseTimer pt("cc_build");
  Scratch& sc = ctx().scratch;
  const uint64_t L = H.L;
  uint64_t* k = sc.get<uint64_t>("cc_bk", L + 1);
  uint32_t* v = sc.get<uint32_t>("cc_bv", L + 1);
  uint64_t* kt = sc.get<uint64_t>("cc_bkt", L + 1);
  uint32_t* vt = sc.get<uint32_t>("cc_bvt", L + 1);
  if (H.n) {
    k_cc_keys<<<wave_grid(H.n), 256, 0, s>>>(H.pcs.p, H.off.p, H.group.p, H.n, k, v);
    SYZ_LAUNCHED();
  }
  radix_sort_pairs(k, v, kt, vt, L, 64, s);
  uint32_t* f = sc.get<uint32_t>("cc_bf", L + 1);
  uint64_t* pos = sc.get<uint64_t>("cc_bpos", L + 1);
  if (L) {
    k_cc_uflag<<<grid_for(L, 256, 8192), 256, 0, s>>>(k, L, f);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(f, pos, L, s);
  uint64_t* h = ctx().pinned.get<uint64_t>(1);
  SYZ_HIP(hipMemcpyAsync(h, pos + L, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint64_t nu = *h;
  S.key.ensure(nu + 1);
  if (L) {
    k_cc_ucompact<<<grid_for(L, 256, 8192), 256, 0, s>>>(k, L, f, pos, S.key.p);
    SYZ_LAUNCHED();
  }
  S.dkey.ensure(1024);
  S.n = nu;
  S.dn = 0;
  S.built = true;
  SYZ_HIP(hipStreamSynchronize(s));
  pt.mark("sort_unique", s);
}

void cc_add(CorpusHandle& H, const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t m,
            uint64_t Lm, hipStream_t s) {
  if (!H.cc.built) return;
  cc_commit(H.cc, cc_classify(H.cc, pcs, off, group, m, Lm, H.G, nullptr, s), s);
}

uint64_t corpus_new_inputs(CorpusHandle& H, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                           const uint16_t* prog_len, size_t m, uint8_t* is_new, hipStream_t s) {
  if (!off || (m && !group)) fail(SYZGPU_EINVAL, "null pointer");
  PhaseTimer pt("new_inputs");
  cc_ensure(H, s);
  Scratch& sc = ctx().scratch;
  uint64_t* h = ctx().pinned.get<uint64_t>(2);
  SYZ_HIP(hipMemcpyAsync(&h[0], off, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(&h[1], off + m, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (h[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
  const uint64_t Lm = h[1];
  if (Lm && !pcs) fail(SYZGPU_EINVAL, "null pointer");
  uint8_t* acc = sc.get<uint8_t>("cc_acc", m + 1);
  if (m) SYZ_HIP(hipMemsetAsync(acc, 0, m, s));
  const uint64_t nu = cc_classify(H.cc, pcs, off, group, m, Lm, H.G, acc, s);
  pt.mark("classify", s);
  uint64_t na = 0;
  if (nu) {
    uint64_t* apos = sc.get<uint64_t>("cc_apos", m + 1);
    exclusive_scan_u8(acc, apos, m, s);
    SYZ_HIP(hipMemcpyAsync(&h[0], apos + m, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    na = h[0];
    if (na == m) {
      append_covers(H, pcs, off, group, prog_len, m, s, false);
    } else {
      uint32_t* len = sc.get<uint32_t>("cc_len", m + 1);
      uint64_t* off2 = sc.get<uint64_t>("cc_off2", na + 1);
      uint64_t* lpos = sc.get<uint64_t>("cc_lpos", m + 1);
      k_cc_lens<<<grid_for(m, 256, 4096), 256, 0, s>>>(off, acc, m, len);
      SYZ_LAUNCHED();
      exclusive_scan_u32(len, lpos, m, s);
      uint32_t* pcs2 = sc.get<uint32_t>("cc_pcs2", Lm + 1);
      uint32_t* group2 = sc.get<uint32_t>("cc_grp2", na + 1);
      uint16_t* pl2 = prog_len ? sc.get<uint16_t>("cc_pl2", na + 1) : nullptr;
      k_cc_offs<<<grid_for(m + 1, 256, 4096), 256, 0, s>>>(acc, apos, lpos, m, off2);
      SYZ_LAUNCHED();
      k_cc_gather<<<wave_grid(m), 256, 0, s>>>(pcs, off, group, prog_len, acc, apos, m, off2, pcs2, group2, pl2);
      SYZ_LAUNCHED();
      append_covers(H, pcs2, off2, group2, pl2, na, s, false);
    }
    cc_commit(H.cc, nu, s);
  }
  if (is_new && m) SYZ_HIP(hipMemcpyAsync(is_new, acc, m, hipMemcpyDefault, s));
  SYZ_HIP(hipStreamSynchronize(s));
  pt.mark("append", s);
  return na;
}

uint64_t cc_export(CorpusHandle& H, uint32_t* out, uint64_t* out_off, uint64_t cap, hipStream_t s) {
  cc_ensure(H, s);
  CoverSet& S = H.cc;
  const uint64_t nt = S.n + S.dn;
  if (nt > cap) return nt;
  uint64_t* all = ctx().scratch.get<uint64_t>("cc_all", nt + 1);
  k_cc_merge<<<grid_for(nt, 256, 16384), 256, 0, s>>>(S.key.p, S.n, S.dkey.p, S.dn, all);
  SYZ_LAUNCHED();
  k_cc_export<<<grid_for(nt + H.G + 1, 256, 16384), 256, 0, s>>>(all, nt, H.G, out, out_off);
  SYZ_LAUNCHED();
  SYZ_HIP(hipStreamSynchronize(s));
  return nt;
}

}  // namespace syz

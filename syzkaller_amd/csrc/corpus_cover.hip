// corpusCover on the resident store: syz-manager's per-call union of every accepted cover
// (manager.go:65, :121) and NewInput's gate on it (manager.go:609-616):
//
//     if len(cover.Difference(a.Cover, mgr.corpusCover[call])) == 0 { return }
//     mgr.corpusCover[call] = cover.Union(mgr.corpusCover[call], a.Cover)
//     mgr.corpus = append(mgr.corpus, a.RpcInput)
//
// The set is the store's: a device hash set of (call << 32 | PC) keys (keyhash.hpp), so a lookup is one
// or two loads and an update is a CAS per new key, O(batch). It holds every cover the store has held
// (the manager's corpus only grows through NewInput), built from the store's covers on first use — the
// first gate, or a keep that could drop a call's PCs (minimizeCorpus's own keep cannot: Minimize keeps
// a first holder of every PC) — and kept current by every append. PC 0xFFFFFFFF (cover.go's sentinel)
// is never in it: foreach drops it from every Difference and Union.
//
// The gate over a batch without the sequential loop: a key x missing from corpusCover is brought in by
// the FIRST input of the batch holding it (at that input x is still missing, so the input is accepted
// and unions x in; every later holder sees x covered). So input k is accepted iff it is the first
// holder of some missing key (the first-occurrence form of the fuzzer's maxCover update, without
// flakes). Two passes over the batch's PCs: (1) keys missing from corpusCover claim a slot in a batch
// table and take the least input holding them (atomicMin); (2) each missing key's least holder is
// accepted and inserts the key into corpusCover. Batches past CC_BT_MAX PCs sort their missing
// (key, input) pairs instead.
#include <algorithm>

#include "corpus.hpp"
#include "pipeline.hpp"

namespace syz {

// ---- the hash table (keyhash.hpp) ----------------------------------------------------------------

__global__ void k_kh_rehash(const uint64_t* ok, const uint32_t* ov, uint64_t ocap, uint64_t* nk, uint32_t* nv,
                            uint64_t nmask) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ocap; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = ok[i];
    if (k == KH_EMPTY) continue;
    uint64_t slot;
    kh_insert(nk, nmask, k, &slot);
    if (nv) nv[slot] = ov[i];
  }
}

__global__ void k_kh_insert(uint64_t* keys, uint32_t* vals, uint64_t mask, const uint64_t* in, const uint32_t* inv,
                            uint64_t n, unsigned long long* count) {
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = i0 + threadIdx.x;
    bool c = false;
    if (i < n) {
      uint64_t slot;
      c = kh_insert(keys, mask, in[i], &slot);
      if (vals) vals[slot] = inv ? inv[i] : 0u;
    }
    kh_count_claims(count, c);
  }
}

__global__ void k_kh_flag(const uint64_t* keys, uint64_t cap, uint32_t* f) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x)
    f[i] = keys[i] != KH_EMPTY ? 1u : 0u;
}

__global__ void k_kh_compact(const uint64_t* keys, uint64_t cap, const uint32_t* f, const uint64_t* pos,
                             uint64_t* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x)
    if (f[i]) out[pos[i]] = keys[i];
}

static uint64_t kh_cap_for(uint64_t n) {
  uint64_t c = 1024;
  while (c < 2 * n + 16) c <<= 1;
  return c;
}

void kh_init(KeyHash& H, uint64_t n, bool with_vals, hipStream_t s) {
  H.cap = kh_cap_for(n);
  H.with_vals = with_vals;
  H.keys.ensure(H.cap);
  SYZ_HIP(hipMemsetAsync(H.keys.p, 0xFF, H.cap * 8, s));
  if (with_vals) H.vals.ensure(H.cap);
  H.count.ensure(1);
  SYZ_HIP(hipMemsetAsync(H.count.p, 0, 8, s));
  H.bound = 0;
}

void kh_reserve(KeyHash& H, uint64_t more, hipStream_t s) {
  if (2 * (H.bound + more) + 16 <= H.cap) return;
  unsigned long long* hc = ctx().pinned.get<unsigned long long>(1);  // the exact count first
  SYZ_HIP(hipMemcpyAsync(hc, H.count.p, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  H.bound = *hc;
  if (2 * (H.bound + more) + 16 <= H.cap) return;
  const uint64_t ncap = kh_cap_for(2 * (H.bound + more));  // room for as many again
  DevArr<uint64_t> nk;
  DevArr<uint32_t> nv;
  nk.alloc(ncap);
  SYZ_HIP(hipMemsetAsync(nk.p, 0xFF, ncap * 8, s));
  if (H.with_vals) nv.alloc(ncap);
  k_kh_rehash<<<grid_for(H.cap, 256, 16384), 256, 0, s>>>(H.keys.p, H.with_vals ? H.vals.p : nullptr, H.cap, nk.p,
                                                         H.with_vals ? nv.p : nullptr, ncap - 1);
  SYZ_LAUNCHED();
  SYZ_HIP(hipStreamSynchronize(s));
  std::swap(H.keys.p, nk.p);
  std::swap(H.keys.n, nk.n);
  std::swap(H.vals.p, nv.p);
  std::swap(H.vals.n, nv.n);
  H.cap = ncap;
  nk.free();
  nv.free();
}

void kh_insert_sorted(KeyHash& H, const uint64_t* keys, const uint32_t* vals, uint64_t n, hipStream_t s) {
  if (!n) return;
  kh_reserve(H, n, s);
  k_kh_insert<<<grid_for(n, 256, 16384), 256, 0, s>>>(H.keys.p, H.with_vals ? H.vals.p : nullptr, H.mask(), keys,
                                                     vals, n, H.count.p);
  SYZ_LAUNCHED();
  H.bound += n;
}

uint64_t kh_export_sorted(KeyHash& H, uint64_t** out, hipStream_t s) {
  Scratch& sc = ctx().scratch;
  uint32_t* f = sc.get<uint32_t>("kh_f", H.cap + 1);
  uint64_t* pos = sc.get<uint64_t>("kh_pos", H.cap + 1);
  k_kh_flag<<<grid_for(H.cap, 256, 16384), 256, 0, s>>>(H.keys.p, H.cap, f);
  SYZ_LAUNCHED();
  exclusive_scan_u32(f, pos, H.cap, s);
  uint64_t* hn = ctx().pinned.get<uint64_t>(1);
  SYZ_HIP(hipMemcpyAsync(hn, pos + H.cap, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint64_t n = *hn;
  uint64_t* k = sc.get<uint64_t>("kh_out", n + 1);
  uint64_t* kt = sc.get<uint64_t>("kh_outt", n + 1);
  uint32_t* v = sc.get<uint32_t>("kh_outv", n + 1);
  uint32_t* vt = sc.get<uint32_t>("kh_outvt", n + 1);
  k_kh_compact<<<grid_for(H.cap, 256, 16384), 256, 0, s>>>(H.keys.p, H.cap, f, pos, k);
  SYZ_LAUNCHED();
  SYZ_HIP(hipMemsetAsync(v, 0, n * 4 + 4, s));
  radix_sort_pairs(k, v, kt, vt, n, 44, s);
  *out = k;
  return n;
}

namespace {

constexpr uint32_t CC_SENT = 0xFFFFFFFFu;
constexpr uint64_t CC_BT_MAX = 1ull << 22;  // batch PCs up to which the gate uses a batch table

// gate pass 1, one wave per input: err |= 1 for a call id >= G, |= 2 for a cover that is not strictly
// increasing; a key missing from corpusCover (miss[p] = 1) claims a batch-table slot and keeps the
// least input holding it
__global__ __launch_bounds__(256) void k_cc_gate1(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                  size_t m, uint32_t G, const uint64_t* cc, uint64_t ccmask,
                                                  uint64_t* bt, uint32_t* btv, uint64_t btmask, uint8_t* miss,
                                                  uint32_t* err) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t e = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < m; e += waves) {
    const uint32_t g = group[e];
    const uint64_t a = off[e], b = off[e + 1];
    if (g >= G) {
      if (__lane_id() == 0) atomicOr(err, 1u);
      for (uint64_t p = a + __lane_id(); p < b; p += 64) miss[p] = 0;
      continue;
    }
    for (uint64_t p = a + __lane_id(); p < b; p += 64) {
      const uint32_t pc = pcs[p];
      if (p > a && pcs[p - 1] >= pc) atomicOr(err, 2u);
      const uint64_t k = ((uint64_t)g << 32) | pc;
      const bool ms = pc != CC_SENT && kh_find(cc, ccmask, k) == KH_EMPTY;
      miss[p] = ms ? 1 : 0;
      if (ms) {
        uint64_t slot;
        kh_insert(bt, btmask, k, &slot);
        atomicMin(&btv[slot], (uint32_t)e);
      }
    }
  }
}

// gate pass 2: the least holder of each missing key is accepted and puts the key into corpusCover
__global__ __launch_bounds__(256) void k_cc_gate2(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                  size_t m, const uint8_t* miss, const uint64_t* bt,
                                                  const uint32_t* btv, uint64_t btmask, uint64_t* cc,
                                                  uint64_t ccmask, unsigned long long* cccount, uint8_t* acc) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t e = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < m; e += waves) {
    const uint64_t g = group[e];
    bool any = false;
    for (uint64_t p0 = off[e]; p0 < off[e + 1]; p0 += 64) {
      const uint64_t p = p0 + __lane_id();
      bool claimed = false;
      if (p < off[e + 1] && miss[p]) {
        const uint64_t k = (g << 32) | pcs[p];
        if (btv[kh_find(bt, btmask, k)] == (uint32_t)e) {
          any = true;
          uint64_t slot;
          claimed = kh_insert(cc, ccmask, k, &slot);
        }
      }
      kh_count_claims(cccount, claimed);
    }
    if (__ballot(any) && __lane_id() == 0) acc[e] = 1;
  }
}

// an unconditional append: every key of the covers into corpusCover (covers need not be canonical)
__global__ __launch_bounds__(256) void k_cc_add(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                size_t m, uint64_t* cc, uint64_t ccmask,
                                                unsigned long long* cccount) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t e = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < m; e += waves) {
    const uint64_t g = group[e];
    for (uint64_t p0 = off[e]; p0 < off[e + 1]; p0 += 64) {
      const uint64_t p = p0 + __lane_id();
      bool claimed = false;
      if (p < off[e + 1] && pcs[p] != CC_SENT) {
        uint64_t slot;
        claimed = kh_insert(cc, ccmask, (g << 32) | pcs[p], &slot);
      }
      kh_count_claims(cccount, claimed);
    }
  }
}

// large batches: the missing flags (u32, for the scan) and the checks of pass 1, no batch table
__global__ __launch_bounds__(256) void k_cc_lookup(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                   size_t m, uint32_t G, const uint64_t* cc, uint64_t ccmask,
                                                   uint32_t* miss, uint32_t* err) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t e = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < m; e += waves) {
    const uint32_t g = group[e];
    const uint64_t a = off[e], b = off[e + 1];
    if (g >= G) {
      if (__lane_id() == 0) atomicOr(err, 1u);
      for (uint64_t p = a + __lane_id(); p < b; p += 64) miss[p] = 0;
      continue;
    }
    for (uint64_t p = a + __lane_id(); p < b; p += 64) {
      const uint32_t pc = pcs[p];
      if (p > a && pcs[p - 1] >= pc) atomicOr(err, 2u);
      miss[p] = (pc != CC_SENT && kh_find(cc, ccmask, ((uint64_t)g << 32) | pc) == KH_EMPTY) ? 1u : 0u;
    }
  }
}

// the missing pairs, compacted in (input, PC) order: key and input
__global__ __launch_bounds__(256) void k_cc_pairs(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                  size_t m, const uint32_t* miss, const uint64_t* mpos,
                                                  uint64_t* mk, uint32_t* mv) {
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t e = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < m; e += waves) {
    const uint64_t g = group[e];
    for (uint64_t p = off[e] + __lane_id(); p < off[e + 1]; p += 64)
      if (miss[p]) {
        const uint64_t q = mpos[p];
        mk[q] = (g << 32) | pcs[p];
        mv[q] = (uint32_t)e;
      }
  }
}

// after a stable sort of the pairs by key: the first of each key's run accepts its input
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

// corpusCover's sorted keys as PCs, and each call's first place
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

void cc_fail(uint32_t e) {
  if (e & 1) fail(SYZGPU_EINVAL, "group id >= ngroups");
  if (e & 2) fail(SYZGPU_EINVAL, "NewInput covers must be canonical (strictly increasing)");
}

// acc[e] = 1 for the first holder of a missing key, the keys inserted into corpusCover; returns the
// number accepted (apos = the exclusive scan of acc). Throws on bad input before anything changes.
uint64_t cc_gate(KeyHash& S, const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t m, uint64_t Lm,
                 uint32_t G, uint8_t* acc, uint64_t* apos, hipStream_t s) {
  Scratch& sc = ctx().scratch;
  uint32_t* err = sc.get<uint32_t>("cc_err", 1);
  uint64_t* h = ctx().pinned.get<uint64_t>(2);
  SYZ_HIP(hipMemsetAsync(err, 0, 4, s));
  if (m) SYZ_HIP(hipMemsetAsync(acc, 0, m, s));
  kh_reserve(S, Lm, s);
  if (Lm <= CC_BT_MAX) {
    const uint64_t bcap = kh_cap_for(Lm);
    uint64_t* bt = sc.get<uint64_t>("cc_bt", bcap);
    uint32_t* btv = sc.get<uint32_t>("cc_btv", bcap);
    uint8_t* miss = sc.get<uint8_t>("cc_miss8", Lm + 1);
    SYZ_HIP(hipMemsetAsync(bt, 0xFF, bcap * 8, s));
    SYZ_HIP(hipMemsetAsync(btv, 0xFF, bcap * 4, s));
    if (m) {
      k_cc_gate1<<<wave_grid(m), 256, 0, s>>>(pcs, off, group, m, G, S.keys.p, S.mask(), bt, btv, bcap - 1, miss, err);
      SYZ_LAUNCHED();
    }
    // the checks are read before pass 2 changes corpusCover (a rejected batch changes nothing)
    SYZ_HIP(hipMemcpyAsync(&h[0], err, 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    cc_fail((uint32_t)h[0]);
    if (m) {
      k_cc_gate2<<<wave_grid(m), 256, 0, s>>>(pcs, off, group, m, miss, bt, btv, bcap - 1, S.keys.p, S.mask(),
                                              S.count.p, acc);
      SYZ_LAUNCHED();
    }
    S.bound += Lm;
  } else {
    uint32_t* miss = sc.get<uint32_t>("cc_miss", Lm + 1);
    uint64_t* mpos = sc.get<uint64_t>("cc_mpos", Lm + 1);
    k_cc_lookup<<<wave_grid(m), 256, 0, s>>>(pcs, off, group, m, G, S.keys.p, S.mask(), miss, err);
    SYZ_LAUNCHED();
    exclusive_scan_u32(miss, mpos, Lm, s);
    SYZ_HIP(hipMemcpyAsync(&h[0], mpos + Lm, 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(&h[1], err, 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    cc_fail((uint32_t)h[1]);
    const uint64_t nmiss = h[0];
    if (nmiss) {
      uint64_t* mk = sc.get<uint64_t>("cc_mk", nmiss + 1);
      uint32_t* mv = sc.get<uint32_t>("cc_mv", nmiss + 1);
      uint64_t* mkt = sc.get<uint64_t>("cc_mkt", nmiss + 1);
      uint32_t* mvt = sc.get<uint32_t>("cc_mvt", nmiss + 1);
      k_cc_pairs<<<wave_grid(m), 256, 0, s>>>(pcs, off, group, m, miss, mpos, mk, mv);
      SYZ_LAUNCHED();
      radix_sort_pairs(mk, mv, mkt, mvt, nmiss, 44, s);  // stable: each key's pairs stay in input order
      uint32_t* f = sc.get<uint32_t>("cc_f", nmiss + 1);
      uint64_t* fpos = sc.get<uint64_t>("cc_fpos", nmiss + 1);
      k_cc_first<<<grid_for(nmiss, 256, 8192), 256, 0, s>>>(mk, mv, nmiss, acc, f);
      SYZ_LAUNCHED();
      exclusive_scan_u32(f, fpos, nmiss, s);
      uint64_t* u = sc.get<uint64_t>("cc_u", nmiss + 1);
      k_cc_ucompact<<<grid_for(nmiss, 256, 8192), 256, 0, s>>>(mk, nmiss, f, fpos, u);
      SYZ_LAUNCHED();
      // the distinct keys are u[0, fpos[nmiss]); the rest of u is not written: insert up to nmiss with
      // the count read first
      SYZ_HIP(hipMemcpyAsync(&h[0], fpos + nmiss, 8, hipMemcpyDeviceToHost, s));
      SYZ_HIP(hipStreamSynchronize(s));
      kh_insert_sorted(S, u, nullptr, h[0], s);
    }
  }
  exclusive_scan_u8(acc, apos, m, s);
  SYZ_HIP(hipMemcpyAsync(&h[0], apos + m, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  return h[0];
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
  uint64_t* u = kt;  // (the sort's other buffer is free now)
  if (L) {
    k_cc_ucompact<<<grid_for(L, 256, 8192), 256, 0, s>>>(k, L, f, pos, u);
    SYZ_LAUNCHED();
  }
  kh_init(S.h, 2 * nu + (1u << 20), false, s);  // room to grow before the first rehash
  kh_insert_sorted(S.h, u, nullptr, nu, s);
  S.built = true;
  SYZ_HIP(hipStreamSynchronize(s));
  pt.mark("sort_unique_insert", s);
}

void cc_add(CorpusHandle& H, const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t m,
            uint64_t Lm, hipStream_t s) {
  if (!H.cc.built || !m) return;
  KeyHash& S = H.cc.h;
  kh_reserve(S, Lm, s);
  k_cc_add<<<wave_grid(m), 256, 0, s>>>(pcs, off, group, m, S.keys.p, S.mask(), S.count.p);
  SYZ_LAUNCHED();
  S.bound += Lm;
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
  // the append after the gate must not fail once the gate has put keys into corpusCover: the entry
  // limit and the store's capacity for the worst case (every input accepted) are settled first
  append_reserve(H, m, Lm, s);
  uint8_t* acc = is_new ? is_new : sc.get<uint8_t>("cc_acc", m + 1);
  uint64_t* apos = sc.get<uint64_t>("cc_apos", m + 1);
  // the compaction's buffers too, at their worst-case sizes (every input accepted)
  uint32_t* len = sc.get<uint32_t>("cc_len", m + 1);
  uint64_t* lpos = sc.get<uint64_t>("cc_lpos", m + 1);
  uint64_t* off2 = sc.get<uint64_t>("cc_off2", m + 1);
  uint32_t* pcs2 = sc.get<uint32_t>("cc_pcs2", Lm + 1);
  uint32_t* group2 = sc.get<uint32_t>("cc_grp2", m + 1);
  uint16_t* pl2 = prog_len ? sc.get<uint16_t>("cc_pl2", m + 1) : nullptr;
  const uint64_t na = cc_gate(H.cc.h, pcs, off, group, m, Lm, H.G, acc, apos, s);
  pt.mark("gate", s);
  if (na == m) {
    append_covers(H, pcs, off, group, prog_len, m, s, false);
  } else if (na) {
    k_cc_lens<<<grid_for(m, 256, 4096), 256, 0, s>>>(off, acc, m, len);
    SYZ_LAUNCHED();
    exclusive_scan_u32(len, lpos, m, s);
    k_cc_offs<<<grid_for(m + 1, 256, 4096), 256, 0, s>>>(acc, apos, lpos, m, off2);
    SYZ_LAUNCHED();
    k_cc_gather<<<wave_grid(m), 256, 0, s>>>(pcs, off, group, prog_len, acc, apos, m, off2, pcs2, group2, pl2);
    SYZ_LAUNCHED();
    append_covers(H, pcs2, off2, group2, pl2, na, s, false);
  }
  pt.mark("append", s);
  return na;
}

uint64_t cc_export(CorpusHandle& H, uint32_t* out, uint64_t* out_off, uint64_t cap, hipStream_t s) {
  cc_ensure(H, s);
  uint64_t* k = nullptr;
  const uint64_t n = kh_export_sorted(H.cc.h, &k, s);
  if (n > cap) return n;
  k_cc_export<<<grid_for(n + H.G + 1, 256, 16384), 256, 0, s>>>(k, n, H.G, out, out_off);
  SYZ_LAUNCHED();
  SYZ_HIP(hipStreamSynchronize(s));
  return n;
}

}  // namespace syz

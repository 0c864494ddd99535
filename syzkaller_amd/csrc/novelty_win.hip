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
//   P  k_part3<NOV>: the members' PCs transposed into 2^SB-address windows (one HBM read per PC), every
//      list checked strictly increasing on the way
//   M  k_nw_min: a workgroup per (call, window): direct min-rank table in LDS, then one pass over it in
//      PC order: a key is kept if the table holds it or a non-flake cover does (flakes of the window in
//      an LDS bitmap), a cover that wins a kept key is new (byte stores, deduplicated by an LDS rank
//      bitmap); the kept keys leave as a 4 KB bitmap per window, their count beside it
//   E  scan of the counts, then every window's bitmap expands to its PCs at its offset (the updated
//      tables, sorted by (call, PC)), a table's 0xFFFFFFFF last unless the call took a Union
//
// Integer work throughout; bit-exact by construction. Windows are direct-mapped only, so the PC span
// must fit WMAX windows (2^15 x 1024 = 32M addresses); a wider span (or G > 4096) falls back to the
// keyed table (novelty.hip).
#include <algorithm>
#include <cstdlib>
#include <numeric>

#include "panels_dev.hpp"
#include "pipeline.hpp"

namespace syz {

// window bits SB: 15 = 32K-entry tables (128 KB of LDS, one 1024-thread workgroup per CU), 14 = 16K-entry
// tables (64 KB, two 512-thread workgroups per CU, so one's metadata and table set-up overlap the
// other's walk)
template <uint32_t SB>
struct NwCfg {
  static constexpr uint32_t BITS = 1u << SB;      // addresses per window
  static constexpr uint32_t WORDS64 = BITS / 64;  // u64 words of a window's kept bitmap
  static constexpr uint32_t FLK = BITS / 32;      // LDS flake bitmap words
  static constexpr int BLOCK = SB >= 15 ? 1024 : 512;
  static constexpr uint32_t BMW = SB >= 15 ? PBM_WORDS : 2048;  // LDS rank bitmap words (winner dedup)
  static constexpr int EBLOCK = (int)(WORDS64 / 2);              // k_nw_emit: two words per thread
};

// combined members: call g's list is [table g (entry id n + g), its covers in batch order]
__global__ void k_nw_members(const uint32_t* members, const uint64_t* gstart, const uint32_t* group, size_t n,
                             uint32_t G, uint32_t* cmem, uint64_t* cstart) {
  const size_t tot = n > (size_t)G + 1 ? n : (size_t)G + 1;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
    if (i < n) {
      const uint32_t e = members[i];
      const uint32_t g = group[e] < G ? group[e] : 0u;  // an invalid id was counted in group 0
      cmem[i + g + 1] = e;
    }
    if (i < G) cmem[gstart[i] + i] = (uint32_t)n + (uint32_t)i;
    if (i <= G) cstart[i] = gstart[i] + i;
  }
}

// member lengths without a trailing 0xFFFFFFFF (foreach never matches it, cover.go:81-102; a table's
// is put back after the windows), which tables had one, and the span of the other PCs
__global__ __launch_bounds__(256) void k_nw_meta(const uint32_t* pcs, const uint64_t* off, const uint32_t* mc,
                                                 const uint64_t* mc_off, const uint32_t* cmem, size_t nm, uint32_t n1,
                                                 uint32_t* mlen, uint8_t* has_sent, uint32_t* span) {
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nm; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t e = cmem[i];
    const bool tab = e >= n1;
    const uint32_t* src = tab ? mc + mc_off[e - n1] : pcs + off[e];
    uint64_t len = tab ? mc_off[e - n1 + 1] - mc_off[e - n1] : off[e + 1] - off[e];
    if (len && src[len - 1] == SENT) {
      len--;
      if (tab) has_sent[e - n1] = 1;
    }
    mlen[i] = (uint32_t)len;
    if (len) {
      lo = min(lo, src[0]);
      hi = max(hi, src[len - 1]);
    }
  }
  lo = wave_min(lo);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t y = __shfl_xor(hi, d, 64);
    hi = y > hi ? y : hi;
  }
  if (__lane_id() == 0) {
    atomicMin(&span[0], lo);
    atomicMax(&span[1], hi);
  }
}

// M: one (call, window). tab = min member position per window offset; the table's position cstart[g]
// is OLD.
template <uint32_t SB>
__global__ __launch_bounds__(NwCfg<SB>::BLOCK) void k_nw_min(
    const PItem* items, const PChunk* __restrict__ chunks, const uint64_t* gchunk, const uint64_t* gdesc,
    const PGroup* pg, const uint16_t* __restrict__ desc, const uint32_t* __restrict__ elems, const uint64_t* cstart,
    uint32_t lo, const uint32_t* __restrict__ fl, const uint32_t* __restrict__ fstart, unsigned long long* kbits,
    uint32_t* wcount, uint8_t* sel8, uint8_t* upd, int dbg) {
  using K = NwCfg<SB>;
  constexpr int BLOCK = K::BLOCK;
  __shared__ uint32_t tab[K::BITS];
  __shared__ uint32_t bm[K::BMW];
  __shared__ uint32_t flk[K::FLK];
  __shared__ uint32_t red[BLOCK / 64 + 1];
  const PItem it = items[blockIdx.x];
  const uint32_t g = it.g, w = it.w, W = pg[g].W;
  for (uint32_t i = threadIdx.x; i < K::BITS; i += BLOCK) tab[i] = RANK_NONE;
  for (uint32_t i = threadIdx.x; i < K::FLK; i += BLOCK) flk[i] = 0;
  __syncthreads();
  // the flakes inside this window's addresses: fl[fstart[w], fstart[w + 1])
  const uint32_t wlo = lo + (w << SB);
  for (uint32_t i = fstart[w] + threadIdx.x; i < fstart[w + 1]; i += BLOCK) {
    const uint32_t o = fl[i] - wlo;
    atomicOr(&flk[o >> 5], 1u << (o & 31));
  }
  if (!(dbg & 1))
    for_window_elems<SYZ_DIRECT_RB, true>(it, chunks, gchunk, gdesc, pg, desc, elems, nullptr, 0u, BLOCK / 64,
                                          [&](uint32_t o, uint32_t R) {
                                            if (tab[o] > R) atomicMin(&tab[o], R);
                                          });
  if (dbg & 2) return;
  const uint64_t gb = cstart[g], ng = cstart[g + 1] - gb;
  const uint32_t span = (uint32_t)min<uint64_t>((uint64_t)K::BMW * 32, ng);
  const uint32_t words = (span + 31) / 32;
  for (uint32_t i = threadIdx.x; i < words; i += BLOCK) bm[i] = 0;
  __syncthreads();
  // in PC order: kept keys as bitmap words, new covers marked
  const unsigned lane = __lane_id();
  const uint64_t slot_bits = ((uint64_t)g * W + w) * K::WORDS64;
  uint32_t cnt = 0;
  int anynew = 0;
#pragma unroll 4
  for (uint32_t i = 0; i < K::BITS / BLOCK; i++) {
    const uint32_t o = i * BLOCK + threadIdx.x;
    const uint32_t r = tab[o];
    const bool old = r == (uint32_t)gb;
    const bool flake = (flk[o >> 5] >> (o & 31)) & 1u;
    const bool keep = r != RANK_NONE && (old || !flake);
    const uint64_t bal = __ballot(keep);
    if (lane == 0) {
      kbits[slot_bits + (o >> 6)] = bal;
      cnt += (uint32_t)__popcll(bal);
    }
    if (keep && !old) {
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
  const uint32_t tot = block_sum<BLOCK>(cnt, red);
  if (threadIdx.x == 0) wcount[(uint64_t)g * (W + 1) + w] = tot;
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

// fstart[w] = the first flake at or above window w's first address (w in [0, W]; nfl past the span)
__global__ void k_nw_fstart(const uint32_t* fl, uint64_t nfl, uint32_t lo, uint32_t W, uint32_t sb, uint32_t* fstart) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w <= W; w += gridDim.x * blockDim.x) {
    const uint64_t a = (uint64_t)lo + ((uint64_t)w << sb);
    fstart[w] = a > 0xFFFFFFFFull ? (uint32_t)nfl : (uint32_t)lower_bound_dev<uint32_t>(fl, 0, nfl, (uint32_t)a);
  }
}

// slot W of every call: its table's 0xFFFFFFFF stays unless the call took a Union (Union goes through
// foreach, cover.go:81-102)
__global__ void k_nw_sent(const uint8_t* has_sent, const uint8_t* upd, uint32_t G, uint32_t W, uint32_t* wcount) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x)
    wcount[(uint64_t)g * (W + 1) + W] = has_sent[g] && !upd[g] ? 1u : 0u;
}

// E: one slot per workgroup; the window's kept bitmap -> its PCs at wpos[slot]
template <uint32_t SB>
__global__ __launch_bounds__(NwCfg<SB>::EBLOCK) void k_nw_emit(const unsigned long long* __restrict__ kbits,
                                                      const uint64_t* __restrict__ wpos, uint32_t G, uint32_t W,
                                                      uint32_t lo, uint32_t* out, uint64_t cap, uint64_t* ooff,
                                                      int* err) {
  using K = NwCfg<SB>;
  constexpr int NE_BLOCK = K::EBLOCK;
  __shared__ uint32_t red[NE_BLOCK / 64 + 1];
  const uint64_t slot = blockIdx.x;
  const uint32_t g = (uint32_t)(slot / (W + 1)), w = (uint32_t)(slot % (W + 1));
  const uint64_t p0 = wpos[slot], c = wpos[slot + 1] - p0;
  if (threadIdx.x == 0 && w == 0) {
    ooff[g] = p0;
    if (g + 1 == G) ooff[G] = wpos[(uint64_t)G * (W + 1)];
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
  const uint64_t base = ((uint64_t)g * W + w) * K::WORDS64 + 2 * threadIdx.x;
  const unsigned long long b0 = kbits[base], b1 = kbits[base + 1];
  uint32_t tot;
  uint64_t p = p0 + block_excl_scan<NE_BLOCK>((uint32_t)(__popcll(b0) + __popcll(b1)), red, &tot);
  const uint32_t a0 = lo + (w << SB) + 128u * threadIdx.x;
  for (int h = 0; h < 2; h++) {
    unsigned long long m = h ? b1 : b0;
    while (m) {
      const int i = __ffsll(m) - 1;
      m &= m - 1;
      out[p++] = a0 + 64u * h + (uint32_t)i;
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
  static const int v = getenv("SYZGPU_NW_DBG") ? atoi(getenv("SYZGPU_NW_DBG")) : 0;
  return v;
}

// SYZGPU_NW_BITS=14|15: window bits (default: 14 while the span fits 1024 such windows, else 15)
static uint32_t nw_bits_forced() {
  static const uint32_t v = getenv("SYZGPU_NW_BITS") ? (uint32_t)atoi(getenv("SYZGPU_NW_BITS")) : 0u;
  return v == 14 || v == 15 ? v : 0u;
}

// false: the span does not fit the direct windows (or G is too large): use another strategy. err gets
// novelty.hip's bits (1 table, 2 group id, 4 cover, 8 capacity).
bool novelty_windows(const uint32_t* d_pcs, const uint64_t* d_off, const uint32_t* d_grp, size_t n, uint32_t G,
                     const uint32_t* d_mc, const uint64_t* d_mco, const uint32_t* d_fl, size_t nfl, uint8_t* d_new,
                     uint32_t* d_out, size_t out_cap, uint64_t* d_ooff, int* err, hipStream_t s) {
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
  uint64_t* mpos = sc.get<uint64_t>("nw_mpos", nm + 1);
  uint8_t* has_sent = sc.get<uint8_t>("nw_has_sent", G + 1);
  uint8_t* upd = sc.get<uint8_t>("nw_upd", G + 1);
  uint32_t* span = sc.get<uint32_t>("nw_span", 4);
  int* perr = sc.get<int>("nw_perr", 2);
  SYZ_HIP(hipMemsetAsync(perr, 0, 8, s));
  SYZ_HIP(hipMemsetAsync(has_sent, 0, G + 1, s));
  SYZ_HIP(hipMemsetAsync(upd, 0, G + 1, s));
  uint32_t* hinit = c.pinned.get<uint32_t>(16);
  hinit[0] = 0xFFFFFFFFu;
  hinit[1] = 0;
  SYZ_HIP(hipMemcpyAsync(span, hinit, 8, hipMemcpyHostToDevice, s));
  {
    ProfScope ps("novelty_group", s, (uint64_t)n * 28 + (uint64_t)nm * 24);
    group_partition_dev(d_grp, d_off, n, G, gstart, members, el, perr, s);
    k_nw_members<<<grid_for(std::max<size_t>(n, G + 1), 256, 8192), 256, 0, s>>>(members, gstart, d_grp, n, G, cmem,
                                                                                 cstart);
    SYZ_LAUNCHED();
    k_nw_meta<<<grid_for(nm, 256, 4096), 256, 0, s>>>(d_pcs, d_off, d_mc, d_mco, cmem, nm, (uint32_t)n, mlen, has_sent,
                                                      span);
    SYZ_LAUNCHED();
    exclusive_scan_u32(mlen, mpos, nm, s);
  }
  uint64_t* hbuf = c.pinned.get<uint64_t>((size_t)G + 8);
  SYZ_HIP(hipMemcpyAsync(hbuf, cstart, (G + 1) * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hbuf + G + 1, mpos + nm, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hbuf + G + 2, span, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hbuf + G + 3, perr, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (*reinterpret_cast<int*>(hbuf + G + 3)) fail(SYZGPU_EINVAL, "group id >= ngroups");
  const std::vector<uint64_t> hstart(hbuf, hbuf + G + 1);
  const uint64_t total = hbuf[G + 1];
  uint32_t lo = reinterpret_cast<uint32_t*>(hbuf + G + 2)[0], hi = reinterpret_cast<uint32_t*>(hbuf + G + 2)[1];
  if (lo > hi) lo = hi = 0;  // no PCs outside the sentinel
  auto nwin = [&](uint32_t sb) { return (((uint64_t)hi - (lo & ~((1u << sb) - 1))) >> sb) + 1; };
  uint32_t SB = nw_bits_forced();
  if (!SB) SB = nwin(14) <= WMAX ? 14 : 15;
  if (nwin(SB) > WMAX) return false;
  lo &= ~((1u << SB) - 1);  // windows on 2^SB boundaries: a window's addresses never wrap
  const uint32_t W = (uint32_t)nwin(SB);
  const uint32_t words64 = (1u << SB) / 64;
  // ---- plan: every call direct-mapped on W windows; blocks of 64 members; work items ----
  std::vector<uint32_t> hgblock(G + 1, 0), hbgroup;
  for (uint32_t g = 0; g < G; g++) {
    const uint32_t nb = (uint32_t)((hstart[g + 1] - hstart[g] + MEMB - 1) / MEMB);
    hgblock[g + 1] = hgblock[g] + nb;
    hbgroup.insert(hbgroup.end(), nb, g);
  }
  const uint32_t B = hgblock[G];
  const uint64_t chunk_bound = B + total / PCAP + 1;
  const uint64_t desc_bound = chunk_bound * (W + 1);
  // items: larger calls first (their windows are the long ones), so the grid's tail is short
  std::vector<uint32_t> order(G);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
    return hstart[x + 1] - hstart[x] > hstart[y + 1] - hstart[y];
  });
  const size_t nitems = (size_t)G * W;
  const size_t stage_bytes = (G + 1) * sizeof(PGroup) + (G + 1) * 4 + ((size_t)B + 1) * 4 + nitems * sizeof(PItem);
  uint8_t* stage = c.pinned.get<uint8_t>(stage_bytes + 64);
  PGroup* dpg = sc.get<PGroup>("nw_pg", G + 1);
  uint32_t* dgblock = sc.get<uint32_t>("nw_gblock", G + 1);
  uint32_t* dbgroup = sc.get<uint32_t>("nw_bgroup", (size_t)B + 1);
  PItem* ditems = sc.get<PItem>("nw_items", nitems + 1);
  {
    uint8_t* p = stage;
    PGroup* hp = reinterpret_cast<PGroup*>(p);
    for (uint32_t g = 0; g < G; g++) hp[g] = PGroup{SB, W, PMODE_DIRECT, 0};
    SYZ_HIP(hipMemcpyAsync(dpg, p, G * sizeof(PGroup), hipMemcpyHostToDevice, s));
    p += (G + 1) * sizeof(PGroup);
    std::memcpy(p, hgblock.data(), (G + 1) * 4);
    SYZ_HIP(hipMemcpyAsync(dgblock, p, (G + 1) * 4, hipMemcpyHostToDevice, s));
    p += (G + 1) * 4;
    if (B) {
      std::memcpy(p, hbgroup.data(), (size_t)B * 4);
      SYZ_HIP(hipMemcpyAsync(dbgroup, p, (size_t)B * 4, hipMemcpyHostToDevice, s));
    }
    p += ((size_t)B + 1) * 4;
    PItem* hi_ = reinterpret_cast<PItem*>(p);
    size_t k = 0;
    for (uint32_t g : order)
      for (uint32_t w = 0; w < W; w++) hi_[k++] = PItem{g, w};
    SYZ_HIP(hipMemcpyAsync(ditems, p, nitems * sizeof(PItem), hipMemcpyHostToDevice, s));
  }
  uint32_t* nsub = sc.get<uint32_t>("nw_nsub", (size_t)B + 1);
  uint64_t* cstartb = sc.get<uint64_t>("nw_cstartb", (size_t)B + 1);
  PChunk* chunks = sc.get<PChunk>("nw_chunks", chunk_bound + 1);
  uint64_t* gchunk = sc.get<uint64_t>("nw_gchunk", G + 1);
  uint64_t* gdesc = sc.get<uint64_t>("nw_gdesc", G + 1);
  uint16_t* desc = sc.get<uint16_t>("nw_desc", desc_bound + 1);
  uint32_t* elems = sc.get<uint32_t>("pm_elems", total + 1);
  const size_t nslots = (size_t)G * (W + 1);
  unsigned long long* kbits = sc.get<unsigned long long>("nw_kbits", nitems * words64 + 1);
  uint32_t* wcount = sc.get<uint32_t>("nw_wcount", nslots + 1);
  uint64_t* wpos = sc.get<uint64_t>("nw_wpos", nslots + 1);
  uint8_t* sel8 = sc.get<uint8_t>("nw_sel8", nm + 1);
  SYZ_HIP(hipMemsetAsync(sel8, 0, nm + 1, s));
  {
    ProfScope ps("novelty_part", s, total * 8 + (uint64_t)nm * 24);
    if (B) {
      k_blocks<<<grid_for(B, 256, 4096), 256, 0, s>>>(dbgroup, B, dgblock, cstart, mpos, nsub);
      SYZ_LAUNCHED();
    }
    exclusive_scan_u32(nsub, cstartb, B, s);
    if (B) {
      k_chunks<<<grid_for(B, 256, 4096), 256, 0, s>>>(dbgroup, B, dgblock, cstart, mpos, cstartb, chunks);
      SYZ_LAUNCHED();
    }
    k_gchunk<<<1, 1024, 0, s>>>(dgblock, G, cstartb, dpg, gchunk, gdesc);
    SYZ_LAUNCHED();
    NovSrc ns;
    ns.mc = d_mc;
    ns.mc_off = d_mco;
    ns.n1 = (uint32_t)n;
    k_part3<P3_BLOCK, P3_TPW, true><<<(unsigned)chunk_bound, P3_BLOCK, 0, s>>>(
        d_pcs, d_off, cmem, mpos, nullptr, chunks, cstartb + B, dpg, gchunk, gdesc, lo, elems, desc, err, ns);
    SYZ_LAUNCHED();
  }
  uint32_t* fstart = sc.get<uint32_t>("nw_fstart", (size_t)W + 2);
  {
    ProfScope ps("novelty_min", s, total * 4 + nitems * words64 * 8);
    k_nw_fstart<<<grid_for(W + 1, 256, 64), 256, 0, s>>>(d_fl, nfl, lo, W, SB, fstart);
    SYZ_LAUNCHED();
    if (SB == 14)
      k_nw_min<14><<<(unsigned)nitems, NwCfg<14>::BLOCK, 0, s>>>(ditems, chunks, gchunk, gdesc, dpg, desc, elems, cstart,
                                                                 lo, d_fl, fstart, kbits, wcount, sel8, upd, nw_dbg());
    else
      k_nw_min<15><<<(unsigned)nitems, NwCfg<15>::BLOCK, 0, s>>>(ditems, chunks, gchunk, gdesc, dpg, desc, elems, cstart,
                                                                 lo, d_fl, fstart, kbits, wcount, sel8, upd, nw_dbg());
    SYZ_LAUNCHED();
  }
  {
    ProfScope ps("novelty_emit", s, nitems * words64 * 8 + (uint64_t)nm * 6);
    k_nw_sent<<<grid_for(G, 256, 64), 256, 0, s>>>(has_sent, upd, G, W, wcount);
    SYZ_LAUNCHED();
    exclusive_scan_u32(wcount, wpos, nslots, s);
    if (SB == 14)
      k_nw_emit<14><<<(unsigned)nslots, NwCfg<14>::EBLOCK, 0, s>>>(kbits, wpos, G, W, lo, d_out, out_cap, d_ooff, err);
    else
      k_nw_emit<15><<<(unsigned)nslots, NwCfg<15>::EBLOCK, 0, s>>>(kbits, wpos, G, W, lo, d_out, out_cap, d_ooff, err);
    SYZ_LAUNCHED();
    k_nw_isnew<<<grid_for(nm, 256, 8192), 256, 0, s>>>(cmem, sel8, nm, (uint32_t)n, d_new);
    SYZ_LAUNCHED();
  }
  return true;
}

}  // namespace syz

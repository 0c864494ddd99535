// cover.Minimize for every call group of a corpus (cover/cover.go:105-131 driven by
// syz-manager/manager.go:507-527 minimizeCorpus), on the GPU.
//
// Exact reformulation: Minimize keeps input k (at Go-sort position k of its group)
// iff some PC of cov_k does not occur in any earlier-positioned input of the group — an input that
// is skipped adds nothing to the covered map, so covered after step k is the union of ALL inputs up
// to k. Minimize is therefore a first-occurrence problem over (group, pc) keys:
//   1. stable partition of entries by group (corpus order inside a group = Go's inputs[] order);
//   2. Go sort.Sort permutation of every group (gosort.hip) -> rank R of each entry;
//   3. bucket pass: each (pc, R) pair goes to a bucket of its group chosen by hash(pc), so that all
//      occurrences of a key meet in one bucket and a bucket's keys fit a workgroup's LDS;
//   4. hash pass: per bucket, an LDS open-addressing table computes min R per pc; the winning R of
//      every key marks its entry selected;
//   5. selected ranks in increasing order per group = Go's selection order.
// Everything is integer work: bit-exact by construction.
#include <algorithm>
#include <cstdlib>
#include <memory>
#include <numeric>

#include "panels.hpp"

namespace syz {

// ---- 1. stable partition by group -------------------------------------------------------------
// entries per wave chunk of the group partition (rounds of 64): short chunks give the latency-bound
// placement more waves (measured at config 4: 1024 -> 256 entries takes it from 0.23 to 0.17 ms), as
// long as the G x chunks counter table stays small (<= 8M counters); SYZGPU_GRP_PW overrides (A/B)
static uint32_t grp_pw(size_t n, uint32_t G) {
  const char* e = dev_env("SYZGPU_GRP_PW");
  if (e && *e) return (uint32_t)std::min(8192, std::max(64, atoi(e))) / 64 * 64;
  uint32_t pw = 256;
  while (pw < 8192 && (uint64_t)G * ((n + pw - 1) / pw) > (1ull << 23)) pw *= 2;
  return pw;
}

constexpr uint32_t MAX_GROUPS = 4096;  // calls (CallName ids) per corpus; len(sys.Calls) ~ 1.2k

// One wave per chunk of pw entries; per-wave group counters live in LDS (dynamic, 4*G u32).
__global__ __launch_bounds__(256) void k_grp_count(const uint32_t* group, size_t n, uint32_t G, uint32_t nchunks, uint32_t pw,
                                                   uint32_t* cnt, int* err) {
  extern __shared__ uint32_t run[];  // [4][G]
  const int w = threadIdx.x >> 6;
  uint32_t* mine = run + (size_t)w * G;
  for (uint32_t g = __lane_id(); g < G; g += 64) mine[g] = 0;
  wave_sync();
  const uint32_t chunk = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (chunk >= nchunks) return;
  const size_t beg = (size_t)chunk * pw;
  const size_t end = std::min(n, beg + pw);
  for (size_t i = beg + __lane_id(); i < end; i += 64) {
    uint32_t g = group[i];
    if (g >= G) {
      atomicOr(err, 1);
      g = 0;
    }
    atomicAdd(&mine[g], 1u);
  }
  wave_sync();
  // cnt is group-major: cnt[g * nchunks + chunk]
  for (uint32_t g = __lane_id(); g < G; g += 64) cnt[(size_t)g * nchunks + chunk] = mine[g];
}

__global__ __launch_bounds__(256) void k_grp_sumlen(const uint32_t* group, const uint64_t* off, size_t n,
                                                    uint32_t G, uint64_t* gpcs) {
  extern __shared__ unsigned long long lsum[];
  for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) lsum[g] = 0;
  __syncthreads();
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t g = group[i];
    if (g < G) atomicAdd(&lsum[g], (unsigned long long)(off[i + 1] - off[i]));
  }
  __syncthreads();
  for (uint32_t g = threadIdx.x; g < G; g += blockDim.x)
    if (lsum[g]) atomicAdd((unsigned long long*)&gpcs[g], lsum[g]);
}

// Stable placement: each wave walks its chunk in order; lanes of one group inside a 64-entry round
// are ranked with a ballot, the per-group running slot is kept in LDS. Also (PartOut, each optional):
// the group starts, the identity ranks (rank_of_member[m] = m, ent_of_rank[m] = members[m]: groups of
// one entry are never sorted) and the member lengths, so the step needs no pass of its own for them.
__global__ __launch_bounds__(256) void k_grp_scatter(const uint32_t* group, const uint64_t* off, size_t n,
                                                     uint32_t G, uint32_t nchunks, uint32_t pw,
                                                     const uint64_t* cnt_scan,
                                                     uint32_t* members, uint64_t* el, PartOut po) {
  extern __shared__ uint32_t run[];  // [4][G]
  const int w = threadIdx.x >> 6;
  uint32_t* mine = run + (size_t)w * G;
  if (po.gstart)
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g <= G; g += gridDim.x * blockDim.x)
      po.gstart[g] = g < G ? cnt_scan[(size_t)g * nchunks] : (uint64_t)n;
  const uint32_t chunk = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (chunk >= nchunks) return;
  for (uint32_t g = __lane_id(); g < G; g += 64) mine[g] = (uint32_t)cnt_scan[(size_t)g * nchunks + chunk];
  wave_sync();
  const size_t beg = (size_t)chunk * pw;
  const size_t end = std::min(n, beg + pw);
  for (size_t base = beg; base < end; base += 64) {
    const size_t i = base + __lane_id();
    const bool valid = i < end;
    // an invalid id goes to group 0, exactly as k_grp_count counted it, so every slot stays inside
    // [0, n) until the host reports the error
    const uint32_t g = valid && group[i] < G ? group[i] : 0;
    // the round's lengths are loaded once, up front: inside the leader loop below a load would be
    // waited for once per distinct group of the round (~60 at G = 289)
    const uint64_t len = valid ? off[i + 1] - off[i] : 0;
    uint64_t todo = __ballot(valid);
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const uint32_t gl = __shfl(g, leader, 64);
      const uint64_t mask = __ballot(valid && g == gl);
      const uint32_t b0 = mine[gl];
      if (valid && g == gl) {
        const uint32_t pos = b0 + __popcll(mask & lanemask_lt());
        members[pos] = (uint32_t)i;
        el[pos] = (len << 32) | pos;
        if (po.rank_of_member) {
          po.rank_of_member[pos] = pos;
          po.ent_of_rank[pos] = (uint32_t)i;
        }
        if (po.mlen) po.mlen[pos] = (uint32_t)len;
      }
      wave_sync();
      if (__lane_id() == (unsigned)leader) mine[gl] = b0 + __popcll(mask);
      wave_sync();
      todo &= ~mask;
    }
  }
}

__global__ void k_grp_starts(const uint64_t* cnt_scan, uint32_t G, uint32_t nchunks, size_t n, uint64_t* gstart) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g <= G; g += gridDim.x * blockDim.x)
    gstart[g] = g < G ? cnt_scan[(size_t)g * nchunks] : (uint64_t)n;
}

// ---- 2. ranks ------------------------------------------------------------------------------------
__global__ void k_ranks(const uint64_t* el, const uint32_t* perm, size_t n, const uint32_t* members,
                        uint32_t* rank_of_member, uint32_t* ent_of_rank) {
  for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (size_t)gridDim.x * blockDim.x) {
    const uint32_t gidx = (uint32_t)el[perm[r]];
    rank_of_member[gidx] = (uint32_t)r;
    ent_of_rank[r] = members[gidx];
  }
}

// the same over element ranges given as {lo, hi, ...} records (gosort packs or big call groups):
// blockIdx.y picks the range, the x blocks stride over it
__global__ void k_ranks_ranges(const uint64_t* el, const uint32_t* perm, const uint4* ranges, const uint32_t* members,
                               uint32_t* rank_of_member, uint32_t* ent_of_rank) {
  const uint4 rg = ranges[blockIdx.y];
  for (uint32_t r = rg.x + blockIdx.x * blockDim.x + threadIdx.x; r < rg.y; r += gridDim.x * blockDim.x) {
    const uint32_t gidx = (uint32_t)el[perm[r]];
    rank_of_member[gidx] = r;
    ent_of_rank[r] = members[gidx];
  }
}

// the same with the rank stored per ENTRY (the corpus index: its id vectors name entries, which
// appends never renumber)
__global__ void k_ranks_ranges_ent(const uint64_t* el, const uint32_t* perm, const uint4* ranges,
                                   const uint32_t* members, uint32_t* rank_of_entry, uint32_t* ent_of_rank) {
  const uint4 rg = ranges[blockIdx.y];
  for (uint32_t r = rg.x + blockIdx.x * blockDim.x + threadIdx.x; r < rg.y; r += gridDim.x * blockDim.x) {
    const uint32_t e = members[(uint32_t)el[perm[r]]];
    rank_of_entry[e] = r;
    ent_of_rank[r] = e;
  }
}

// ---- 3. bucket passes ------------------------------------------------------------------------------
struct Chunk {
  uint32_t g, mbeg, mend, pad;
};
struct GBucket {
  uint32_t base;  // first bucket id of the group
  uint32_t bits;  // log2(number of buckets of the group)
};

constexpr int BK_BLOCK = 256;
constexpr uint32_t HIST_LDS = 16384;  // buckets per group histogrammed in LDS

__device__ __forceinline__ uint32_t bucket_local(uint32_t pc, uint32_t bits) {
  return bits ? (hash32(pc) >> (32 - bits)) : 0u;
}

__global__ __launch_bounds__(BK_BLOCK) void k_bucket_count(const Chunk* chunks, const GBucket* gb, const uint32_t* members,
                                                           const uint64_t* off, const uint32_t* pcs, uint32_t* bcount) {
  __shared__ uint32_t hist[HIST_LDS];
  const Chunk ch = chunks[blockIdx.x];
  const GBucket b = gb[ch.g];
  const uint32_t nb = 1u << b.bits;
  const bool lds = nb <= HIST_LDS;
  if (lds) {
    for (uint32_t i = threadIdx.x; i < nb; i += BK_BLOCK) hist[i] = 0;
    __syncthreads();
  }
  for (uint32_t m = ch.mbeg; m < ch.mend; m++) {
    const uint32_t e = members[m];
    const uint64_t beg = off[e], end = off[e + 1];
    for (uint64_t k = beg + threadIdx.x; k < end; k += BK_BLOCK) {
      const uint32_t lb = bucket_local(pcs[k], b.bits);
      if (lds)
        atomicAdd(&hist[lb], 1u);
      else
        atomicAdd(&bcount[b.base + lb], 1u);
    }
  }
  if (lds) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += BK_BLOCK)
      if (hist[i]) atomicAdd(&bcount[b.base + i], hist[i]);
  }
}

// ---- 4. hash pass: min rank per pc inside one bucket -------------------------------------------
constexpr int HT_BLOCK = 512;
constexpr uint32_t HT_SLOTS = 16384;
constexpr uint32_t HT_EMPTY = 0xFFFFFFFFu;  // pc == 0xFFFFFFFF is handled out of table
constexpr uint32_t HT_ROUND_ITEMS = 12288;

__device__ __forceinline__ uint32_t hslot(uint32_t pc) { return (pc * 0x9E3779B1u) >> 18; }  // 14 bits

// ---- 5. selection outputs ------------------------------------------------------------------------
// Store path: kept flags in ENTRY order (coalesced stores; the rank-ordered form walks a permutation)
// and the len(p.Calls) histogram of kept programs of the groups this rank counts (count_hist[g]).
__global__ __launch_bounds__(256) void k_select_store(const uint32_t* sel_bits, const uint32_t* rank_of_entry, size_t n,
                                                      const uint16_t* prog_len, const uint32_t* group,
                                                      const uint8_t* count_hist, int32_t C, uint8_t* selected,
                                                      int64_t* hist, int* err) {
  extern __shared__ unsigned long long lh[];
  const bool do_hist = hist != nullptr;
  if (do_hist) {
    for (int32_t i = threadIdx.x; i <= C; i += blockDim.x) lh[i] = 0;
    __syncthreads();
  }
  // SS_U entries per thread at once: the dependent gathers (rank -> winner bit) of all of them are in
  // flight together instead of one chain per grid-stride step
  constexpr int SS_U = 8;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t e0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e0 < n; e0 += stride * SS_U) {
    uint32_t r[SS_U], b[SS_U];
#pragma unroll
    for (int k = 0; k < SS_U; k++) r[k] = e0 + k * stride < n ? rank_of_entry[e0 + k * stride] : 0;
#pragma unroll
    for (int k = 0; k < SS_U; k++) b[k] = e0 + k * stride < n ? sel_bits[r[k] >> 5] : 0;
#pragma unroll
    for (int k = 0; k < SS_U; k++) {
      const size_t e = e0 + k * stride;
      const bool in = e < n;
      const uint32_t s = (b[k] >> (r[k] & 31)) & 1u;
      if (in && selected) selected[e] = (uint8_t)s;
      if (in && do_hist && s && (!count_hist || count_hist[group[e]])) {
        const uint32_t L = prog_len[e];
        if ((int32_t)L > C)
          atomicOr(err, 2);
        else
          atomicAdd(&lh[L], 1ull);
      }
    }
  }
  if (do_hist) {
    __syncthreads();
    for (int32_t i = threadIdx.x; i <= C; i += blockDim.x)
      if (lh[i]) atomicAdd((unsigned long long*)&hist[i], lh[i]);
  }
}

__global__ void k_invert(const uint32_t* members, size_t n, uint32_t* member_of) {
  for (size_t m = (size_t)blockIdx.x * blockDim.x + threadIdx.x; m < n; m += (size_t)gridDim.x * blockDim.x)
    member_of[members[m]] = (uint32_t)m;
}

// ---- host orchestration ------------------------------------------------------------------------------

// syzgpu_minimize_order helpers: elements (len << 32) | index, output index within the group
__global__ void k_order_el(const uint64_t* lens, size_t n, uint64_t* el) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    el[i] = (lens[i] << 32) | (uint64_t)i;
}

__global__ void k_order_out(const uint64_t* el, const uint32_t* perm, const uint64_t* goff, uint32_t G, size_t n,
                            int64_t* out) {
  for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (size_t)gridDim.x * blockDim.x) {
    const uint32_t g = (uint32_t)upper_bound_dev<uint64_t>(goff, 0, G + 1, r) - 1;
    out[r] = (int64_t)(uint32_t)el[perm[r]] - (int64_t)goff[g];
  }
}

void group_partition_dev(const uint32_t* group, const uint64_t* off, size_t n, uint32_t G, uint64_t* gstart,
                         uint32_t* members, uint64_t* el, int* err, hipStream_t s, PartOut po) {
  Scratch& sc = ctx().scratch;
  const uint32_t pw = grp_pw(n, G);
  const uint32_t nchunks = (uint32_t)((n + pw - 1) / pw);
  uint32_t* cnt = sc.get<uint32_t>("mz_cnt", (size_t)G * nchunks + 1);
  uint64_t* cnt_scan = sc.get<uint64_t>("mz_cnt_scan", (size_t)G * nchunks + 1);
  const unsigned wg = (unsigned)(((size_t)nchunks * 64 + 255) / 256);
  if (n) {  // (k_grp_count writes every count the scan reads: no clearing)
    k_grp_count<<<wg, 256, 4 * G * 4, s>>>(group, n, G, nchunks, pw, cnt, err);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(cnt, cnt_scan, (size_t)G * nchunks, s);
  if (n) {
    po.gstart = gstart;
    k_grp_scatter<<<wg, 256, 4 * G * 4, s>>>(group, off, n, G, nchunks, pw, cnt_scan, members, el, po);
    SYZ_LAUNCHED();
  } else {
    k_grp_starts<<<grid_for(G + 1, 256, 1024), 256, 0, s>>>(cnt_scan, G, nchunks, n, gstart);
    SYZ_LAUNCHED();
  }
}

// groups of one entry are not sorted (no pack or round touches them): their rank is their position
__global__ void k_rank_init(const uint32_t* members, size_t n, uint32_t* rank_of_member, uint32_t* ent_of_rank) {
  for (size_t m = (size_t)blockIdx.x * blockDim.x + threadIdx.x; m < n; m += (size_t)gridDim.x * blockDim.x) {
    rank_of_member[m] = (uint32_t)m;
    ent_of_rank[m] = members[m];
  }
}

void rank_init_dev(const uint32_t* members, size_t n, uint32_t* rank_of_member, uint32_t* ent_of_rank, hipStream_t s) {
  if (!n) return;
  k_rank_init<<<grid_for(n, 256, 4096), 256, 0, s>>>(members, n, rank_of_member, ent_of_rank);
  SYZ_LAUNCHED();
}

void ranks_packs(const uint64_t* el, const uint32_t* perm, const GosortPlan& P, const uint32_t* members,
                 uint32_t* rank_of_member, uint32_t* ent_of_rank, hipStream_t q) {
  if (!P.npacks) return;  // a pack holds at most GS_T_SEG elements
  k_ranks_ranges<<<dim3(GS_T_SEG / 1024, P.npacks), 256, 0, q>>>(el, perm, reinterpret_cast<const uint4*>(P.packs),
                                                                 members, rank_of_member, ent_of_rank);
  SYZ_LAUNCHED();
}

void ranks_big(const uint64_t* el, const uint32_t* perm, const GosortPlan& P, const uint32_t* members,
               uint32_t* rank_of_member, uint32_t* ent_of_rank, hipStream_t q) {
  if (!P.nbig) return;
  const unsigned gx = (unsigned)std::min<uint64_t>(std::max<uint64_t>(1, P.big_max / 2048), 256);
  k_ranks_ranges<<<dim3(gx, P.nbig), 256, 0, q>>>(el, perm, reinterpret_cast<const uint4*>(P.big), members,
                                                 rank_of_member, ent_of_rank);
  SYZ_LAUNCHED();
}

static MinJob& lane_job() {
  Context& c = ctx();
  if (!c.own_job) c.own_job = std::make_shared<MinJob>();
  return *c.own_job;
}

// the lane of this thread's last one-call minimize (syzgpu_minimize_grouped_fetch runs there)
static thread_local Context* t_min_lane = nullptr;
static thread_local uint64_t t_min_gen = 0;

// one call: begin + outputs on the lane's own job (remembered for syzgpu_minimize_grouped_fetch)
void minimize_grouped_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, const uint16_t* prog_len,
                          size_t n, uint32_t G, int32_t C, uint8_t* selected, int64_t* len_hist, int64_t* out_idx,
                          uint64_t* group_out_off, hipStream_t s) {
  Context& c = ctx();
  MinJob& J = lane_job();
  c.last_job = nullptr;
  RawMinArgs a{pcs, off, group, prog_len, n, G};
  a.s = s;
  minimize_raw_begin(J, a);
  RawEndArgs e;
  e.C = C;
  e.selected = selected;
  e.len_hist = len_hist;
  e.out_idx = out_idx;
  e.group_out_off = group_out_off;
  e.s = s;
  minimize_raw_end(J, e);
  c.last_job = &J;
  c.last_thread = std::this_thread::get_id();
  t_min_lane = &c;
  t_min_gen = c.gen;
}

void minimize_fetch(int64_t* out_idx, uint64_t* group_out_off, size_t n, uint32_t G) {
  Context& c = ctx();
  if (!c.own_job || c.last_job != c.own_job.get() || c.last_thread != std::this_thread::get_id() ||
      c.own_job->n != n || c.own_job->G != G)
    fail(SYZGPU_EINVAL, "no matching minimize result on this thread");
  minimize_raw_fetch(*c.own_job, out_idx, group_out_off);
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzgpu_minimize_grouped_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                const uint16_t* prog_len, size_t n, uint32_t ngroups, int32_t C, uint8_t* selected,
                                int64_t* len_hist, void* stream) {
  SYZ_API_BODY({
    if (len_hist && (C <= 0 || !prog_len)) fail(SYZGPU_EINVAL, "len_hist needs prog_len and C > 0");
    minimize_grouped_dev(pcs, off, group, prog_len, n, ngroups, C, selected, len_hist, nullptr, nullptr,
                         (hipStream_t)stream);
  })
}

int syzgpu_minimize_grouped_ordered_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                        const uint16_t* prog_len, size_t n, uint32_t ngroups, int32_t C,
                                        uint8_t* selected, int64_t* len_hist, int64_t* out_idx,
                                        uint64_t* group_out_off, void* stream) {
  SYZ_API_BODY({
    if (len_hist && (C <= 0 || !prog_len)) fail(SYZGPU_EINVAL, "len_hist needs prog_len and C > 0");
    if (!off || (n && !group)) fail(SYZGPU_EINVAL, "null pointer");
    minimize_grouped_dev(pcs, off, group, prog_len, n, ngroups, C, selected, len_hist, out_idx, group_out_off,
                         (hipStream_t)stream);
  })
}

int syzgpu_minimize_grouped_fetch(int64_t* out_idx, uint64_t* group_out_off, size_t n, uint32_t ngroups) {
  want_lane(t_min_lane, t_min_gen);
  SYZ_API_BODY({
    if (!group_out_off) fail(SYZGPU_EINVAL, "null pointer");
    minimize_fetch(out_idx, group_out_off, n, ngroups);
  })
}

int syzgpu_minimize_grouped(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                            uint32_t ngroups, int64_t* out_idx, uint64_t* group_out_off) {
  SYZ_API_BODY({
    if (!off || !group_out_off || (n && (!group || !out_idx))) fail(SYZGPU_EINVAL, "null pointer");
    if (off[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
    hipStream_t s = C_.stream;
    const uint64_t tot = off[n];
    uint32_t* dp = C_.scratch.get<uint32_t>("mg_pcs", tot + 1);
    uint64_t* doff = C_.scratch.get<uint64_t>("mg_off", n + 1);
    uint32_t* dg = C_.scratch.get<uint32_t>("mg_grp", n + 1);
    if (tot) SYZ_HIP(hipMemcpyAsync(dp, pcs, tot * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(doff, off, (n + 1) * 8, hipMemcpyHostToDevice, s));
    if (n) SYZ_HIP(hipMemcpyAsync(dg, group, n * 4, hipMemcpyHostToDevice, s));
    MinJob& J = lane_job();
    C_.last_job = nullptr;
    RawMinArgs a{dp, doff, dg, nullptr, n, ngroups};
    a.s = s;
    minimize_raw_begin(J, a);
    minimize_raw_fetch(J, out_idx, group_out_off);
  })
}

int syzgpu_minimize_order(const uint64_t* lens, const uint64_t* group_off, uint32_t ngroups, int64_t* perm) {
  SYZ_API_BODY({
    if (!group_off || ngroups == 0) fail(SYZGPU_EINVAL, "null pointer / no groups");
    if (group_off[0] != 0) fail(SYZGPU_EINVAL, "group offsets must start at 0");
    const size_t n = group_off[ngroups];
    if (n && (!lens || !perm)) fail(SYZGPU_EINVAL, "null pointer");
    if (n >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "too many inputs");
    for (uint32_t g = 0; g < ngroups; g++)
      if (group_off[g + 1] < group_off[g]) fail(SYZGPU_EINVAL, "group offsets must be non-decreasing");
    for (size_t i = 0; i < n; i++)
      if (lens[i] >> 32) fail(SYZGPU_EINVAL, "cover length >= 2^32");
    hipStream_t s = C_.stream;
    Scratch& sc = C_.scratch;
    uint64_t* dl = sc.get<uint64_t>("mo_lens", n + 1);
    uint64_t* dgo = sc.get<uint64_t>("mo_goff", ngroups + 1);
    uint64_t* el = sc.get<uint64_t>("mo_el", n + 1);
    uint32_t* p = sc.get<uint32_t>("mo_perm", n + 1);
    int64_t* out = sc.get<int64_t>("mo_out", n + 1);
    if (n) SYZ_HIP(hipMemcpyAsync(dl, lens, n * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(dgo, group_off, (ngroups + 1) * 8, hipMemcpyHostToDevice, s));
    if (n) {
      k_order_el<<<grid_for(n, 256, 4096), 256, 0, s>>>(dl, n, el);
      SYZ_LAUNCHED();
      std::vector<uint64_t> hs(group_off, group_off + ngroups + 1);
      gosort_groups(el, p, n, hs, ngroups, s);
      k_order_out<<<grid_for(n, 256, 4096), 256, 0, s>>>(el, p, dgo, ngroups, n, out);
      SYZ_LAUNCHED();
      SYZ_HIP(hipMemcpyAsync(perm, out, n * 8, hipMemcpyDeviceToHost, s));
    }
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_minimize(const uint32_t* pcs, const uint64_t* off, size_t ncov, int64_t* out_idx, size_t* out_n) {
  SYZ_API_BODY({
    if (!off || !out_n) fail(SYZGPU_EINVAL, "null pointer");
    std::vector<uint32_t> grp(ncov, 0);
    uint64_t goff[2] = {0, 0};
    if (ncov == 0) {
      *out_n = 0;
      return SYZGPU_OK;
    }
    int rc = syzgpu_minimize_grouped(pcs, off, grp.data(), ncov, 1, out_idx, goff);
    if (rc) return rc;
    *out_n = (size_t)goff[1];
  })
}

}  // extern "C"

namespace syz {


// =====================================================================================================
// Resident corpus store (the device analog of syz-manager's mgr.corpus, manager.go:52-65).
//
// Ingest turns the raw CSR covers into per-call dense PC ids once: every distinct PC of call g gets
// an id in [0, P_g) (hash buckets of the call, an LDS table per bucket), every cover becomes its
// sorted id list, and each cover records where its list crosses every 32768-id window. Minimize on
// the store is then one streaming pass: a workgroup per (call, id-window, cover chunk) keeps the
// window's min Go-sort rank per id in a direct-mapped LDS table (no hashing, no scatter), and the
// rank that wins an id marks its input as kept (cover.go:116-129 as first occurrence).
// =====================================================================================================

__global__ __launch_bounds__(BK_BLOCK) void k_bucket_scatter_pos(const Chunk* chunks, const GBucket* gb,
                                                                 const uint32_t* members, const uint64_t* off,
                                                                 const uint32_t* pcs, const uint64_t* boff,
                                                                 uint32_t* bcursor, uint2* items) {
  __shared__ uint32_t hist[HIST_LDS];
  const Chunk ch = chunks[blockIdx.x];
  const GBucket b = gb[ch.g];
  const uint32_t nb = 1u << b.bits;
  const bool lds = nb <= HIST_LDS;
  if (lds) {
    for (uint32_t i = threadIdx.x; i < nb; i += BK_BLOCK) hist[i] = 0;
    __syncthreads();
    for (uint32_t m = ch.mbeg; m < ch.mend; m++) {
      const uint32_t e = members[m];
      for (uint64_t k = off[e] + threadIdx.x; k < off[e + 1]; k += BK_BLOCK)
        atomicAdd(&hist[bucket_local(pcs[k], b.bits)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += BK_BLOCK)
      if (hist[i]) hist[i] = atomicAdd(&bcursor[b.base + i], hist[i]);
    __syncthreads();
  }
  for (uint32_t m = ch.mbeg; m < ch.mend; m++) {
    const uint32_t e = members[m];
    for (uint64_t k = off[e] + threadIdx.x; k < off[e + 1]; k += BK_BLOCK) {
      const uint32_t pc = pcs[k];
      const uint32_t lb = bucket_local(pc, b.bits);
      const uint32_t slot = lds ? atomicAdd(&hist[lb], 1u) : atomicAdd(&bcursor[b.base + lb], 1u);
      items[boff[b.base + lb] + slot] = make_uint2(pc, (uint32_t)k);
    }
  }
}

// LDS open-addressing set keyed by pc; the sentinel pc 0xFFFFFFFF lives in slot HT_SLOTS (extra).
__device__ __forceinline__ int ht_insert(uint32_t* keys, uint32_t pc) {
  if (pc == HT_EMPTY) {
    keys[HT_SLOTS] = 1;
    return (int)HT_SLOTS;
  }
  uint32_t h = hslot(pc);
  for (uint32_t probes = 0; probes < HT_SLOTS; probes++) {
    const uint32_t cur = keys[h];
    if (cur == pc) return (int)h;
    if (cur == HT_EMPTY) {
      const uint32_t old = atomicCAS(&keys[h], HT_EMPTY, pc);
      if (old == HT_EMPTY || old == pc) return (int)h;
    }
    h = (h + 1) & (HT_SLOTS - 1);
  }
  return -1;
}

__device__ __forceinline__ int ht_find(const uint32_t* keys, uint32_t pc) {
  if (pc == HT_EMPTY) return (int)HT_SLOTS;
  uint32_t h = hslot(pc);
  for (uint32_t probes = 0; probes < HT_SLOTS; probes++) {
    const uint32_t cur = keys[h];
    if (cur == pc) return (int)h;
    if (cur == HT_EMPTY) return -1;
    h = (h + 1) & (HT_SLOTS - 1);
  }
  return -1;
}

// mode 0: count distinct keys per bucket. mode 1: assign ids id_base[b] + rank(slot), write the
// dictionary and ids[k] for every occurrence.
__global__ __launch_bounds__(HT_BLOCK) void k_bucket_ids(int mode, const uint64_t* boff, uint32_t nbuckets,
                                                         const uint2* items, uint32_t* dcount, const uint64_t* dscan,
                                                         const uint32_t* bucket_group, const GBucket* gb,
                                                         const uint64_t* gdict, uint32_t* dict, uint32_t* ids,
                                                         int* err) {
  __shared__ uint32_t keys[HT_SLOTS + 1];
  __shared__ uint32_t rank[HT_SLOTS + 1];
  __shared__ uint32_t red[HT_BLOCK / 64 + 1];
  __shared__ int full;
  for (uint32_t bk = blockIdx.x; bk < nbuckets; bk += gridDim.x) {
    const uint64_t beg = boff[bk], end = boff[bk + 1];
    for (uint32_t i = threadIdx.x; i <= HT_SLOTS; i += HT_BLOCK) keys[i] = i == HT_SLOTS ? 0 : HT_EMPTY;
    if (threadIdx.x == 0) full = 0;
    __syncthreads();
    for (uint64_t k = beg + threadIdx.x; k < end; k += HT_BLOCK)
      if (ht_insert(keys, items[k].x) < 0) full = 1;
    __syncthreads();
    if (full) {
      if (threadIdx.x == 0) atomicOr(err, 4);
      continue;
    }
    // rank occupied slots (slot order; the sentinel slot last)
    uint32_t base = 0;
    for (uint32_t s0 = 0; s0 <= HT_SLOTS; s0 += HT_BLOCK) {
      const uint32_t s = s0 + threadIdx.x;
      uint32_t occ = 0;
      if (s < HT_SLOTS)
        occ = keys[s] != HT_EMPTY;
      else if (s == HT_SLOTS)
        occ = keys[HT_SLOTS] != 0;
      uint32_t tot;
      const uint32_t r = block_excl_scan<HT_BLOCK>(occ, red, &tot);
      if (s <= HT_SLOTS) rank[s] = occ ? base + r : 0xFFFFFFFFu;
      base += tot;
    }
    if (mode == 0) {
      if (threadIdx.x == 0) dcount[bk] = base;
      __syncthreads();
      continue;
    }
    const uint32_t g = bucket_group[bk];
    const uint32_t idb = (uint32_t)(dscan[bk] - dscan[gb[g].base]);
    for (uint32_t s = threadIdx.x; s <= HT_SLOTS; s += HT_BLOCK)
      if (rank[s] != 0xFFFFFFFFu) dict[gdict[g] + idb + rank[s]] = s == HT_SLOTS ? HT_EMPTY : keys[s];
    __syncthreads();
    for (uint64_t k = beg + threadIdx.x; k < end; k += HT_BLOCK) {
      const uint2 it = items[k];
      ids[it.y] = idb + rank[ht_find(keys, it.x)];
    }
    __syncthreads();
  }
}

__global__ void k_bucket_group(const GBucket* gb, uint32_t G, uint32_t* bucket_group) {
  for (uint32_t g = blockIdx.x; g < G; g += gridDim.x)
    for (uint32_t b = threadIdx.x; b < (1u << gb[g].bits); b += blockDim.x) bucket_group[gb[g].base + b] = g;
}

// splits[sbase[e] + j] = offset inside cover e of the first id >= j * WIN, j in [0, nwin(g)]
__global__ void k_splits(const uint32_t* ids, const uint64_t* off, const uint32_t* group, size_t n,
                         const uint32_t* nwin, const uint64_t* sbase, uint32_t* splits) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const uint32_t nw = nwin[group[e]];
    const uint64_t b = off[e], len = off[e + 1] - b;
    uint32_t* sp = splits + sbase[e];
    sp[0] = 0;
    for (uint32_t j = 1; j < nw; j++)
      sp[j] = (uint32_t)(lower_bound_dev<uint32_t>(ids, b, b + len, j << WIN_BITS) - b);
    sp[nw] = (uint32_t)len;
  }
}

__global__ void k_split_count(const uint32_t* group, size_t n, const uint32_t* nwin, uint64_t* cnt) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    cnt[e] = nwin[group[e]] + 1;
}

__global__ void k_el_init(const uint32_t* members, const uint64_t* off, size_t n, uint64_t* el) {
  for (size_t m = (size_t)blockIdx.x * blockDim.x + threadIdx.x; m < n; m += (size_t)gridDim.x * blockDim.x) {
    const uint32_t e = members[m];
    el[m] = ((off[e + 1] - off[e]) << 32) | m;
  }
}

// ---- vector stream ---------------------------------------------------------------------------------
// Panel p = (call g, id window w). Its stream is the concatenation, in member (corpus) order, of every
// cover's slice of ids in window w, as window-relative u16, each slice padded to a multiple of VEC
// with copies of its last id (min is idempotent, so padding never changes a result). Every VEC-id
// vector belongs to exactly one member: vmem[v] names it, so the kernel needs no segment search.

constexpr int VM_BLOCK = 1024;
#ifndef SYZ_VM_DEPTH
#define SYZ_VM_DEPTH 4
#endif
constexpr int VM_DEPTH = SYZ_VM_DEPTH;  // vectors per lane per pipelined batch (k_vec_min)

__device__ __forceinline__ void tab_min(uint32_t* tab, uint32_t id, uint32_t R) {
  if (tab[id] > R) atomicMin(&tab[id], R);
}

__device__ __forceinline__ void vec_update(uint32_t* tab, const uint4 q, uint32_t R) {
  tab_min(tab, q.x & 0xFFFF, R);
  tab_min(tab, q.x >> 16, R);
  tab_min(tab, q.y & 0xFFFF, R);
  tab_min(tab, q.y >> 16, R);
  tab_min(tab, q.z & 0xFFFF, R);
  tab_min(tab, q.z >> 16, R);
  tab_min(tab, q.w & 0xFFFF, R);
  tab_min(tab, q.w >> 16, R);
}

// One workgroup per work item (grid-stride over the items, so a launch can be held to part of the
// chip): min Go-sort rank per id of one window over a chunk of its stream. SIDE only names the
// small-class launch apart in profiles.
template <bool SIDE>
__global__ __launch_bounds__(VM_BLOCK) void k_vec_min(const VecWork* __restrict__ work, uint32_t nitems,
                                                      const uint4* __restrict__ ids16,
                                                      const uint32_t* __restrict__ vmem,
                                                      const uint32_t* __restrict__ rank_of_entry,
                                                      const uint64_t* __restrict__ gstart, uint32_t* sel_bits,
                                                      uint32_t* gtabs, const uint32_t* gtchunks, uint32_t* gtdone) {
  const uint32_t* __restrict__ rank_of_member = rank_of_entry;  // vmem names entries
  __shared__ uint32_t tab[WIN];
  __shared__ uint32_t bm[BM_WORDS];
  __shared__ uint32_t last;
  for (uint32_t wi = blockIdx.x; wi < nitems; wi += gridDim.x) {
    const VecWork w = work[wi];
    for (uint32_t i = threadIdx.x; i < w.nids; i += VM_BLOCK) tab[i] = RANK_NONE;
    __syncthreads();
    // The loop is bound by bytes in flight per CU (a dependent vmem -> rank gather per vector), so
    // it is software-pipelined: VM_DEPTH vectors per lane per batch, and the next batch's ids and
    // members are loaded while the current batch's ranks are gathered and applied.
    uint64_t v = w.vbeg + threadIdx.x;
    constexpr uint64_t STEP = (uint64_t)VM_DEPTH * VM_BLOCK;
    if (v + (VM_DEPTH - 1) * VM_BLOCK < w.vend) {
      uint4 q[VM_DEPTH];
      uint32_t m[VM_DEPTH];
#pragma unroll
      for (int j = 0; j < VM_DEPTH; j++) {
        q[j] = ids16[v + j * VM_BLOCK];
        m[j] = vmem[v + j * VM_BLOCK];
      }
      for (;;) {
        uint32_t r[VM_DEPTH];
#pragma unroll
        for (int j = 0; j < VM_DEPTH; j++) r[j] = rank_of_member[m[j]];
        const uint64_t vn = v + STEP;
        const bool more = vn + (VM_DEPTH - 1) * VM_BLOCK < w.vend;
        uint4 qn[VM_DEPTH];
        uint32_t mn[VM_DEPTH];
        if (more) {
#pragma unroll
          for (int j = 0; j < VM_DEPTH; j++) {
            qn[j] = ids16[vn + j * VM_BLOCK];
            mn[j] = vmem[vn + j * VM_BLOCK];
          }
        }
#pragma unroll
        for (int j = 0; j < VM_DEPTH; j++) vec_update(tab, q[j], r[j]);
        v = vn;
        if (!more) break;
#pragma unroll
        for (int j = 0; j < VM_DEPTH; j++) {
          q[j] = qn[j];
          m[j] = mn[j];
        }
      }
    }
    for (; v < w.vend; v += VM_BLOCK) vec_update(tab, ids16[v], rank_of_member[vmem[v]]);
    for (v = w.tbeg + threadIdx.x; v < w.tend; v += VM_BLOCK) vec_update(tab, ids16[v], rank_of_member[vmem[v]]);
    __syncthreads();
    if (w.gtab == RANK_NONE) {
      const uint64_t gb = gstart[w.g];
      emit_winners(tab, w.nids, gb, gstart[w.g + 1] - gb, bm, sel_bits);
    } else {
      uint32_t* gt = gtabs + (size_t)w.gtab * WIN;
      for (uint32_t i = threadIdx.x; i < w.nids; i += VM_BLOCK) {
        const uint32_t r = tab[i];
        if (r != RANK_NONE && __hip_atomic_load(&gt[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > r)
          __hip_atomic_fetch_min(&gt[i], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      // the last chunk of a split panel to arrive emits the shared table's winners. The table is
      // written and read only by agent-scope atomics, so the hand-off needs no cache fences: every
      // wave's atomics are complete (vmcnt) before the arrival is counted.
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        const uint32_t old = __hip_atomic_fetch_add(&gtdone[w.gtab], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = old + 1 == gtchunks[w.gtab];
      }
      __syncthreads();
      if (last) {
        const uint64_t gb = gstart[w.g];
        emit_winners<true>(gt, w.nids, gb, gstart[w.g + 1] - gb, bm, sel_bits);
      }
    }
    __syncthreads();
  }
}



// vcount[tbase[g] + w * N_g + mloc] = vectors of member m's slice in window w
__global__ void k_vcount(const uint32_t* members, const uint32_t* group, const uint64_t* gstart, size_t n,
                         const uint32_t* nwin, const uint64_t* tbase, const uint64_t* sbase, const uint32_t* splits,
                         uint32_t* vcount) {
  for (size_t m = (size_t)blockIdx.x * blockDim.x + threadIdx.x; m < n; m += (size_t)gridDim.x * blockDim.x) {
    const uint32_t e = members[m];
    const uint32_t g = group[e];
    const uint64_t ng = gstart[g + 1] - gstart[g], mloc = m - gstart[g];
    const uint32_t* sp = splits + sbase[e];
    for (uint32_t w = 0; w < nwin[g]; w++)
      vcount[tbase[g] + (uint64_t)w * ng + mloc] = (sp[w + 1] - sp[w] + VEC - 1) / VEC;
  }
}

// One wave per member: write its slices (window-relative u16, padded with the last id) and vmem.
__global__ __launch_bounds__(256) void k_vfill(const uint32_t* members, const uint32_t* group, const uint64_t* gstart,
                                               size_t n, const uint32_t* nwin, const uint64_t* tbase,
                                               const uint64_t* sbase, const uint32_t* splits, const uint64_t* off,
                                               const uint32_t* ids, const uint64_t* voff, uint16_t* ids16,
                                               uint32_t* vmem) {
  const size_t m = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (m >= n) return;
  const unsigned lane = __lane_id();
  const uint32_t e = members[m];
  const uint32_t g = group[e];
  const uint64_t ng = gstart[g + 1] - gstart[g], mloc = m - gstart[g];
  const uint32_t* sp = splits + sbase[e];
  const uint32_t* src = ids + off[e];
  for (uint32_t w = 0; w < nwin[g]; w++) {
    const uint32_t s0 = sp[w], s1 = sp[w + 1];
    if (s1 == s0) continue;
    const uint64_t vo = voff[tbase[g] + (uint64_t)w * ng + mloc];
    const uint32_t len = s1 - s0, padded = (len + VEC - 1) / VEC * VEC;
    const uint32_t wb = w << WIN_BITS;
    for (uint32_t k = lane; k < padded; k += 64)
      ids16[vo * VEC + k] = (uint16_t)(src[s0 + min(k, len - 1)] - wb);
    for (uint32_t k = lane; k < padded / VEC; k += 64) vmem[vo + k] = e;  // the vector's entry
  }
}

__global__ void k_gather_u64(const uint64_t* src, const uint64_t* idx, size_t n, uint64_t* dst) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}

// ---- the store object ----------------------------------------------------------------------------------

// Orders this rank's work items and uploads them: big call groups (sorted by the global rounds)
// first, small ones (LDS packs, sorted on the side stream) after, so each class's Minimize runs as
// soon as its own sort is done; largest first inside a class, so the tail of the grid is short.
void corpus_upload_work(Corpus& K, hipStream_t s) {
  const std::vector<uint64_t>& hstart = K.hstart;
  auto is_big = [&](uint32_t g) { return hstart[g + 1] - hstart[g] > GS_T_SEG; };
  std::stable_sort(K.hwork.begin(), K.hwork.end(), [&](const VecWork& x, const VecWork& y) {
    const bool bx = is_big(x.g), by = is_big(y.g);
    if (bx != by) return bx;
    return x.vend - x.vbeg > y.vend - y.vbeg;
  });
  K.nbig_work = 0;
  K.big_vecs = 0;
  while (K.nbig_work < K.hwork.size() && is_big(K.hwork[K.nbig_work].g))
    K.big_vecs += K.hwork[K.nbig_work].vend - K.hwork[K.nbig_work].vbeg, K.nbig_work++;
  K.work.ensure(K.hwork.size());
  if (!K.hwork.empty())
    SYZ_HIP(hipMemcpyAsync(K.work.p, K.hwork.data(), K.hwork.size() * sizeof(VecWork), hipMemcpyHostToDevice, s));
  // work items per shared table: the vec_min chunk that brings the count to it emits the table
  std::vector<uint32_t> hch(K.ngtabs, 0);
  for (const VecWork& w : K.hwork)
    if (w.gtab != RANK_NONE) hch[w.gtab]++;
  if (K.ngtabs) SYZ_HIP(hipMemcpyAsync(K.gtchunks.p, hch.data(), K.ngtabs * 4, hipMemcpyHostToDevice, s));
  SYZ_HIP(hipStreamSynchronize(s));  // hch / hwork are host temporaries
}

// Key-space sharding: call group g's id windows are dealt into nparts[g] parts by
// vector count (longest-processing-time, identical on every rank) and this store keeps part[g].
// The partial selections of one group on its ranks OR together to the full selection, because an
// input is kept iff SOME of its PCs first occurs at it.
void corpus_set_parts(Corpus& K, const uint16_t* part, const uint16_t* nparts, const uint8_t* count_hist,
                             hipStream_t s) {
  const uint32_t G = K.G;
  std::vector<int> keep_part(G, -1);  // -1: whole group
  for (uint32_t g = 0; g < G; g++) {
    const uint32_t k = nparts ? nparts[g] : 1;
    if (k > 1) {
      if (!part || part[g] >= k) fail(SYZGPU_EINVAL, "part[g] must be < nparts[g]");
      keep_part[g] = part[g];
    }
  }
  // vectors per (group, window), then windows -> parts per split group
  std::map<std::pair<uint32_t, uint32_t>, uint64_t> wvec;
  for (const VecWork& w : K.hwork_all)
    if (keep_part[w.g] >= 0) wvec[{w.g, w.win}] += w.vend - w.vbeg;
  std::map<std::pair<uint32_t, uint32_t>, int> wpart;
  for (uint32_t g = 0; g < G; g++) {
    if (keep_part[g] < 0) continue;
    std::vector<std::pair<uint64_t, uint32_t>> ws;  // (vectors, window)
    for (auto it = wvec.lower_bound({g, 0}); it != wvec.end() && it->first.first == g; ++it)
      ws.push_back({it->second, it->first.second});
    std::stable_sort(ws.begin(), ws.end(), [](const auto& a, const auto& b) {
      return a.first != b.first ? a.first > b.first : a.second < b.second;
    });
    std::vector<uint64_t> load(nparts[g], 0);
    for (const auto& x : ws) {
      const int p = (int)(std::min_element(load.begin(), load.end()) - load.begin());
      load[p] += x.first;
      wpart[{g, x.second}] = p;
    }
  }
  K.hwork.clear();
  for (const VecWork& w : K.hwork_all)
    if (keep_part[w.g] < 0 || wpart[{w.g, w.win}] == keep_part[w.g]) K.hwork.push_back(w);
  K.has_count_hist = count_hist != nullptr;
  if (count_hist) {
    K.count_hist.alloc(G);
    SYZ_HIP(hipMemcpyAsync(K.count_hist.p, count_hist, G, hipMemcpyHostToDevice, s));
  }
  corpus_upload_work(K, s);
}

Corpus* corpus_create_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, const uint16_t* prog_len,
                          size_t n, uint32_t G, hipStream_t s) {
  Context& c = ctx();
  if (G == 0 || G > MAX_GROUPS) fail(SYZGPU_EINVAL, "ngroups out of range (1..4096)");
  if (n >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "too many corpus entries");
  std::unique_ptr<Corpus> cp(new Corpus());
  Corpus& K = *cp;
  K.n = n;
  K.G = G;
  Scratch& sc = c.scratch;
  // host copy of the offsets (for sizes and the per-cover sort launch)
  std::vector<uint64_t> hoff(n + 1);
  SYZ_HIP(hipMemcpyAsync(hoff.data(), off, (n + 1) * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (hoff[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
  K.total_pcs = hoff[n];
  if (K.total_pcs >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "more than 2^32 PCs in one store");
  K.off.alloc(n + 1);
  K.group.alloc(n);
  K.prog_len.alloc(n);
  K.members.alloc(n);
  K.gstart.alloc(G + 1);
  uint32_t* ids = sc.get<uint32_t>("cs_ids", K.total_pcs + 1);
  SYZ_HIP(hipMemcpyAsync(K.off.p, off, (n + 1) * 8, hipMemcpyDeviceToDevice, s));
  if (n) SYZ_HIP(hipMemcpyAsync(K.group.p, group, n * 4, hipMemcpyDeviceToDevice, s));
  if (n && prog_len) SYZ_HIP(hipMemcpyAsync(K.prog_len.p, prog_len, n * 2, hipMemcpyDeviceToDevice, s));
  if (n && !prog_len) SYZ_HIP(hipMemsetAsync(K.prog_len.p, 0, n * 2, s));
  // 1. group partition
  const uint32_t pw = grp_pw(n, G);
  const uint32_t nchunks = (uint32_t)((n + pw - 1) / pw);
  int* err = sc.get<int>("cs_err", 2);
  uint32_t* cnt = sc.get<uint32_t>("mz_cnt", (size_t)G * nchunks + 1);
  uint64_t* cnt_scan = sc.get<uint64_t>("mz_cnt_scan", (size_t)G * nchunks + 1);
  uint64_t* gpcs = sc.get<uint64_t>("mz_gpcs", G + 1);
  uint64_t* el = sc.get<uint64_t>("mz_el", n + 1);
  SYZ_HIP(hipMemsetAsync(err, 0, 8, s));
  SYZ_HIP(hipMemsetAsync(cnt, 0, ((size_t)G * nchunks + 1) * 4, s));
  SYZ_HIP(hipMemsetAsync(gpcs, 0, (G + 1) * 8, s));
  if (n) {
    const unsigned wg = (unsigned)(((size_t)nchunks * 64 + 255) / 256);
    k_grp_count<<<wg, 256, 4 * G * 4, s>>>(group, n, G, nchunks, pw, cnt, err);
    SYZ_LAUNCHED();
    k_grp_sumlen<<<grid_for(n, 256, 2048), 256, G * 8, s>>>(group, off, n, G, gpcs);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(cnt, cnt_scan, (size_t)G * nchunks, s);
  k_grp_starts<<<grid_for(G + 1, 256, 1024), 256, 0, s>>>(cnt_scan, G, nchunks, n, K.gstart.p);
  SYZ_LAUNCHED();
  if (n) {
    const unsigned wg = (unsigned)(((size_t)nchunks * 64 + 255) / 256);
    k_grp_scatter<<<wg, 256, 4 * G * 4, s>>>(group, off, n, G, nchunks, pw, cnt_scan, K.members.p, el, PartOut{});
    SYZ_LAUNCHED();
  }
  K.member_of.alloc(n);
  if (n) {
    k_invert<<<grid_for(n, 256, 4096), 256, 0, s>>>(K.members.p, n, K.member_of.p);
    SYZ_LAUNCHED();
  }
  std::vector<uint64_t> hstart(G + 1), hpcs(G);
  int herr[2];
  SYZ_HIP(hipMemcpyAsync(hstart.data(), K.gstart.p, (G + 1) * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hpcs.data(), gpcs, G * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(herr, err, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (herr[0]) fail(SYZGPU_EINVAL, "group id >= ngroups");
  // 2. hash buckets per call (<= HT_ROUND_ITEMS occurrences expected per bucket)
  std::vector<GBucket> hgb(G);
  std::vector<Chunk> hch;
  uint32_t nbuckets = 0;
  for (uint32_t g = 0; g < G; g++) {
    const uint64_t np = hpcs[g];
    uint32_t bits = 0;
    while (bits < 24 && ((uint64_t)HT_ROUND_ITEMS << bits) < np) bits++;
    hgb[g] = GBucket{nbuckets, bits};
    nbuckets += 1u << bits;
    const uint64_t ng = hstart[g + 1] - hstart[g];
    if (ng == 0) continue;
    const uint64_t avg = std::max<uint64_t>(1, np / ng);
    const uint64_t target = std::max<uint64_t>(32768, 4ull << bits);
    const uint32_t per = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ng, target / avg));
    for (uint64_t m = hstart[g]; m < hstart[g + 1]; m += per)
      hch.push_back(Chunk{g, (uint32_t)m, (uint32_t)std::min<uint64_t>(hstart[g + 1], m + per), 0});
  }
  GBucket* dgb = sc.get<GBucket>("mz_gb", G);
  Chunk* dch = sc.get<Chunk>("mz_chunks", hch.size() + 1);
  uint32_t* bcount = sc.get<uint32_t>("mz_bcount", nbuckets + 1);
  uint64_t* boff = sc.get<uint64_t>("mz_boff", nbuckets + 1);
  uint32_t* bcursor = sc.get<uint32_t>("mz_bcursor", nbuckets + 1);
  uint32_t* bgroup = sc.get<uint32_t>("cs_bgroup", nbuckets + 1);
  uint32_t* dcount = sc.get<uint32_t>("cs_dcount", nbuckets + 1);
  uint64_t* dscan = sc.get<uint64_t>("cs_dscan", nbuckets + 1);
  uint2* items = sc.get<uint2>("mz_items", K.total_pcs + 1);
  SYZ_HIP(hipMemcpyAsync(dgb, hgb.data(), G * sizeof(GBucket), hipMemcpyHostToDevice, s));
  if (!hch.empty()) SYZ_HIP(hipMemcpyAsync(dch, hch.data(), hch.size() * sizeof(Chunk), hipMemcpyHostToDevice, s));
  SYZ_HIP(hipMemsetAsync(bcount, 0, (nbuckets + 1) * 4, s));
  SYZ_HIP(hipMemsetAsync(bcursor, 0, (nbuckets + 1) * 4, s));
  k_bucket_group<<<std::min<uint32_t>(G, 1024), 256, 0, s>>>(dgb, G, bgroup);
  SYZ_LAUNCHED();
  if (!hch.empty()) {
    k_bucket_count<<<(unsigned)hch.size(), BK_BLOCK, 0, s>>>(dch, dgb, K.members.p, off, pcs, bcount);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(bcount, boff, nbuckets, s);
  if (!hch.empty()) {
    k_bucket_scatter_pos<<<(unsigned)hch.size(), BK_BLOCK, 0, s>>>(dch, dgb, K.members.p, off, pcs, boff, bcursor,
                                                                   items);
    SYZ_LAUNCHED();
  }
  // 3. dense ids: count distinct per bucket, scan, assign
  const unsigned hb = std::min<uint32_t>(std::max<uint32_t>(nbuckets, 1), 65536);
  k_bucket_ids<<<hb, HT_BLOCK, 0, s>>>(0, boff, nbuckets, items, dcount, nullptr, bgroup, dgb, nullptr, nullptr,
                                       nullptr, err);
  SYZ_LAUNCHED();
  exclusive_scan_u32(dcount, dscan, nbuckets, s);
  std::vector<uint64_t> hds(nbuckets + 1);
  SYZ_HIP(hipMemcpyAsync(hds.data(), dscan, (nbuckets + 1) * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(herr, err, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (herr[0] & 4) fail(SYZGPU_EINTERNAL, "coverstore: hash bucket overflow");
  std::vector<uint64_t> hgdict(G + 1);
  std::vector<uint32_t> hnwin(G);
  for (uint32_t g = 0; g < G; g++) {
    const uint64_t p_g = hds[hgb[g].base + (1u << hgb[g].bits)] - hds[hgb[g].base];
    hgdict[g] = hds[hgb[g].base];
    hnwin[g] = (uint32_t)std::max<uint64_t>(1, (p_g + WIN - 1) / WIN);
  }
  hgdict[G] = hds[nbuckets];
  K.total_ids = hds[nbuckets];
  K.hnids.assign(G, 0);
  for (uint32_t g = 0; g < G; g++) K.hnids[g] = hgdict[g + 1] - hgdict[g];
  K.dict.alloc(K.total_ids);
  K.gdict.alloc(G + 1);
  K.nwin.alloc(G);
  SYZ_HIP(hipMemcpyAsync(K.gdict.p, hgdict.data(), (G + 1) * 8, hipMemcpyHostToDevice, s));
  SYZ_HIP(hipMemcpyAsync(K.nwin.p, hnwin.data(), G * 4, hipMemcpyHostToDevice, s));
  k_bucket_ids<<<hb, HT_BLOCK, 0, s>>>(1, boff, nbuckets, items, dcount, dscan, bgroup, dgb, K.gdict.p, K.dict.p,
                                       ids, err);
  SYZ_LAUNCHED();
  // 4. every cover as a sorted id list (ids are unique within a cover iff its PCs are)
  uint64_t* clen = sc.get<uint64_t>("cs_clen", n + 1);
  canonicalize_batch_dev(ids, K.off.p, hoff.data(), n, clen, s);
  std::vector<uint64_t> hclen(n);
  if (n) SYZ_HIP(hipMemcpyAsync(hclen.data(), clen, n * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  for (size_t e = 0; e < n; e++)
    if (hclen[e] != hoff[e + 1] - hoff[e])
      fail(SYZGPU_EINVAL, "coverstore needs canonical covers (sorted, duplicate-free); Canonicalize first");
  // 5. window splits (ingest intermediates)
  uint64_t* scount = sc.get<uint64_t>("cs_scount", n + 1);
  uint64_t* sbase = sc.get<uint64_t>("cs_sbase", n + 1);
  if (n) {
    k_split_count<<<grid_for(n, 256, 4096), 256, 0, s>>>(K.group.p, n, K.nwin.p, scount);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u64(scount, sbase, n, s);
  uint64_t hsplits = 0;
  SYZ_HIP(hipMemcpyAsync(&hsplits, sbase + n, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  uint32_t* splits = sc.get<uint32_t>("cs_splits", hsplits + 1);
  if (n) {
    k_splits<<<grid_for(n, 256, 8192), 256, 0, s>>>(ids, K.off.p, K.group.p, n, K.nwin.p, sbase, splits);
    SYZ_LAUNCHED();
  }
  // 6. vector stream: panel-major (call, window), member order inside a panel
  std::vector<uint64_t> htbase(G + 1, 0);
  for (uint32_t g = 0; g < G; g++) htbase[g + 1] = htbase[g] + (uint64_t)hnwin[g] * (hstart[g + 1] - hstart[g]);
  const uint64_t T = htbase[G];
  uint64_t* tbase = sc.get<uint64_t>("cs_tbase", G + 1);
  uint32_t* vcount = sc.get<uint32_t>("cs_vcount", T + 1);
  uint64_t* voff = sc.get<uint64_t>("cs_voff", T + 1);
  SYZ_HIP(hipMemcpyAsync(tbase, htbase.data(), (G + 1) * 8, hipMemcpyHostToDevice, s));
  if (n) {
    k_vcount<<<grid_for(n, 256, 8192), 256, 0, s>>>(K.members.p, K.group.p, K.gstart.p, n, K.nwin.p, tbase, sbase,
                                                     splits, vcount);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(vcount, voff, T, s);
  // panel boundaries: voff at tbase[g] + w * N_g for every (g, w), plus the total
  std::vector<uint64_t> hpidx;
  for (uint32_t g = 0; g < G; g++)
    for (uint32_t w = 0; w < hnwin[g]; w++) hpidx.push_back(htbase[g] + (uint64_t)w * (hstart[g + 1] - hstart[g]));
  hpidx.push_back(T);
  uint64_t* dpidx = sc.get<uint64_t>("cs_pidx", hpidx.size());
  uint64_t* dpv = sc.get<uint64_t>("cs_pv", hpidx.size());
  SYZ_HIP(hipMemcpyAsync(dpidx, hpidx.data(), hpidx.size() * 8, hipMemcpyHostToDevice, s));
  k_gather_u64<<<grid_for(hpidx.size(), 256, 1024), 256, 0, s>>>(voff, dpidx, hpidx.size(), dpv);
  SYZ_LAUNCHED();
  std::vector<uint64_t> hpv(hpidx.size());
  SYZ_HIP(hipMemcpyAsync(hpv.data(), dpv, hpidx.size() * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  K.total_vecs = hpv.back();
  K.ids16.alloc(K.total_vecs * VEC);
  K.vmem.alloc(K.total_vecs);
  if (n) {
    k_vfill<<<(unsigned)((n * 64 + 255) / 256), 256, 0, s>>>(K.members.p, K.group.p, K.gstart.p, n, K.nwin.p, tbase,
                                                            sbase, splits, K.off.p, ids, voff, K.ids16.p, K.vmem.p);
    SYZ_LAUNCHED();
  }
  // 7. work items: chunks of <= CHUNK_VECS vectors of one panel; a split panel merges through a
  // global table. Largest first, so the tail of the grid is short.
  K.ngtabs = 0;
  // Work-item size: about one item per CU for each class (a workgroup fills its CU's LDS, so every
  // item pays a pipeline fill, a table init and an emit with HBM idle; measured at config 4: 64K-vector
  // items 0.235 ms, 196K 0.180 ms, 256K 0.214 ms as the tail grows). total/300, in [16K, 256K].
  uint64_t chunk_vecs = std::min<uint64_t>(
      CHUNK_VECS_MAX, std::max<uint64_t>(CHUNK_VECS_MIN, (K.total_vecs / 300 + 4095) / 4096 * 4096));
  if (const char* cv = getenv("SYZGPU_CHUNK_VECS")) chunk_vecs = std::max<uint64_t>(1, strtoull(cv, nullptr, 10));
  K.chunk_vecs = chunk_vecs;
  size_t pi = 0;
  for (uint32_t g = 0; g < G; g++) {
    const uint64_t p_g = hgdict[g + 1] - hgdict[g];
    for (uint32_t w = 0; w < hnwin[g]; w++, pi++) {
      const uint64_t vb = hpv[pi], ve = hpv[pi + 1];
      if (ve == vb) continue;
      const uint32_t nids = (uint32_t)std::min<uint64_t>(WIN, p_g - (uint64_t)w * WIN);
      const uint64_t nch = (ve - vb + chunk_vecs - 1) / chunk_vecs;
      uint32_t gt = RANK_NONE;
      if (nch > 1) {
        gt = K.ngtabs++;
      }
      const uint64_t per = (ve - vb + nch - 1) / nch;
      for (uint64_t v = vb; v < ve; v += per) K.hwork.push_back(VecWork{g, nids, v, std::min(ve, v + per), gt, w});
    }
  }
  K.hstart = hstart;
  for (uint32_t g = 0; g < G; g++)
    if (hstart[g + 1] - hstart[g] > GS_T_SEG) {
      K.big_entries += hstart[g + 1] - hstart[g];
      K.big_pcs += hpcs[g];
    }
  K.hwork_all = K.hwork;
  for (const VecWork& w : K.hwork_all)
    if (hstart[w.g + 1] - hstart[w.g] > GS_T_SEG) K.big_vecs_all += w.vend - w.vbeg;
  K.gtabs.alloc((size_t)K.ngtabs * WIN);
  K.gtchunks.alloc(K.ngtabs);
  K.gtdone.alloc(K.ngtabs);
  corpus_upload_work(K, s);
  SYZ_HIP(hipMemcpyAsync(herr, err, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (herr[0] & 4) fail(SYZGPU_EINTERNAL, "coverstore: hash bucket overflow");
  K.hstart = hstart;
  gosort_plan(K.gsplan, hstart, G, s);
  K.el0.alloc(n);
  if (n) {
    k_el_init<<<grid_for(n, 256, 8192), 256, 0, s>>>(K.members.p, K.off.p, n, K.el0.p);
    SYZ_LAUNCHED();
  }
  if (n && prog_len) {  // len(p.Calls) > C is rejected per call without a device round trip
    std::vector<uint16_t> hl(n);
    SYZ_HIP(hipMemcpyAsync(hl.data(), prog_len, n * 2, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    K.max_prog_len = *std::max_element(hl.begin(), hl.end());
  }
  return cp.release();
}


// The group partition of K's current entries (K.off, K.group, K.n): members, gstart, member_of, the
// Go-sort keys el0, hstart and the Go-sort plan; hpcs = PCs per call. The incremental index
// (corpus_inc.hip) re-runs it after an append or a keep; it is corpus_create_dev's step 1.
void corpus_partition(Corpus& K, std::vector<uint64_t>& hpcs, hipStream_t s) {
  Scratch& sc = ctx().scratch;
  const size_t n = K.n;
  const uint32_t G = K.G;
  const uint32_t pw = grp_pw(n, G);
  const uint32_t nchunks = (uint32_t)((n + pw - 1) / pw);
  int* err = sc.get<int>("cs_err", 2);
  uint32_t* cnt = sc.get<uint32_t>("mz_cnt", (size_t)G * nchunks + 1);
  uint64_t* cnt_scan = sc.get<uint64_t>("mz_cnt_scan", (size_t)G * nchunks + 1);
  uint64_t* gpcs = sc.get<uint64_t>("mz_gpcs", G + 1);
  K.members.ensure(n + 1);
  K.member_of.ensure(n + 1);
  K.el0.ensure(n + 1);
  if (!K.gstart.p) K.gstart.alloc(G + 1);
  SYZ_HIP(hipMemsetAsync(err, 0, 8, s));
  SYZ_HIP(hipMemsetAsync(cnt, 0, ((size_t)G * nchunks + 1) * 4, s));
  SYZ_HIP(hipMemsetAsync(gpcs, 0, (G + 1) * 8, s));
  if (n) {
    const unsigned wg = (unsigned)(((size_t)nchunks * 64 + 255) / 256);
    k_grp_count<<<wg, 256, 4 * G * 4, s>>>(K.group.p, n, G, nchunks, pw, cnt, err);
    SYZ_LAUNCHED();
    k_grp_sumlen<<<grid_for(n, 256, 2048), 256, G * 8, s>>>(K.group.p, K.off.p, n, G, gpcs);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u32(cnt, cnt_scan, (size_t)G * nchunks, s);
  k_grp_starts<<<grid_for(G + 1, 256, 1024), 256, 0, s>>>(cnt_scan, G, nchunks, n, K.gstart.p);
  SYZ_LAUNCHED();
  if (n) {
    const unsigned wg = (unsigned)(((size_t)nchunks * 64 + 255) / 256);
    k_grp_scatter<<<wg, 256, 4 * G * 4, s>>>(K.group.p, K.off.p, n, G, nchunks, pw, cnt_scan, K.members.p, K.el0.p,
                                                PartOut{});
    SYZ_LAUNCHED();
    k_invert<<<grid_for(n, 256, 4096), 256, 0, s>>>(K.members.p, n, K.member_of.p);
    SYZ_LAUNCHED();
  }
  std::vector<uint64_t> hstart(G + 1);
  hpcs.assign(G, 0);
  int herr[2];
  SYZ_HIP(hipMemcpyAsync(hstart.data(), K.gstart.p, (G + 1) * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(hpcs.data(), gpcs, G * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(herr, err, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (herr[0]) fail(SYZGPU_EINVAL, "group id >= ngroups");
  K.hstart = hstart;
  K.big_entries = K.big_pcs = 0;
  for (uint32_t g = 0; g < G; g++)
    if (hstart[g + 1] - hstart[g] > GS_T_SEG) {
      K.big_entries += hstart[g + 1] - hstart[g];
      K.big_pcs += hpcs[g];
    }
  gosort_plan(K.gsplan, hstart, G, s);
}

// minimizeCorpus, first half: the Go-sort ranks and the first-occurrence pass into the rank bitmap
// (this rank's key parts only, see corpus_set_parts).
void corpus_minimize_begin(Corpus& K, hipStream_t s) {
  Context& c = ctx();
  Scratch& sc = c.scratch;
  const size_t n = K.n;
  int* err = sc.get<int>("mz_err", 2);
  uint64_t* el = sc.get<uint64_t>("mz_el", n + 1);
  uint32_t* perm = sc.get<uint32_t>("mz_perm", n + 1);
  K.rom.ensure(n + 1);
  K.eor.ensure(n + 1);
  K.sel_bits.ensure(n / 32 + 2);
  uint32_t* rank_of_entry = K.rom.p;  // (the index's vectors name entries)
  uint32_t* ent_of_rank = K.eor.p;
  SYZ_HIP(hipMemsetAsync(err, 0, 2 * sizeof(int), s));
  uint32_t* sel_bits = K.sel_bits.p;
  SYZ_HIP(hipMemsetAsync(sel_bits, 0, (n / 32 + 2) * 4, s));
  if (K.ngtabs) {
    SYZ_HIP(hipMemsetAsync(K.gtabs.p, 0xFF, (size_t)K.ngtabs * WIN * 4, s));
    SYZ_HIP(hipMemsetAsync(K.gtdone.p, 0, (size_t)K.ngtabs * 4, s));
  }
  {
    ProfScope ps("el_init", s, (uint64_t)n * 20);
    if (n) {
      // the sort keys (len(cov) << 32 | member) are part of the stored corpus (built at ingest),
      // copied into the sort buffer, which the sort permutes in place
      SYZ_HIP(hipMemcpyAsync(el, K.el0.p, n * 8, hipMemcpyDeviceToDevice, s));
    }
  }
  // ranks + Minimize per class, each right after its own sort: the small call groups' on the side
  // stream while the big ones still run their global rounds
  const GosortPlan& P = K.gsplan;
  // the small class runs beside the big class's latency-bound global rounds: it is held to part of
  // the chip (its workgroups fill a CU's LDS), so the rounds keep CUs to run on
  static const unsigned side_cus = dev_env("SYZGPU_SIDE_CUS") ? (unsigned)atoi(dev_env("SYZGPU_SIDE_CUS")) : 128u;
  auto vec_min = [&](hipStream_t q, size_t first, size_t count, bool side) {
    if (!count) return;
    const unsigned grid = (unsigned)std::min<size_t>(count, side ? side_cus : (1u << 20));
    auto* k = side ? k_vec_min<true> : k_vec_min<false>;
    k<<<grid, VM_BLOCK, 0, q>>>(K.work.p + first, (uint32_t)count, reinterpret_cast<const uint4*>(K.ids16.p),
                                K.vmem.p, rank_of_entry, K.gstart.p, sel_bits, K.gtabs.p, K.gtchunks.p,
                                K.gtdone.p);
    SYZ_LAUNCHED();
  };
  auto small_done = [&](hipStream_t q) {
    if (P.npacks) {  // a pack holds at most GS_T_SEG elements
      k_ranks_ranges_ent<<<dim3(GS_T_SEG / 1024, P.npacks), 256, 0, q>>>(
          el, perm, reinterpret_cast<const uint4*>(P.packs), K.members.p, rank_of_entry, ent_of_rank);
      SYZ_LAUNCHED();
    }
    ProfScope ps("vec_min_small", q, (K.total_pcs - K.big_pcs) * 4 + (n - K.big_entries) * 10);
    vec_min(q, K.nbig_work, K.hwork.size() - K.nbig_work, true);
  };
  auto big_done = [&](hipStream_t q) {
    if (P.nbig) {
      const unsigned gx = (unsigned)std::min<uint64_t>(std::max<uint64_t>(1, P.big_max / 2048), 256);
      k_ranks_ranges_ent<<<dim3(gx, P.nbig), 256, 0, q>>>(el, perm, reinterpret_cast<const uint4*>(P.big),
                                                         K.members.p, rank_of_entry, ent_of_rank);
      SYZ_LAUNCHED();
    }
    // algorithmic bytes of this rank's share: the PCs of its key parts (in proportion to their id
    // vectors) plus offsets and group id of every big-group entry
    const double share = K.big_vecs_all ? (double)K.big_vecs / (double)K.big_vecs_all : 0.0;
    ProfScope ps("vec_min", q, (uint64_t)(K.big_pcs * 4 * share) + K.big_entries * 10);
    vec_min(q, 0, K.nbig_work, false);
  };
  if (n) gosort_run(el, perm, n, P, s, small_done, big_done);
  K.begun = true;
}

// Selection of the listed call groups as one byte per group-relative rank, at byte offsets boff[j]
// of buf (export), or OR-ed back into the rank bitmap (import): the cross-rank exchange of split
// groups. blockIdx.y = list index.
__global__ void k_sel_xchg(uint32_t* sel_bits, const uint64_t* gstart, const uint32_t* groups, const uint64_t* boff,
                           uint8_t* buf, int import) {
  const uint32_t g = groups[blockIdx.y];
  const uint64_t gb = gstart[g], ng = gstart[g + 1] - gb, o = boff[blockIdx.y];
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < ng; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t R = gb + r;
    if (import) {
      if (buf[o + r]) atomicOr(&sel_bits[R >> 5], 1u << (R & 31));
    } else {
      buf[o + r] = (uint8_t)((sel_bits[R >> 5] >> (R & 31)) & 1u);
    }
  }
}

void corpus_sel_xchg(Corpus& K, const uint32_t* groups, const uint64_t* offsets, uint32_t ng, uint8_t* buf,
                     int import, hipStream_t s) {
  if (!ng) return;
  if (!groups || !offsets || !buf) fail(SYZGPU_EINVAL, "null pointer");
  uint64_t maxn = 0;
  for (uint32_t j = 0; j < ng; j++) {
    if (groups[j] >= K.G) fail(SYZGPU_EINVAL, "group id >= ngroups");
    maxn = std::max<uint64_t>(maxn, K.hstart[groups[j] + 1] - K.hstart[groups[j]]);
  }
  if (!K.begun) fail(SYZGPU_EINVAL, "corpus: minimize_begin first");
  uint32_t* sel_bits = K.sel_bits.p;
  // the exchange list is the same on every step: uploaded once per distinct list, so the step itself
  // never waits on the host
  std::vector<uint64_t> key(groups, groups + ng);
  key.insert(key.end(), offsets, offsets + ng);
  if (key != K.xkey) {
    K.xg.alloc(ng);
    K.xo.alloc(ng);
    SYZ_HIP(hipMemcpyAsync(K.xg.p, groups, ng * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(K.xo.p, offsets, ng * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipStreamSynchronize(s));  // caller-owned host memory
    K.xkey = key;
  }
  const unsigned gx = (unsigned)std::min<uint64_t>(std::max<uint64_t>(1, (maxn + 1023) / 1024), 1024);
  k_sel_xchg<<<dim3(gx, ng), 256, 0, s>>>(sel_bits, K.gstart.p, K.xg.p, K.xo.p, buf, import);
  SYZ_LAUNCHED();
}

// minimizeCorpus, second half: kept flags per entry and the length histogram of the kept programs
// of the groups this rank counts.
void corpus_minimize_end(Corpus& K, int32_t C, uint8_t* selected, int64_t* len_hist, hipStream_t s) {
  if (len_hist && (int64_t)K.max_prog_len > (int64_t)C)
    fail(SYZGPU_EINVAL, "len(p.Calls) > C (prog/prio.go:148 would panic)");
  Scratch& sc = ctx().scratch;
  const size_t n = K.n;
  int* err = sc.get<int>("mz_err", 2);
  if (!K.begun) fail(SYZGPU_EINVAL, "corpus: minimize_begin first");
  uint32_t* rank_of_entry = K.rom.p;
  uint32_t* sel_bits = K.sel_bits.p;
  if (len_hist) SYZ_HIP(hipMemsetAsync(len_hist, 0, (size_t)(C + 1) * 8, s));
  ProfScope ps("select_out", s, (uint64_t)n * 8);
  if (n) {
    k_select_store<<<grid_for(n, 256, 512), 256, len_hist ? (size_t)(C + 1) * 8 : 0, s>>>(
        sel_bits, rank_of_entry, n, len_hist ? K.prog_len.p : nullptr, K.group.p,
        K.has_count_hist ? K.count_hist.p : nullptr, C, selected, len_hist, err);
    SYZ_LAUNCHED();
  }
}

void corpus_minimize_dev(Corpus& K, int32_t C, uint8_t* selected, int64_t* len_hist, hipStream_t s) {
  if (len_hist && (int64_t)K.max_prog_len > (int64_t)C)
    fail(SYZGPU_EINVAL, "len(p.Calls) > C (prog/prio.go:148 would panic)");
  corpus_minimize_begin(K, s);
  corpus_minimize_end(K, C, selected, len_hist, s);
}

}  // namespace syz


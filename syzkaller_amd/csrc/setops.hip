// Coverage set algebra on sorted uint32 PC lists — cover/cover.go:28-102.
//
// foreach (cover.go:81-102) walks two sorted lists with two pointers that both advance on equal
// values. On sorted inputs that is a multiset merge: for a value v occurring ca times in a and cb
// times in b, the first min(ca, cb) copies are paired. So each element's fate is a local function of
// (its rank inside its run of equal values, the count of v in the other list):
//   Difference            keep a[x] iff rank_a >= cb
//   Intersection          keep a[x] iff rank_a <  cb
//   Union                 keep every a[x]; keep b[y] iff rank_b >= ca
//   SymmetricDifference   keep a[x] iff rank_a >= cb; keep b[y] iff rank_b >= ca
// and 0xFFFFFFFF (the sentinel, cover.go:17) is never emitted. Outputs are placed by prefix sums
// of the keep flags — one lane per element (a wave per pair), no sequential merge.
//
// Canonicalize (cover.go:28-40): per-cover sort in LDS (bitonic, up to 16384 PCs = the kcov limit,
// executor.cc:48) or a global bitonic network beyond, then unique with last = sentinel.
#include <algorithm>

#include "pipeline.hpp"

namespace syz {

// ---- batched set operations -------------------------------------------------------------------


// Work unit: a segment of <= SO_SEG consecutive elements of one pair's list (a pair of n elements has
// ceil(n / SO_SEG) segments; segoff = their exclusive scan over the pairs), one wave per segment
// (grid-stride): the pair is found once per segment, so an element costs only its searches inside
// the other list, whose few lines the wave's lanes share through L1; long lists still spread over
// many waves.
constexpr uint64_t SO_SEG = 1024;

__global__ void k_setop_nseg(const uint64_t* off, uint32_t npairs, uint32_t* nseg) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += gridDim.x * blockDim.x)
    nseg[p] = (uint32_t)((off[p + 1] - off[p] + SO_SEG - 1) / SO_SEG);
}

// segment sid -> (pair, element range)
__device__ __forceinline__ uint32_t seg_pair(const uint64_t* segoff, uint32_t npairs, uint64_t sid, const uint64_t* off,
                                             uint64_t* x0, uint64_t* x1) {
  const uint32_t p = (uint32_t)upper_bound_dev<uint64_t>(segoff, 0, npairs + 1, sid) - 1;
  *x0 = off[p] + (sid - segoff[p]) * SO_SEG;
  *x1 = min(off[p + 1], *x0 + SO_SEG);
  return p;
}

// side 0 classifies a-elements against b, side 1 b-elements against a.
__global__ __launch_bounds__(256) void k_setop_classify(int op, int side, const uint32_t* a, const uint64_t* aoff,
                                                        const uint32_t* b, const uint64_t* boff, uint32_t npairs,
                                                        const uint64_t* segoff, uint8_t* keep, int* err) {
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6, nseg = segoff[npairs];
  for (uint64_t sid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; sid < nseg; sid += waves) {
    uint64_t x0, x1;
    const uint32_t p = seg_pair(segoff, npairs, sid, aoff, &x0, &x1);
    const uint64_t beg = aoff[p], end = aoff[p + 1], b0 = boff[p], b1 = boff[p + 1];
    for (uint64_t x = x0 + __lane_id(); x < x1; x += 64) {
      const uint32_t v = a[x];
      if (x + 1 < end && a[x + 1] < v) atomicOr(err, 1);  // unsorted input
      uint8_t k = 0;
      if (v != SENT) {
        uint64_t rank = 0;
        if (x > beg && a[x - 1] == v) rank = x - lower_bound_dev<uint32_t>(a, beg, x, v);
        const uint64_t lb = lower_bound_dev<uint32_t>(b, b0, b1, v);
        uint64_t cnt = 0;
        if (lb < b1 && b[lb] == v) cnt = upper_bound_dev<uint32_t>(b, lb, b1, v) - lb;
        if (side == 0) {
          switch (op) {
            case SYZGPU_DIFFERENCE:
            case SYZGPU_SYMMETRIC_DIFFERENCE: k = rank >= cnt; break;
            case SYZGPU_UNION: k = 1; break;
            default: k = rank < cnt; break;
          }
        } else {
          k = (op == SYZGPU_UNION || op == SYZGPU_SYMMETRIC_DIFFERENCE) ? (rank >= cnt) : 0;
        }
      }
      keep[x] = k;
    }
  }
}

__global__ void k_setop_pairlen(const uint64_t* aoff, const uint64_t* boff, const uint64_t* ka, const uint64_t* kb,
                                uint32_t npairs, uint64_t* plen) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += gridDim.x * blockDim.x)
    plen[p] = (ka[aoff[p + 1]] - ka[aoff[p]]) + (kb[boff[p + 1]] - kb[boff[p]]);
}

// Scatter kept elements of one side. For side 0 (a): pos = KA(x) + KB(lb_b(v)); side 1 (b):
// pos = KB(y) + KA(ub_a(w)) — equal values from a precede those from b (they are identical). One wave
// per pair, as k_setop_classify.
__global__ __launch_bounds__(256) void k_setop_scatter(int side, const uint32_t* a, const uint64_t* aoff,
                                                       const uint32_t* b, const uint64_t* boff, uint32_t npairs,
                                                       const uint64_t* segoff, const uint8_t* keep, const uint64_t* ka,
                                                       const uint64_t* kb, const uint64_t* outoff, uint32_t* out) {
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6, nseg = segoff[npairs];
  for (uint64_t sid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; sid < nseg; sid += waves) {
    uint64_t x0, x1;
    const uint32_t p = seg_pair(segoff, npairs, sid, aoff, &x0, &x1);
    const uint64_t beg = aoff[p], b0 = boff[p], b1 = boff[p + 1];
    const uint64_t base = outoff[p] - ka[beg] - kb[b0];
    for (uint64_t x = x0 + __lane_id(); x < x1; x += 64) {
      if (!keep[x]) continue;
      const uint32_t v = a[x];
      const uint64_t other = side == 0 ? lower_bound_dev<uint32_t>(b, b0, b1, v) : upper_bound_dev<uint32_t>(b, b0, b1, v);
      out[base + ka[x] + kb[other]] = v;
    }
  }
}

// Device-side batched set op. All pointers device; out_off_dev gets npairs+1 offsets.
// Returns total output length (host), throws on unsorted input / capacity.
uint64_t setop_batch_dev(int op, const uint32_t* a, const uint64_t* aoff, uint64_t na, const uint32_t* b,
                         const uint64_t* boff, uint64_t nb, uint32_t npairs, uint32_t* out, uint64_t out_cap,
                         uint64_t* out_off_dev, hipStream_t s) {
  Context& c = ctx();
  uint8_t* keepa = c.scratch.get<uint8_t>("so_keepa", na + 1);
  uint8_t* keepb = c.scratch.get<uint8_t>("so_keepb", nb + 1);
  uint64_t* ka = c.scratch.get<uint64_t>("so_ka", na + 1);
  uint64_t* kb = c.scratch.get<uint64_t>("so_kb", nb + 1);
  uint64_t* plen = c.scratch.get<uint64_t>("so_plen", npairs + 1);
  int* err = c.scratch.get<int>("so_err", 1);
  uint32_t* nsa = c.scratch.get<uint32_t>("so_nsa", npairs + 1);
  uint32_t* nsb = c.scratch.get<uint32_t>("so_nsb", npairs + 1);
  uint64_t* sga = c.scratch.get<uint64_t>("so_sga", npairs + 1);
  uint64_t* sgb = c.scratch.get<uint64_t>("so_sgb", npairs + 1);
  SYZ_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  k_setop_nseg<<<grid_for(npairs, 256, 4096), 256, 0, s>>>(aoff, npairs, nsa);
  SYZ_LAUNCHED();
  k_setop_nseg<<<grid_for(npairs, 256, 4096), 256, 0, s>>>(boff, npairs, nsb);
  SYZ_LAUNCHED();
  exclusive_scan_u32(nsa, sga, npairs, s);
  exclusive_scan_u32(nsb, sgb, npairs, s);
  const uint64_t sega = npairs + na / SO_SEG + 1, segb = npairs + nb / SO_SEG + 1;  // segment bounds
  if (na) {
    k_setop_classify<<<grid_for(sega * 64, 256, 65536), 256, 0, s>>>(op, 0, a, aoff, b, boff, npairs, sga, keepa, err);
    SYZ_LAUNCHED();
  }
  if (nb) {
    k_setop_classify<<<grid_for(segb * 64, 256, 65536), 256, 0, s>>>(op, 1, b, boff, a, aoff, npairs, sgb, keepb, err);
    SYZ_LAUNCHED();
  }
  exclusive_scan_u8(keepa, ka, na, s);
  exclusive_scan_u8(keepb, kb, nb, s);
  k_setop_pairlen<<<grid_for(npairs, 256, 4096), 256, 0, s>>>(aoff, boff, ka, kb, npairs, plen);
  SYZ_LAUNCHED();
  exclusive_scan_u64(plen, out_off_dev, npairs, s);
  int* herr = c.pinned.get<int>(4);
  uint64_t* htot = reinterpret_cast<uint64_t*>(herr + 2);
  SYZ_HIP(hipMemcpyAsync(herr, err, sizeof(int), hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(htot, out_off_dev + npairs, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (*herr) fail(SYZGPU_EINVAL, "set operation input is not sorted ascending");
  const uint64_t total = *htot;
  if (total > out_cap) fail(SYZGPU_ECAPACITY, "set operation output capacity too small");
  if (na) {
    k_setop_scatter<<<grid_for(sega * 64, 256, 65536), 256, 0, s>>>(0, a, aoff, b, boff, npairs, sga, keepa, ka, kb,
                                                                    out_off_dev, out);
    SYZ_LAUNCHED();
  }
  if (nb) {
    k_setop_scatter<<<grid_for(segb * 64, 256, 65536), 256, 0, s>>>(1, b, boff, a, aoff, npairs, sgb, keepb, kb, ka,
                                                                    out_off_dev, out);
    SYZ_LAUNCHED();
  }
  return total;
}

// ---- Canonicalize -------------------------------------------------------------------------------

constexpr int CANON_LDS = 16384;  // PCs sorted in LDS per cover (kCoverSize = 16<<10)
constexpr int CANON_BLOCK = 1024;

// One workgroup per cover of length <= CANON_LDS: bitonic sort in LDS (padded with the sentinel,
// which sorts last and is cut off), then unique with last = sentinel, written back in place.
__global__ __launch_bounds__(CANON_BLOCK) void k_canon_lds(uint32_t* pcs, const uint64_t* off,
                                                           const uint32_t* list, uint32_t nlist,
                                                           uint64_t* out_len) {
  __shared__ uint32_t s[CANON_LDS];
  __shared__ uint32_t red[CANON_BLOCK / 64 + 1];
  for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
    const uint32_t seg = list[li];
    const uint64_t beg = off[seg];
    const uint32_t n = (uint32_t)(off[seg + 1] - beg);
    uint32_t P = 1;
    while (P < n) P <<= 1;
    for (uint32_t i = threadIdx.x; i < P; i += CANON_BLOCK) s[i] = i < n ? pcs[beg + i] : SENT;
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t i = threadIdx.x; i < P; i += CANON_BLOCK) {
          const uint32_t ij = i ^ j;
          if (ij > i) {
            const uint32_t x = s[i], y = s[ij];
            const bool up = (i & k) == 0;
            if ((x > y) == up) {
              s[i] = y;
              s[ij] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    // unique: keep[i] = s[i] != (i ? s[i-1] : SENT); chunked ordered compaction
    uint32_t outp = 0;
    for (uint32_t base = 0; base < n; base += CANON_BLOCK) {
      const uint32_t i = base + threadIdx.x;
      uint32_t v = 0, k = 0;
      if (i < n) {
        v = s[i];
        const uint32_t prev = i ? s[i - 1] : SENT;
        k = v != prev;
      }
      uint32_t tot;
      const uint32_t r = block_excl_scan<CANON_BLOCK>(k, red, &tot);
      if (k) pcs[beg + outp + r] = v;
      outp += tot;
    }
    if (threadIdx.x == 0) out_len[seg] = outp;
    __syncthreads();
  }
}

// Large covers: global bitonic network over a padded copy, one (k, j) step per launch.
__global__ void k_canon_pad(const uint32_t* src, uint64_t n, uint32_t* dst, uint64_t P) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = i < n ? src[i] : SENT;
}
__global__ void k_bitonic_step(uint32_t* s, uint64_t P, uint64_t k, uint64_t j) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t ij = i ^ j;
    if (ij > i) {
      const uint32_t x = s[i], y = s[ij];
      const bool up = (i & k) == 0;
      if ((x > y) == up) {
        s[i] = y;
        s[ij] = x;
      }
    }
  }
}
__global__ void k_unique_flags(const uint32_t* s, uint64_t n, uint8_t* keep) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    keep[i] = s[i] != (i ? s[i - 1] : SENT);
}
__global__ void k_unique_scatter(const uint32_t* s, uint64_t n, const uint8_t* keep, const uint64_t* pos,
                                 uint32_t* dst) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (keep[i]) dst[pos[i]] = s[i];
}
__global__ void k_store_len(const uint64_t* pos, uint64_t n, uint64_t* out_len, uint32_t seg) {
  out_len[seg] = pos[n];
}

// Canonicalize every cover of a device CSR in place. host_off is the host copy of off.
void canonicalize_batch_dev(uint32_t* pcs, const uint64_t* off, const uint64_t* host_off, size_t ncov,
                            uint64_t* out_len, hipStream_t s) {
  Context& c = ctx();
  std::vector<uint32_t> small, big;
  for (size_t i = 0; i < ncov; i++) {
    uint64_t n = host_off[i + 1] - host_off[i];
    if (n <= (uint64_t)CANON_LDS)
      small.push_back((uint32_t)i);
    else
      big.push_back((uint32_t)i);
  }
  if (!small.empty()) {
    uint32_t* dlist = c.scratch.get<uint32_t>("canon_list", small.size());
    SYZ_HIP(hipMemcpyAsync(dlist, small.data(), small.size() * 4, hipMemcpyHostToDevice, s));
    unsigned grid = (unsigned)std::min<size_t>(small.size(), 4096);
    k_canon_lds<<<grid, CANON_BLOCK, 0, s>>>(pcs, off, dlist, (uint32_t)small.size(), out_len);
    SYZ_LAUNCHED();
    SYZ_HIP(hipStreamSynchronize(s));  // dlist reused below / by the next call
  }
  for (uint32_t seg : big) {
    const uint64_t n = host_off[seg + 1] - host_off[seg];
    uint64_t P = 1;
    while (P < n) P <<= 1;
    uint32_t* tmp = c.scratch.get<uint32_t>("canon_big", P);
    uint8_t* keep = c.scratch.get<uint8_t>("canon_keep", n);
    uint64_t* pos = c.scratch.get<uint64_t>("canon_pos", n + 1);
    const unsigned g = grid_for(P, 256, 65536);
    k_canon_pad<<<g, 256, 0, s>>>(pcs + host_off[seg], n, tmp, P);
    SYZ_LAUNCHED();
    for (uint64_t k = 2; k <= P; k <<= 1)
      for (uint64_t j = k >> 1; j > 0; j >>= 1) {
        k_bitonic_step<<<g, 256, 0, s>>>(tmp, P, k, j);
        SYZ_LAUNCHED();
      }
    k_unique_flags<<<grid_for(n, 256, 65536), 256, 0, s>>>(tmp, n, keep);
    SYZ_LAUNCHED();
    exclusive_scan_u8(keep, pos, n, s);
    k_unique_scatter<<<grid_for(n, 256, 65536), 256, 0, s>>>(tmp, n, keep, pos, pcs + host_off[seg]);
    SYZ_LAUNCHED();
    k_store_len<<<1, 1, 0, s>>>(pos, n, out_len, seg);
    SYZ_LAUNCHED();
  }
}

}  // namespace syz

using namespace syz;

namespace {

int pair_op(int op, const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, size_t cap,
            size_t* out_n) {
  SYZ_API_BODY({
    hipStream_t s = C_.stream;
    if ((na && !a) || (nb && !b) || !out_n) fail(SYZGPU_EINVAL, "null pointer");
    uint32_t* da = C_.scratch.get<uint32_t>("po_a", na + 1);
    uint32_t* db = C_.scratch.get<uint32_t>("po_b", nb + 1);
    uint64_t* doff = C_.scratch.get<uint64_t>("po_off", 4);
    uint32_t* dout = C_.scratch.get<uint32_t>("po_out", na + nb + 1);
    uint64_t* doo = C_.scratch.get<uint64_t>("po_oo", 2);
    uint64_t hoff[4] = {0, (uint64_t)na, 0, (uint64_t)nb};
    if (na) SYZ_HIP(hipMemcpyAsync(da, a, na * 4, hipMemcpyHostToDevice, s));
    if (nb) SYZ_HIP(hipMemcpyAsync(db, b, nb * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(doff, hoff, sizeof(hoff), hipMemcpyHostToDevice, s));
    uint64_t tot = setop_batch_dev(op, da, doff, na, db, doff + 2, nb, 1, dout, na + nb, doo, s);
    if (tot > cap) fail(SYZGPU_ECAPACITY, "output capacity too small");
    if (tot) SYZ_HIP(hipMemcpyAsync(out, dout, tot * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    *out_n = tot;
  })
}

}  // namespace

extern "C" {

int syzgpu_difference(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, size_t cap,
                      size_t* out_n) {
  return pair_op(SYZGPU_DIFFERENCE, a, na, b, nb, out, cap, out_n);
}
int syzgpu_symmetric_difference(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out,
                                size_t cap, size_t* out_n) {
  return pair_op(SYZGPU_SYMMETRIC_DIFFERENCE, a, na, b, nb, out, cap, out_n);
}
int syzgpu_union(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, size_t cap,
                 size_t* out_n) {
  return pair_op(SYZGPU_UNION, a, na, b, nb, out, cap, out_n);
}
int syzgpu_intersection(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, size_t cap,
                        size_t* out_n) {
  return pair_op(SYZGPU_INTERSECTION, a, na, b, nb, out, cap, out_n);
}

int syzgpu_setop_batch(int op, const uint32_t* a, const uint64_t* a_off, const uint32_t* b, const uint64_t* b_off,
                       size_t npairs, uint32_t* out, size_t out_cap, uint64_t* out_off) {
  SYZ_API_BODY({
    if (op < 0 || op > 3) fail(SYZGPU_EINVAL, "bad set operation");
    if (!a_off || !b_off || !out_off) fail(SYZGPU_EINVAL, "null pointer");
    if (npairs == 0) {
      out_off[0] = 0;
      return SYZGPU_OK;
    }
    hipStream_t s = C_.stream;
    const uint64_t na = a_off[npairs], nb = b_off[npairs];
    if (a_off[0] != 0 || b_off[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
    uint32_t* da = C_.scratch.get<uint32_t>("sb_a", na + 1);
    uint32_t* db = C_.scratch.get<uint32_t>("sb_b", nb + 1);
    uint64_t* dao = C_.scratch.get<uint64_t>("sb_ao", npairs + 1);
    uint64_t* dbo = C_.scratch.get<uint64_t>("sb_bo", npairs + 1);
    uint64_t* doo = C_.scratch.get<uint64_t>("sb_oo", npairs + 1);
    uint64_t cap_needed = 0;
    switch (op) {
      case SYZGPU_DIFFERENCE: cap_needed = na; break;
      case SYZGPU_INTERSECTION: cap_needed = std::min(na, nb); break;
      default: cap_needed = na + nb;
    }
    uint32_t* dout = C_.scratch.get<uint32_t>("sb_out", cap_needed + 1);
    if (na) SYZ_HIP(hipMemcpyAsync(da, a, na * 4, hipMemcpyHostToDevice, s));
    if (nb) SYZ_HIP(hipMemcpyAsync(db, b, nb * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(dao, a_off, (npairs + 1) * 8, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(dbo, b_off, (npairs + 1) * 8, hipMemcpyHostToDevice, s));
    uint64_t tot = setop_batch_dev(op, da, dao, na, db, dbo, nb, (uint32_t)npairs, dout, cap_needed, doo, s);
    if (tot > out_cap) fail(SYZGPU_ECAPACITY, "output capacity too small");
    if (tot) SYZ_HIP(hipMemcpyAsync(out, dout, tot * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(out_off, doo, (npairs + 1) * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_setop_batch_dev(int op, const uint32_t* a, const uint64_t* a_off, uint64_t na, const uint32_t* b,
                           const uint64_t* b_off, uint64_t nb, size_t npairs, uint32_t* out, size_t out_cap,
                           uint64_t* out_off, void* stream, uint64_t* total) {
  SYZ_API_BODY({
    if (op < 0 || op > 3) fail(SYZGPU_EINVAL, "bad set operation");
    if (!a_off || !b_off || !out_off || (na && !a) || (nb && !b)) fail(SYZGPU_EINVAL, "null pointer");
    if (npairs >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "too many pairs");
    hipStream_t s = (hipStream_t)stream;
    uint64_t tot = 0;
    if (npairs == 0) {
      SYZ_HIP(hipMemsetAsync(out_off, 0, 8, s));
      SYZ_HIP(hipStreamSynchronize(s));
    } else {
      tot = setop_batch_dev(op, a, a_off, na, b, b_off, nb, (uint32_t)npairs, out, out_cap, out_off, s);
      SYZ_HIP(hipStreamSynchronize(s));
    }
    if (total) *total = tot;
  })
}

int syzgpu_canonicalize_batch(uint32_t* pcs, const uint64_t* off, size_t ncov, uint64_t* out_len) {
  SYZ_API_BODY({
    if (!off || !out_len) fail(SYZGPU_EINVAL, "null pointer");
    if (ncov == 0) return SYZGPU_OK;
    hipStream_t s = C_.stream;
    const uint64_t n = off[ncov];
    uint32_t* dp = C_.scratch.get<uint32_t>("cb_pcs", n + 1);
    uint64_t* doff = C_.scratch.get<uint64_t>("cb_off", ncov + 1);
    uint64_t* dlen = C_.scratch.get<uint64_t>("cb_len", ncov + 1);
    if (n) SYZ_HIP(hipMemcpyAsync(dp, pcs, n * 4, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(doff, off, (ncov + 1) * 8, hipMemcpyHostToDevice, s));
    canonicalize_batch_dev(dp, doff, off, ncov, dlen, s);
    if (n) SYZ_HIP(hipMemcpyAsync(pcs, dp, n * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(out_len, dlen, ncov * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_canonicalize(uint32_t* cov, size_t n, size_t* out_n) {
  if (!out_n || (n && !cov)) return SYZGPU_EINVAL;
  if (n == 0) {
    *out_n = 0;
    return SYZGPU_OK;
  }
  uint64_t off[2] = {0, (uint64_t)n};
  uint64_t len = 0;
  int rc = syzgpu_canonicalize_batch(cov, off, 1, &len);
  if (rc == SYZGPU_OK) *out_n = (size_t)len;
  return rc;
}

}  // extern "C"

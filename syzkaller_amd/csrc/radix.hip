// Stable LSD radix sort of (u64 key, u32 value) pairs: the sorting primitive behind the batch
// novelty check (novelty.hip) and of the cover analytics (analytics.hip). 8-bit digits; per pass one
// histogram kernel, one device-wide scan of the digit-major tile counts, and one scatter kernel that
// ranks every item stably inside its tile and writes each digit's run out of LDS contiguously. Passes
// over digits on which all keys agree are skipped (kernel PCs share their top byte).
#include "pipeline.hpp"

namespace syz {

constexpr int RS_BLOCK = 512;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_BLOCK * RS_ITEMS;
constexpr int RS_RADIX = 1 << RADIX_BITS;
constexpr int RS_WAVES = RS_BLOCK / 64;

template <class KT>
__global__ __launch_bounds__(RS_BLOCK) void k_rs_hist(const KT* __restrict__ keys, size_t n, int shift,
                                                      uint32_t ntiles, uint32_t* __restrict__ counts) {
  __shared__ uint32_t h[RS_WAVES][RS_RADIX];
  for (int i = threadIdx.x; i < RS_WAVES * RS_RADIX; i += RS_BLOCK) (&h[0][0])[i] = 0;
  __syncthreads();
  const int w = threadIdx.x >> 6;
  const size_t base = (size_t)blockIdx.x * RS_TILE + threadIdx.x;
  KT k[RS_ITEMS];
#pragma unroll
  for (int i = 0; i < RS_ITEMS; i++) {
    const size_t p = base + (size_t)i * RS_BLOCK;
    k[i] = p < n ? keys[p] : 0;
  }
#pragma unroll
  for (int i = 0; i < RS_ITEMS; i++)
    if (base + (size_t)i * RS_BLOCK < n) atomicAdd(&h[w][(uint32_t)(k[i] >> shift) & (RS_RADIX - 1)], 1u);
  __syncthreads();
  for (int d = threadIdx.x; d < RS_RADIX; d += RS_BLOCK) {
    uint32_t s = 0;
#pragma unroll
    for (int x = 0; x < RS_WAVES; x++) s += h[x][d];
    counts[(size_t)d * ntiles + blockIdx.x] = s;
  }
}

// Scatter of one tile, stable. The tile is split into RS_WAVES contiguous wave slices (wave w holds
// tile positions [w*WAVE_ITEMS, (w+1)*WAVE_ITEMS), lane-interleaved per round, so loads coalesce).
// A wave ranks its own items with ballots against per-wave LDS digit counters - no workgroup barrier
// per round - then one pass turns the counters into slice bases (tile digit offset + earlier waves),
// the items land digit-sorted in LDS, and each digit's run leaves as consecutive stores.
template <class KT>
__global__ __launch_bounds__(RS_BLOCK) void k_rs_scatter(const KT* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin, size_t n, int shift,
                                                         uint32_t ntiles, const uint64_t* __restrict__ offs,
                                                         KT* __restrict__ kout, uint32_t* __restrict__ vout) {
  constexpr int WAVE_ITEMS = RS_ITEMS * 64;
  __shared__ KT sk[RS_TILE];
  __shared__ uint32_t sv[RS_TILE];
  __shared__ uint32_t wc[RS_WAVES][RS_RADIX];
  __shared__ uint64_t gshift[RS_RADIX];
  __shared__ uint32_t lds[RS_BLOCK / 64 + 1];
  for (int i = threadIdx.x; i < RS_WAVES * RS_RADIX; i += RS_BLOCK) (&wc[0][0])[i] = 0;
  const int w = threadIdx.x >> 6;
  const uint32_t lane = __lane_id();
  const size_t tile0 = (size_t)blockIdx.x * RS_TILE;
  const uint32_t tn = (uint32_t)(n - tile0 < (size_t)RS_TILE ? n - tile0 : RS_TILE);
  const uint32_t wbase = (uint32_t)w * WAVE_ITEMS + lane;
  KT k[RS_ITEMS];
  uint32_t v[RS_ITEMS];
#pragma unroll
  for (int i = 0; i < RS_ITEMS; i++) {
    const uint32_t p = wbase + i * 64;
    k[i] = p < tn ? kin[tile0 + p] : 0;
    v[i] = p < tn ? vin[tile0 + p] : 0;
  }
  __syncthreads();
  const uint64_t lt = lanemask_lt();
  uint32_t r[RS_ITEMS];
#pragma unroll
  for (int i = 0; i < RS_ITEMS; i++) {
    const bool valid = wbase + i * 64 < tn;
    const uint32_t d = (uint32_t)(k[i] >> shift) & (RS_RADIX - 1);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < RADIX_BITS; b++) {
      const bool bit = (d >> b) & 1;
      const uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const uint32_t wrank = __popcll(peers & lt);
    const uint32_t before = wc[w][d];  // every peer reads before the leader's add (wave program order)
    r[i] = before + wrank;
    if (valid && wrank == 0) wc[w][d] = before + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  // per digit: tile offset (scan over digits), then each wave's base inside it
  uint32_t tot_d = 0;
  if (threadIdx.x < RS_RADIX) {
#pragma unroll
    for (int x = 0; x < RS_WAVES; x++) tot_d += wc[x][threadIdx.x];
  }
  uint32_t total;
  const uint32_t loff = block_excl_scan<RS_BLOCK>(tot_d, lds, &total);
  if (threadIdx.x < RS_RADIX) {
    uint32_t run = loff;
#pragma unroll
    for (int x = 0; x < RS_WAVES; x++) {
      const uint32_t c = wc[x][threadIdx.x];
      wc[x][threadIdx.x] = run;
      run += c;
    }
    gshift[threadIdx.x] = offs[(size_t)threadIdx.x * ntiles + blockIdx.x] - (uint64_t)loff;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < RS_ITEMS; i++) {
    if (wbase + i * 64 < tn) {
      const uint32_t d = (uint32_t)(k[i] >> shift) & (RS_RADIX - 1);
      const uint32_t p = wc[w][d] + r[i];
      sk[p] = k[i];
      sv[p] = v[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < RS_ITEMS; i++) {
    const uint32_t p = threadIdx.x + i * RS_BLOCK;
    if (p < tn) {
      const KT key = sk[p];
      const uint64_t dst = gshift[(uint32_t)(key >> shift) & (RS_RADIX - 1)] + p;
      kout[dst] = key;
      vout[dst] = sv[p];
    }
  }
}

// OR and AND of every key (bits[0] |=, bits[1] &=): a digit whose bits agree across all keys puts
// every item in one bucket, so its pass would be an identity copy and is skipped.
template <class KT>
__global__ void k_rs_bits(const KT* __restrict__ keys, size_t n, unsigned long long* bits) {
  unsigned long long o = 0, a = ~0ull;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    o |= keys[i];
    a &= keys[i];
  }
  for (int d = 32; d >= 1; d >>= 1) {
    o |= __shfl_xor(o, d, 64);
    a &= __shfl_xor(a, d, 64);
  }
  if (__lane_id() == 0) {
    atomicOr(&bits[0], o);
    atomicAnd(&bits[1], a);
  }
}

// Sorts n pairs by key bits [0, end_bit), stably. Ping-pongs between (keys, vals) and (ktmp, vtmp);
// on return keys/vals point at the sorted arrays (the pointers may be swapped with the tmp ones).
template <class KT>
static void radix_sort_pairs_t(KT*& keys, uint32_t*& vals, KT*& ktmp, uint32_t*& vtmp, size_t n, int end_bit,
                               hipStream_t s) {
  if (n <= 1) return;
  if (n >= (1ull << 40)) fail(SYZGPU_EINVAL, "radix sort: too many items");
  const size_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  if (ntiles * RS_RADIX >= 0xFFFFFFFFull) fail(SYZGPU_EINVAL, "radix sort: too many tiles");
  Scratch& sc = ctx().scratch;
  uint32_t* counts = sc.get<uint32_t>("rs_counts", ntiles * RS_RADIX + 1);
  uint64_t* offs = sc.get<uint64_t>("rs_offs", ntiles * RS_RADIX + 1);
  // one readback: the bits that differ between keys (RS_ALL_PASSES=1 runs every pass, for A/B)
  unsigned long long* d_bits = sc.get<unsigned long long>("rs_bits", 2);
  SYZ_HIP(hipMemsetAsync(d_bits, 0, 8, s));
  SYZ_HIP(hipMemsetAsync(d_bits + 1, 0xFF, 8, s));
  k_rs_bits<KT><<<grid_for(n, 256, 2048), 256, 0, s>>>(keys, n, d_bits);
  SYZ_LAUNCHED();
  unsigned long long* h_bits = ctx().pinned.get<unsigned long long>(2);
  SYZ_HIP(hipMemcpyAsync(h_bits, d_bits, 16, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const unsigned long long differ = dev_env("SYZGPU_RS_ALL_PASSES") ? ~0ull : (h_bits[0] ^ h_bits[1]);
  for (int shift = 0; shift < end_bit; shift += RADIX_BITS) {
    if (!((differ >> shift) & (RS_RADIX - 1))) continue;
    k_rs_hist<KT><<<(unsigned)ntiles, RS_BLOCK, 0, s>>>(keys, n, shift, (uint32_t)ntiles, counts);
    SYZ_LAUNCHED();
    exclusive_scan_u32(counts, offs, ntiles * RS_RADIX, s);
    k_rs_scatter<KT><<<(unsigned)ntiles, RS_BLOCK, 0, s>>>(keys, vals, n, shift, (uint32_t)ntiles, offs, ktmp, vtmp);
    SYZ_LAUNCHED();
    std::swap(keys, ktmp);
    std::swap(vals, vtmp);
  }
}

void radix_sort_pairs(uint64_t*& keys, uint32_t*& vals, uint64_t*& ktmp, uint32_t*& vtmp, size_t n, int end_bit,
                      hipStream_t s) {
  radix_sort_pairs_t(keys, vals, ktmp, vtmp, n, end_bit, s);
}

void radix_sort_pairs(uint32_t*& keys, uint32_t*& vals, uint32_t*& ktmp, uint32_t*& vtmp, size_t n, int end_bit,
                      hipStream_t s) {
  radix_sort_pairs_t(keys, vals, ktmp, vtmp, n, end_bit, s);
}

}  // namespace syz

// Stable LSD radix sort of (u64 key, u32 value) pairs: the sorting primitive behind the batch
// novelty check (novelty.hip). 8-bit digits; per pass one histogram kernel, one device-wide scan of
// the digit-major tile counts, and one scatter kernel that ranks every item stably inside its tile
// (wave ballots give the rank among same-digit lanes, per-wave LDS counters order the waves).
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

template <class KT>
__global__ __launch_bounds__(RS_BLOCK) void k_rs_scatter(const KT* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin, size_t n, int shift,
                                                         uint32_t ntiles, const uint64_t* __restrict__ offs,
                                                         KT* __restrict__ kout, uint32_t* __restrict__ vout) {
  __shared__ uint32_t run[RS_RADIX];
  __shared__ uint32_t wc[RS_WAVES][RS_RADIX];
  __shared__ uint64_t goff[RS_RADIX];
  for (int d = threadIdx.x; d < RS_RADIX; d += RS_BLOCK) {
    run[d] = 0;
    goff[d] = offs[(size_t)d * ntiles + blockIdx.x];
  }
  for (int i = threadIdx.x; i < RS_WAVES * RS_RADIX; i += RS_BLOCK) (&wc[0][0])[i] = 0;
  const int w = threadIdx.x >> 6;
  const size_t base = (size_t)blockIdx.x * RS_TILE + threadIdx.x;
  KT k[RS_ITEMS];
  uint32_t v[RS_ITEMS];
#pragma unroll
  for (int i = 0; i < RS_ITEMS; i++) {
    const size_t p = base + (size_t)i * RS_BLOCK;
    k[i] = p < n ? kin[p] : 0;
    v[i] = p < n ? vin[p] : 0;
  }
  __syncthreads();
  const uint64_t lt = lanemask_lt();
#pragma unroll
  for (int i = 0; i < RS_ITEMS; i++) {
    // round i holds tile positions [i*BLOCK, (i+1)*BLOCK) in thread order: ranks stay stable
    const bool valid = base + (size_t)i * RS_BLOCK < n;
    const uint32_t d = valid ? (uint32_t)(k[i] >> shift) & (RS_RADIX - 1) : 0;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const bool bit = (d >> b) & 1;
      const uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const uint32_t wrank = __popcll(peers & lt);
    if (valid && wrank == 0) wc[w][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pre = run[d];
      for (int x = 0; x < w; x++) pre += wc[x][d];
      const uint64_t dst = goff[d] + pre + wrank;
      kout[dst] = k[i];
      vout[dst] = v[i];
    }
    __syncthreads();
    for (int dd = threadIdx.x; dd < RS_RADIX; dd += RS_BLOCK) {
      uint32_t s = 0;
#pragma unroll
      for (int x = 0; x < RS_WAVES; x++) {
        s += wc[x][dd];
        wc[x][dd] = 0;
      }
      run[dd] += s;
    }
    __syncthreads();
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
  for (int shift = 0; shift < end_bit; shift += RADIX_BITS) {
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

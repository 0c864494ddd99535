// Device-wide exclusive scan in one pass (decoupled look-back), over values a functor produces, one or
// two sequences at once.
//
// Tiles of SCAN_TILE elements go in ticket order (an atomic counter, so a tile's predecessors are
// resident or done). Each tile publishes its sums (flag 1) and, once its look-back has found an
// inclusive prefix (flag 2), its own, as words holding flag, epoch and value together, so relaxed
// device-scope atomics carry them between XCDs without fences (a release / acquire pair per tile
// writes back / invalidates the L2: measured 75 us for a 276-tile scan). The epoch lets the words go
// uncleared for 63 scans; the tile that takes the last ticket resets the counter. One launch per scan:
// the reduce / scan-of-sums / apply form took three or four, ~6 us each at the step's small sizes.
// Values: sums below 2^56 (a tile whose inclusive prefix reaches 2^56 sets the fault word, below).
// A look-back that waits 2^24 polls for a predecessor that never publishes (a bug: every predecessor
// holds a ticket taken before, so it is resident or done) stops waiting and sets the fault word too; the
// process's entry points then fail with SYZGPU_EINTERNAL (check_faults) rather than return its output.
// scan_f must not be captured into a HIP graph: each launch takes the next epoch on the host, which a
// replayed capture would reuse.
#pragma once
#include "common.hpp"

namespace syz {

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// the look-back state of one tag: the ticket (its own line), words[tiles * NV]
struct ScanState {
  uint64_t* words;
  uint32_t* ticket;
  uint32_t epoch;   // 1..63
  uint32_t* fault;  // the process's fault word (host-mapped, fault_word_dev)
};
ScanState scan_state(const char* tag, size_t tiles, int nv, hipStream_t s);  // runtime.hip
constexpr uint64_t SCAN_VMASK = (1ull << 56) - 1;

// Tile t's exclusive prefix by decoupled look-back, run by ONE whole wave: publishes t's sums tot
// (flag 1), reads 64 predecessors' words at once (the nearest inclusive prefix ends it, else the
// window's sums are added and it moves 64 tiles back), publishes t's inclusive prefix (flag 2) and
// returns the exclusive one in excl on every lane. Tiles must be taken in ticket order (st.ticket), so
// every predecessor belongs to a running workgroup.
template <int NV>
__device__ __forceinline__ void scan_lookback(const ScanState& st, uint32_t t, const uint64_t* tot, uint64_t* excl) {
  const unsigned lane = __lane_id();
  const uint64_t ep = (uint64_t)st.epoch << 56, f_agg = (1ull << 62) | ep, f_inc = (2ull << 62) | ep;
  auto put = [&](uint64_t f, const uint64_t* x) {
#pragma unroll
    for (int q = 0; q < NV; q++)
      __hip_atomic_store(&st.words[(size_t)t * NV + q], f | (x[q] & SCAN_VMASK), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  };
#pragma unroll
  for (int q = 0; q < NV; q++) excl[q] = 0;
  if (t > 0) {
    if (lane == 0) put(f_agg, tot);
    uint32_t spins = 0;
    for (int64_t w0 = (int64_t)t - 1; w0 >= 0;) {  // window: tiles w0, w0 - 1, ..., w0 - 63
      const int64_t i = w0 - (int64_t)lane;
      uint64_t w[NV];
      bool ready = true, inc = false;
      if (i >= 0) {
#pragma unroll
        for (int q = 0; q < NV; q++)
          w[q] = __hip_atomic_load(&st.words[(size_t)i * NV + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t h = w[0] & ~SCAN_VMASK;
        ready = h == f_agg || h == f_inc;
#pragma unroll
        for (int q = 1; q < NV; q++) ready = ready && (w[q] & ~SCAN_VMASK) == h;  // (both words one state)
        inc = ready && h == f_inc;
      } else {
#pragma unroll
        for (int q = 0; q < NV; q++) w[q] = 0;
      }
      const uint64_t incm = __ballot(inc);
      // lanes up to the nearest inclusive prefix must all be ready
      const int last = incm ? __ffsll((unsigned long long)incm) - 1 : 63;
      const uint64_t need = last >= 63 ? ~0ull : ((2ull << last) - 1);
      if ((__ballot(ready) & need) != need) {
        // (a predecessor that never publishes is a bug: left, not waited for forever; the output is
        // then wrong and the parity tests say so)
        if (++spins == (1u << 24)) {
          if (lane == 0) __hip_atomic_fetch_or(st.fault, FAULT_SCAN_WAIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
#pragma unroll
      for (int q = 0; q < NV; q++) excl[q] += wave_sum_u64((int)lane <= last ? (w[q] & SCAN_VMASK) : 0ull);
      if (incm || w0 < 64) break;
      w0 -= 64;
    }
  }
  if (lane == 0) {
    uint64_t inc[NV];
#pragma unroll
    for (int q = 0; q < NV; q++) {
      inc[q] = excl[q] + tot[q];
      if (inc[q] > SCAN_VMASK) __hip_atomic_fetch_or(st.fault, FAULT_SCAN_RANGE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    put(f_inc, inc);
  }
}

// f(i, v): the NV values of element i (i < n). out_k[i] = the sum of sequence k before i; out_k[n] =
// its total.
template <int NV, class F>
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_f(F f, size_t n, uint64_t* out0, uint64_t* out1, ScanState st,
                                                       uint32_t tiles) {
  __shared__ uint64_t lds[SCAN_BLOCK / 64 + 1];
  __shared__ uint32_t tile_s;
  __shared__ uint64_t excl_s[NV];
  if (threadIdx.x == 0) {
    const uint32_t t = atomicAdd(st.ticket, 1u);
    if (t == tiles - 1) atomicExch(st.ticket, 0u);  // every ticket of this launch is taken
    tile_s = t;
  }
  __syncthreads();
  const uint32_t t = tile_s;
  const size_t base = (size_t)t * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
  uint64_t v[NV][SCAN_ITEMS];
  uint64_t pre[NV], tot[NV];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    uint64_t x[NV];
#pragma unroll
    for (int q = 0; q < NV; q++) x[q] = 0;
    if (base + k < n) f(base + k, x);
#pragma unroll
    for (int q = 0; q < NV; q++) v[q][k] = x[q];
  }
#pragma unroll
  for (int q = 0; q < NV; q++) {
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) s += v[q][k];
    pre[q] = block_excl_scan<SCAN_BLOCK>(s, lds, &tot[q]);
  }
  if (threadIdx.x < 64) {
    uint64_t excl[NV];
    scan_lookback<NV>(st, t, tot, excl);
    if (threadIdx.x == 0)
#pragma unroll
      for (int q = 0; q < NV; q++) excl_s[q] = excl[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; q++) {
    uint64_t* out = q == 0 ? out0 : out1;
    uint64_t p = pre[q] + excl_s[q];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
      if (base + k < n) out[base + k] = p;
      p += v[q][k];
    }
    if (t == tiles - 1 && threadIdx.x == SCAN_BLOCK - 1) out[n] = p;
  }
}

__global__ void k_scan_zero(uint64_t* out0, uint64_t* out1);  // runtime.hip: the totals of an empty scan

// Long scans (more tiles than SCAN_LB_MAX): reduce-then-scan instead, since every tile of a long
// single-pass scan is in flight at once and its look-back walks back far before it meets an inclusive
// prefix (a 9M-element scan measured slower than three launches). Tile sums, a scan of them, then the
// tiles again with their offsets.
constexpr size_t SCAN_LB_MAX = 512;
template <int NV, class F>
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_sums_f(F f, size_t n, uint64_t* sums, uint32_t tiles) {
  __shared__ uint64_t lds[SCAN_BLOCK / 64 + 1];
  const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
  uint64_t acc[NV];
#pragma unroll
  for (int q = 0; q < NV; q++) acc[q] = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    uint64_t x[NV];
#pragma unroll
    for (int q = 0; q < NV; q++) x[q] = 0;
    if (base + k < n) f(base + k, x);
#pragma unroll
    for (int q = 0; q < NV; q++) acc[q] += x[q];
  }
#pragma unroll
  for (int q = 0; q < NV; q++) {
    uint64_t tot;
    block_excl_scan<SCAN_BLOCK>(acc[q], lds, &tot);
    if (threadIdx.x == 0) sums[(size_t)q * tiles + blockIdx.x] = tot;
  }
}
template <int NV, class F>
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_apply_f(F f, size_t n, const uint64_t* offs0, const uint64_t* offs1,
                                                             uint64_t* out0, uint64_t* out1, uint32_t tiles) {
  __shared__ uint64_t lds[SCAN_BLOCK / 64 + 1];
  const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
  uint64_t v[NV][SCAN_ITEMS];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    uint64_t x[NV];
#pragma unroll
    for (int q = 0; q < NV; q++) x[q] = 0;
    if (base + k < n) f(base + k, x);
#pragma unroll
    for (int q = 0; q < NV; q++) v[q][k] = x[q];
  }
#pragma unroll
  for (int q = 0; q < NV; q++) {
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) s += v[q][k];
    uint64_t tot;
    uint64_t p = block_excl_scan<SCAN_BLOCK>(s, lds, &tot) + (q == 0 ? offs0 : offs1)[blockIdx.x];
    uint64_t* out = q == 0 ? out0 : out1;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
      if (base + k < n) out[base + k] = p;
      p += v[q][k];
    }
    if (blockIdx.x == tiles - 1 && threadIdx.x == SCAN_BLOCK - 1) out[n] = p;
  }
}
template <int NV>
struct ScanSumsFn {
  const uint64_t* sums;
  uint32_t tiles;
  __device__ void operator()(size_t i, uint64_t* v) const {
#pragma unroll
    for (int q = 0; q < NV; q++) v[q] = sums[(size_t)q * tiles + i];
  }
};
uint64_t* scan_scratch(const char* tag, int depth, size_t words);  // runtime.hip

// tag: scans that may run at the same time (other streams) take different tags
template <int NV, class F>
void scan_f(F f, size_t n, uint64_t* out0, uint64_t* out1, hipStream_t s, const char* tag, int depth = 0) {
  if (n == 0) {
    k_scan_zero<<<1, 1, 0, s>>>(out0, NV > 1 ? out1 : nullptr);
    SYZ_LAUNCHED();
    return;
  }
  const size_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (tiles > SCAN_LB_MAX) {
    if (tiles >= 0xFFFFFFFFull) fail(SYZGPU_EINVAL, "scan too long");
    uint64_t* buf = scan_scratch(tag, depth, (NV + NV) * (tiles + 1));
    uint64_t* sums = buf;
    uint64_t* offs = buf + NV * (tiles + 1);
    k_scan_sums_f<NV, F><<<(unsigned)tiles, SCAN_BLOCK, 0, s>>>(f, n, sums, (uint32_t)tiles);
    SYZ_LAUNCHED();
    scan_f<NV>(ScanSumsFn<NV>{sums, (uint32_t)tiles}, tiles, offs, NV > 1 ? offs + (tiles + 1) : nullptr, s, tag,
               depth + 1);
    k_scan_apply_f<NV, F><<<(unsigned)tiles, SCAN_BLOCK, 0, s>>>(f, n, offs, NV > 1 ? offs + (tiles + 1) : nullptr,
                                                                  out0, out1, (uint32_t)tiles);
    SYZ_LAUNCHED();
    return;
  }
  char t2[64];
  snprintf(t2, sizeof t2, "%s.%d", tag, depth);
  const ScanState st = scan_state(depth ? t2 : tag, tiles, NV, s);
  k_scan_f<NV, F><<<(unsigned)tiles, SCAN_BLOCK, 0, s>>>(f, n, out0, out1, st, (uint32_t)tiles);
  SYZ_LAUNCHED();
}

}  // namespace syz

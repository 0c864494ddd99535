// Call co-occurrence XᵀX on int8 MFMA: the north_star's "true dense contraction" reading of
// calcDynamicPrio (prog/prio.go:137-152). The reference adds 1 to prios[i0][i1]
// for every pair of distinct call POSITIONS i0 != i1 of a program (so its result depends only on the
// program lengths; syzgpu_dynamic_prio reproduces that bit-exactly). This entry computes the call-ID
// form the loop was meant to have: out[a][b] = the number of ordered pairs of distinct positions of a
// program whose calls are (a, b), summed over the corpus — with X[a][p] = occurrences of call a in
// program p, out = XᵀX - diag(total occurrences). It is NOT the reference's quantity; it is exact
// integer work (int8 operands, int32 accumulation), checked bit-exact by tests/test_gpu_cooccur.py.
//
//   build  X in K-blocks of 32 programs, Xb[kb][c][32] int8 (a 32-row operand of one K-block is 1 KB
//          contiguous), one program per thread (byte counts through u32 atomics), and the total
//          occurrences per call through an LDS histogram
//   gemm   a wave per 64x64 output tile (2x2 v_mfma_i32_32x32x32_i8), four waves per 128x128
//          workgroup tile, the upper triangle of tiles only (an off-diagonal tile adds its transpose
//          too), the K blocks split over KS workgroups, each storing its partial tile; every
//          lane's operand is 16 consecutive program bytes of one call, so A and B agree on the K
//          order inside a step (as in static_prio.hip). Default: both 128-row operand tiles of two
//          K blocks staged through double-buffered LDS per barrier (k_co_gemm_lds<128, 2>);
//          SYZGPU_CO_FORM=0 loads the operands per wave instead (k_co_gemm<1>)
//   reduce out = the sum of the KS partials (and its transpose), out[a][a] -= occurrences of a, in
//          int64; a count that cannot fit int32 is an error, never a wrapped value
#include <algorithm>

#include "pipeline.hpp"

namespace syz {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int CO_KB = 32;     // programs per K block
constexpr int CO_TILE = 128;  // output rows/columns per workgroup

// one program per thread; err: 1 = call id >= C, 2 = a call occurs more than 127 times in a program;
// kbound[kb] = sum of len^2 over the K block's programs (a bound on any cell's count from the block)
__global__ __launch_bounds__(256) void k_co_build(const uint16_t* __restrict__ calls, const uint64_t* __restrict__ off,
                                                  size_t n, int32_t C, uint32_t Cp, uint32_t* Xw,
                                                  unsigned long long* occ, unsigned long long* kbound, int* err) {
  extern __shared__ uint32_t lh[];
  for (int32_t c = threadIdx.x; c < C; c += blockDim.x) lh[c] = 0;
  __syncthreads();
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x) {
    const uint64_t b = off[p], e = off[p + 1];
    const uint64_t kb = p / CO_KB;
    const uint32_t kk = (uint32_t)(p % CO_KB);
    // every count this program adds to one cell is at most cnt_a * cnt_b <= len^2: the K block's bound
    if (e > b) atomicAdd(&kbound[kb], (unsigned long long)(e - b) * (e - b));
    if (e - b > 127) {
      // a call could repeat more than an int8 holds: count this program's repeats first
      for (uint64_t j = b; j < e; j++) {
        uint32_t cnt = 0;
        for (uint64_t i = b; i < e; i++) cnt += calls[i] == calls[j];
        if (cnt > 127) atomicOr(err, 2);
      }
    }
    for (uint64_t j = b; j < e; j++) {
      const uint32_t c = calls[j];
      if ((int32_t)c >= C) {
        atomicOr(err, 1);
        continue;
      }
      const size_t byte = ((size_t)kb * Cp + c) * CO_KB + kk;
      atomicAdd(&Xw[byte >> 2], 1u << (8 * (byte & 3)));
      atomicAdd(&lh[c], 1u);
    }
  }
  __syncthreads();
  for (int32_t c = threadIdx.x; c < C; c += blockDim.x)
    if (lh[c]) atomicAdd(&occ[c], (unsigned long long)lh[c]);
}

// a wave's 64x64 accumulators into its workgroup's partial tile P[kg][tile][TILE][TILE] (plain stores:
// the KS partials are summed by k_co_reduce). Result register r of lane l: row (r & 3) + 8 (r >> 2) +
// 4 (l >> 5), column l & 31 (gfx950 32x32).
template <int TILE>
__device__ __forceinline__ void co_store_partial(const v16i (&acc)[2][2], int* __restrict__ P, size_t tbase,
                                                 uint32_t wr, uint32_t wc, unsigned lane) {
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t col = wc + 32 * j + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const uint32_t row = wr + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        P[tbase + (size_t)row * TILE + col] = acc[i][j][r];
      }
    }
}

// tiles x KS workgroups over the upper triangle of the T x T workgroup tiles (XᵀX is symmetric: an
// off-diagonal tile also adds its transpose) and KS ranges of K blocks; a wave's tile: rows
// r0 + [0, 64), columns c0 + [0, 64). XCD-aware when KS % 8 == 0: workgroups are dealt to the 8 XCDs
// round-robin, so block b runs on XCD b % 8; every tile of one K range is placed on the same XCD,
// so each X block is fetched from HBM into one L2 and re-read there by the tiles that share its rows
template <int PF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_co_gemm(const int8_t* __restrict__ X, int32_t C, uint32_t Cp, uint32_t T,
                                                 uint32_t tiles, uint32_t ks, uint32_t nkb, uint32_t kb_per,
                                                 int* __restrict__ P) {
  uint32_t t, kg;
  if (ks % 8 == 0) {
    const uint32_t j = blockIdx.x >> 3;
    t = j % tiles;
    kg = (j / tiles) * 8 + (blockIdx.x & 7);
  } else {
    t = blockIdx.x % tiles;
    kg = blockIdx.x / tiles;
  }
  const uint32_t tid = t;
  uint32_t ty = 0;  // t -> (ty, tx), tx >= ty
  while (t >= T - ty) t -= T - ty++;
  const uint32_t tx = ty + t;
  const int wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  const uint32_t r0 = ty * CO_TILE + (wv >> 1) * 64, c0 = tx * CO_TILE + (wv & 1) * 64;
  const uint32_t kb0 = kg * kb_per, kb1 = min(nkb, kb0 + kb_per);
  v16i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) acc[i][j] = v16i{};
  // lane l: 16 bytes [16 (l >> 5), +16) of row (l & 31) of a 32-row operand
  const size_t lo = (size_t)(lane & 31) * CO_KB + 16 * (lane >> 5);
  const size_t kstride = (size_t)Cp * CO_KB;
  const int8_t* pa = X + (size_t)r0 * CO_KB + lo;
  const int8_t* pb = X + (size_t)c0 * CO_KB + lo;
  // PF K blocks of operands in flight: stage i holds block kb + i while block kb's MFMAs run
  v4i st[PF][4];
#pragma unroll
  for (int i = 0; i < PF; i++)
    if (kb0 + i < kb1) {
      const size_t o = (size_t)(kb0 + i) * kstride;
      st[i][0] = *reinterpret_cast<const v4i*>(pa + o);
      st[i][1] = *reinterpret_cast<const v4i*>(pa + o + 32 * CO_KB);
      st[i][2] = *reinterpret_cast<const v4i*>(pb + o);
      st[i][3] = *reinterpret_cast<const v4i*>(pb + o + 32 * CO_KB);
    }
  for (uint32_t kb = kb0; kb < kb1; kb += PF) {
#pragma unroll
    for (int i = 0; i < PF; i++) {
      if (kb + i >= kb1) break;
      const v4i a0 = st[i][0], a1 = st[i][1], b0 = st[i][2], b1 = st[i][3];
      if (kb + i + PF < kb1) {
        const size_t o = (size_t)(kb + i + PF) * kstride;
        st[i][0] = *reinterpret_cast<const v4i*>(pa + o);
        st[i][1] = *reinterpret_cast<const v4i*>(pa + o + 32 * CO_KB);
        st[i][2] = *reinterpret_cast<const v4i*>(pb + o);
        st[i][3] = *reinterpret_cast<const v4i*>(pb + o + 32 * CO_KB);
      }
      acc[0][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  co_store_partial<CO_TILE>(acc, P, ((size_t)kg * tiles + tid) * CO_TILE * CO_TILE, (wv >> 1) * 64, (wv & 1) * 64, lane);
}

// LDS-staged form: a workgroup of (TILE / 64)^2 waves stages each K block's A rows [ty TILE, +TILE) and
// B rows [tx TILE, +TILE) (TILE x 32 bytes each, contiguous in Xb) through double-buffered LDS, one
// 16-byte global load per thread per operand; each wave then reads its 2 + 2 operands from LDS
// (ds_read_b128). The two 16-byte halves of row r sit swapped when bit 3 of r is set, so the lane
// groups of a ds_read_b128 (rows {0-3, 12-15, 20-27}, ...) hit 16 distinct 4-bank sets.
template <int TILE, int KPB>
__global__ __launch_bounds__(TILE* TILE / 64) __attribute__((amdgpu_waves_per_eu(4))) void k_co_gemm_lds(
    const int8_t* __restrict__ X, int32_t C, uint32_t Cp, uint32_t T, uint32_t tiles, uint32_t ks, uint32_t nkb,
    uint32_t kb_per, int* __restrict__ P) {
  constexpr int NT = TILE * TILE / 64;        // threads
  constexpr int OPB = TILE * CO_KB;           // bytes of one operand tile per K block
  constexpr int LPT = 2 * OPB / 16 / NT;      // 16-byte loads per thread per K block (A and B)
  static_assert(LPT >= 1 && (2 * OPB / 16) % NT == 0, "staging split");
  __shared__ __align__(16) int8_t sm[2][KPB][2 * OPB];  // [buffer][K block of the stage][A tile | B tile]
  uint32_t t, kg;
  if (ks % 8 == 0) {
    const uint32_t j = blockIdx.x >> 3;
    t = j % tiles;
    kg = (j / tiles) * 8 + (blockIdx.x & 7);
  } else {
    t = blockIdx.x % tiles;
    kg = blockIdx.x / tiles;
  }
  const uint32_t tid = t;
  uint32_t ty = 0;
  while (t >= T - ty) t -= T - ty++;
  const uint32_t tx = ty + t;
  const int wv = threadIdx.x >> 6;
  const unsigned lane = __lane_id();
  constexpr int WPR = TILE / 64;  // waves per tile row
  const uint32_t wr = (wv / WPR) * 64, wc = (wv % WPR) * 64;
  const uint32_t kb0 = kg * kb_per, kb1 = min(nkb, kb0 + kb_per);
  const size_t kstride = (size_t)Cp * CO_KB;
  // staging: chunk q = threadIdx.x + i NT of [A tile | B tile]; its row and half, swizzled LDS offset
  const int8_t* gsrc[LPT];
  int soff[LPT];
#pragma unroll
  for (int i = 0; i < LPT; i++) {
    const int q = threadIdx.x + i * NT;
    const int isb = q >= OPB / 16, qq = isb ? q - OPB / 16 : q;
    const int row = qq >> 1, half = qq & 1;
    gsrc[i] = X + (size_t)((isb ? tx : ty) * TILE + row) * CO_KB + 16 * half;
    soff[i] = isb * OPB + row * CO_KB + 16 * (half ^ ((row >> 3) & 1));
  }
  // operand reads: lane l takes half (l >> 5) of row (l & 31) of a 32-row block
  const int lrow = lane & 31, lhalf = lane >> 5;
  int aoff[2], boff[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int ra = wr + 32 * i + lrow, rb = wc + 32 * i + lrow;
    aoff[i] = ra * CO_KB + 16 * (lhalf ^ ((ra >> 3) & 1));
    boff[i] = OPB + rb * CO_KB + 16 * (lhalf ^ ((rb >> 3) & 1));
  }
  v16i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) acc[i][j] = v16i{};
  // KPB K blocks per stage (one barrier per stage); loads past the range's last block re-read it and
  // their MFMAs are branched around
  if (kb0 < kb1) {
    const uint32_t klast = kb1 - 1;
    v4i g[KPB][LPT];
#pragma unroll
    for (int q = 0; q < KPB; q++)
#pragma unroll
      for (int i = 0; i < LPT; i++)
        g[q][i] = *reinterpret_cast<const v4i*>(gsrc[i] + (size_t)min(kb0 + q, klast) * kstride);
    int cur = 0;
    for (uint32_t kb = kb0; kb < kb1; kb += KPB) {
#pragma unroll
      for (int q = 0; q < KPB; q++)
#pragma unroll
        for (int i = 0; i < LPT; i++) *reinterpret_cast<v4i*>(&sm[cur][q][soff[i]]) = g[q][i];
      __syncthreads();
#pragma unroll
      for (int q = 0; q < KPB; q++)
#pragma unroll
        for (int i = 0; i < LPT; i++)
          g[q][i] = *reinterpret_cast<const v4i*>(gsrc[i] + (size_t)min(kb + KPB + q, klast) * kstride);
#pragma unroll
      for (int q = 0; q < KPB; q++) {
        if (kb + q >= kb1) break;
        const v4i a0 = *reinterpret_cast<const v4i*>(&sm[cur][q][aoff[0]]);
        const v4i a1 = *reinterpret_cast<const v4i*>(&sm[cur][q][aoff[1]]);
        const v4i b0 = *reinterpret_cast<const v4i*>(&sm[cur][q][boff[0]]);
        const v4i b1 = *reinterpret_cast<const v4i*>(&sm[cur][q][boff[1]]);
        acc[0][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, acc[1][1], 0, 0, 0);
      }
      cur ^= 1;
    }
  }
  co_store_partial<TILE>(acc, P, ((size_t)kg * tiles + tid) * TILE * TILE, wr, wc, lane);
}

// A K range's partial cells are exact int32 while the range's sum of len^2 stays below 2^31 (every
// cell adds at most len^2 per program); err 4 otherwise (the caller gets an error, never a wrapped count)
__global__ void k_co_ranges(const unsigned long long* kbound, uint32_t nkb, uint32_t ks, uint32_t kb_per, int* err) {
  for (uint32_t kg = blockIdx.x * blockDim.x + threadIdx.x; kg < ks; kg += gridDim.x * blockDim.x) {
    unsigned long long t = 0;
    for (uint32_t kb = kg * kb_per; kb < nkb && kb < (kg + 1) * kb_per; kb++) t += kbound[kb];
    if (t >= (1ull << 31)) atomicOr(err, 4);
  }
}

// out[row][col] = the sum of the KS partials of (row, col), minus the occurrences of row on the
// diagonal, summed in int64 (err 8 when it leaves int32); one thread per element of an upper-triangle
// tile, which writes the element and, off the diagonal tiles, its transpose (so every element of out
// is written exactly once)
__global__ __launch_bounds__(256) void k_co_reduce(const int* __restrict__ P, uint32_t tiles, uint32_t ks,
                                                   uint32_t T, uint32_t tile, int32_t C,
                                                   const unsigned long long* __restrict__ occ, int* __restrict__ out,
                                                   int* err) {
  uint32_t t = blockIdx.x;
  const uint32_t e = blockIdx.y * blockDim.x + threadIdx.x;
  const size_t tt = (size_t)tile * tile;
  const size_t base = (size_t)t * tt + e;
  uint32_t ty = 0;
  while (t >= T - ty) t -= T - ty++;
  const uint32_t tx = ty + t;
  const uint32_t row = ty * tile + e / tile, col = tx * tile + e % tile;
  if ((int32_t)row >= C || (int32_t)col >= C) return;
  long long v = 0;
  for (uint32_t kg = 0; kg < ks; kg++) v += P[(size_t)kg * tiles * tt + base];
  if (row == col) v -= (long long)occ[row];
  if (v > 0x7FFFFFFFll || v < -0x80000000ll) atomicOr(err, 8);
  out[(size_t)row * C + col] = (int)v;
  if (tx != ty) out[(size_t)col * C + row] = (int)v;
}

// SYZGPU_CO_KS=k forces the K split (tests; read on every call)
static uint32_t co_splits() {
  const char* e = getenv("SYZGPU_CO_KS");
  return e && *e ? (uint32_t)std::max(1, atoi(e)) : 0u;
}

// A/B knob, read on every call: SYZGPU_CO_FORM=0 the direct form (per-wave operand loads, TA-bound:
// profiles/r02_ab/cooccur_ab.md), 1 (default) the LDS-staged form
static int co_env(const char* name, int def, int lo, int hi) {
  const char* e = getenv(name);
  return e && *e ? std::min(hi, std::max(lo, atoi(e))) : def;
}

// out (C x C int32, device) = the call-ID co-occurrence of the programs' call lists (device CSR)
void call_cooccurrence_dev(const uint16_t* calls, const uint64_t* off, size_t n, int32_t C, int32_t* out,
                           hipStream_t s) {
  if (C <= 0 || C > 16384) fail(SYZGPU_EINVAL, "C out of range");
  if (!out || (n && !off)) fail(SYZGPU_EINVAL, "null pointer");
  Context& c = ctx();
  Scratch& sc = c.scratch;
  const uint32_t Cp = ((uint32_t)C + 255) / 256 * 256;  // rows per K block: a multiple of every tile size
  const uint32_t nkb = (uint32_t)((n + CO_KB - 1) / CO_KB);
  const size_t xbytes = (size_t)std::max<uint32_t>(nkb, 1) * Cp * CO_KB;
  uint32_t* Xw = sc.get<uint32_t>("co_x", xbytes / 4 + 1);
  unsigned long long* occ = sc.get<unsigned long long>("co_occ", (size_t)C + 1);
  unsigned long long* kbound = sc.get<unsigned long long>("co_kbound", (size_t)nkb + 1);
  int* err = sc.get<int>("co_err", 2);
  SYZ_HIP(hipMemsetAsync(err, 0, 8, s));
  SYZ_HIP(hipMemsetAsync(kbound, 0, ((size_t)nkb + 1) * 8, s));
  SYZ_HIP(hipMemsetAsync(occ, 0, ((size_t)C + 1) * 8, s));
  {
    ProfScope ps("cooc_build", s, xbytes);
    SYZ_HIP(hipMemsetAsync(Xw, 0, xbytes, s));
    if (n) {
      k_co_build<<<grid_for(n, 256, 1024), 256, (size_t)C * 4, s>>>(calls, off, n, C, Cp, Xw, occ, kbound, err);
      SYZ_LAUNCHED();
    }
  }
  {
    // K split: about two workgroups per CU (all resident at once), in multiples of 8 K ranges (one
    // set of ranges per XCD) once there are enough K blocks for that
    if (!c.ncu) SYZ_HIP(hipDeviceGetAttribute(&c.ncu, hipDeviceAttributeMultiprocessorCount, c.device));
    const int form = co_env("SYZGPU_CO_FORM", 1, 0, 1);
    const uint32_t tile = CO_TILE;
    const uint32_t T = Cp / tile, tiles = T * (T + 1) / 2;
    uint32_t ks = co_splits();
    if (!ks) {
      ks = std::max<uint32_t>(1, std::min<uint32_t>(std::max<uint32_t>(nkb, 1), (2u * c.ncu + tiles - 1) / tiles));
      if (nkb >= 64) ks = std::min<uint32_t>((ks + 7) / 8 * 8, nkb / 8 * 8);
    }
    // the partial tiles stay within 2 GiB
    ks = std::min<uint32_t>(ks, std::max<uint64_t>(1, (1ull << 29) / ((uint64_t)tiles * tile * tile)));
    const uint32_t kb_per = (std::max<uint32_t>(nkb, 1) + ks - 1) / ks;
    const int8_t* Xb = reinterpret_cast<const int8_t*>(Xw);
    int* P = sc.get<int>("co_part", (size_t)ks * tiles * tile * tile);
    {
    ProfScope ps("cooc_gemm", s, 2ull * C * C * (uint64_t)nkb * CO_KB);  // (ops, not bytes)
    if (form == 1)
      k_co_gemm_lds<128, 2><<<tiles * ks, 256, 0, s>>>(Xb, C, Cp, T, tiles, ks, nkb, kb_per, P);
    else
      k_co_gemm<1><<<tiles * ks, 256, 0, s>>>(Xb, C, Cp, T, tiles, ks, nkb, kb_per, P);
    SYZ_LAUNCHED();
    }
    ProfScope ps("cooc_reduce", s, (uint64_t)ks * tiles * tile * tile * 4 + (uint64_t)C * C * 4);
    k_co_ranges<<<grid_for(ks, 256, 64), 256, 0, s>>>(kbound, nkb, ks, kb_per, err);
    SYZ_LAUNCHED();
    k_co_reduce<<<dim3(tiles, tile * tile / 256), 256, 0, s>>>(P, tiles, ks, T, tile, C, occ, out, err);
    SYZ_LAUNCHED();
  }
  int* h = c.pinned.get<int>(2);
  SYZ_HIP(hipMemcpyAsync(h, err, 4, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (h[0] & 1) fail(SYZGPU_EINVAL, "call id >= C");
  if (h[0] & 2) fail(SYZGPU_EINVAL, "a call occurs more than 127 times in one program (int8 operand)");
  if (h[0] & 4) fail(SYZGPU_EINVAL, "a K range's sum of len^2 reaches 2^31: its int32 partial counts could wrap");
  if (h[0] & 8) fail(SYZGPU_EINVAL, "a co-occurrence count exceeds int32");
}

}  // namespace syz

extern "C" int syzgpu_call_cooccurrence_dev(const uint16_t* calls, const uint64_t* off, size_t n, int32_t C,
                                            int32_t* out, void* stream) {
  SYZ_API_BODY({ syz::call_cooccurrence_dev(calls, off, n, C, out, (hipStream_t)stream); })
}

extern "C" int syzgpu_call_cooccurrence(const uint16_t* calls, const uint64_t* off, size_t n, int32_t C,
                                        int32_t* out) {
  SYZ_API_BODY({
    if (!off || !out) syz::fail(SYZGPU_EINVAL, "null pointer");
    if (off[0] != 0) syz::fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
    for (size_t i = 0; i < n; i++)
      if (off[i + 1] < off[i]) syz::fail(SYZGPU_EINVAL, "CSR offsets must be non-decreasing");
    if (C <= 0 || C > 16384) syz::fail(SYZGPU_EINVAL, "C out of range");
    syz::Context& c = syz::ctx();
    hipStream_t s = c.stream;
    const uint64_t L = off[n];
    uint16_t* dc = c.scratch.get<uint16_t>("co_calls", L + 1);
    uint64_t* doff = c.scratch.get<uint64_t>("co_off", n + 1);
    int32_t* dout = c.scratch.get<int32_t>("co_out", (size_t)C * C + 1);
    if (L) SYZ_HIP(hipMemcpyAsync(dc, calls, L * 2, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(doff, off, (n + 1) * 8, hipMemcpyHostToDevice, s));
    syz::call_cooccurrence_dev(dc, doff, n, C, dout, s);
    SYZ_HIP(hipMemcpyAsync(out, dout, (size_t)C * C * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

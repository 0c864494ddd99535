// calcStaticPriorities (prog/prio.go:40-135) on the int8 matrix cores.
//
// The Go code keeps, per usage key (resource kind, pointed-to struct, string sub-kind, filename, vma,
// signalno), the largest weight each call uses it with (prio.go:41-104), then adds w0*w1 into
// prios[c0][c1] for every key and every pair of distinct calls using it (:110-120): a Gram matrix
// WᵀW over the key-by-call weight matrix W, minus its diagonal. The weights come from a handful of
// constants (0.1, 0.2, 0.5, 1.0), so the sum factors exactly:
//
//     prios[c0][c1] = sum over weight classes (a, b) of  n_ab[c0][c1] * float32(w_a * w_b)
//     n_ab[c0][c1]  = #{keys k : W[k][c0] = w_a and W[k][c1] = w_b}
//
// Each n_ab is an integer Gram matrix of 0/1 class indicators: int8 MFMA (v_mfma_i32_32x32x32_i8)
// with int32 accumulation, exact. The class pairs are combined in float64 (every n * w product is
// exact; the <= 64 terms are added in a fixed order) and rounded once to float32. Go instead adds the
// float32 products in its map's iteration order, which Go randomises per run, so its own results
// differ between runs in the last bits; this sum is the one every such order approximates, within
// float32 rounding of the summands (tests/test_gpu_static_prio.py states and checks the bound).
// Self-priority is the row maximum (:124-132) and normalizePrio (:158-192) follows, both in
// prio.hip's row kernel with Go's separate float32 roundings.
//
//   K1 k_st_classes  distinct non-zero weights (at most ST_KMAX) into a small table (atomicCAS)
//   K2 k_st_prep     one thread: classes sorted ascending, the float32 products of every class pair
//   K3 k_st_pack     indicator matrices X[a][c][k] = (W[k][c] == w_a), int8, 32-padded
//   K4 k_st_gram     one 4-wave workgroup per 32x32 tile of calls: MFMA over keys per class pair,
//                    counts through LDS, float64 combination in (a, b) order, the C x C float32 sums
//                    (diagonal 0)
//   K5 k_prio_row    (prio.hip, mode 2) diagonal := row max, normalizePrio, in place
#include <cmath>

#include "pipeline.hpp"

namespace syz {

constexpr int ST_KMAX = 8;  // distinct non-zero weights (calcStaticPriorities uses 4)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

struct StClasses {
  uint32_t nk;
  uint32_t err;   // 1: more than ST_KMAX weights, 2: a non-finite weight
  float w[ST_KMAX];
  double prod[ST_KMAX][ST_KMAX];
};

__global__ __launch_bounds__(256) void k_st_classes(const float* __restrict__ uses, size_t n, uint32_t* tab,
                                                    uint32_t* err) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float w = uses[i];
    if (w == 0.0f) continue;
    if (!isfinite(w)) {
      atomicOr(err, 2u);
      continue;
    }
    const uint32_t bits = __float_as_uint(w);
    int s = 0;
    for (; s < ST_KMAX; s++) {
      const uint32_t t = tab[s];
      if (t == bits) break;
      if (t == 0u) {
        const uint32_t old = atomicCAS(&tab[s], 0u, bits);
        if (old == 0u || old == bits) break;
      }
    }
    if (s == ST_KMAX) atomicOr(err, 1u);
  }
}

__global__ void k_st_prep(const uint32_t* tab, const uint32_t* err, StClasses* cl) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float w[ST_KMAX];
  uint32_t nk = 0;
  for (int s = 0; s < ST_KMAX; s++)
    if (tab[s]) w[nk++] = __uint_as_float(tab[s]);
  for (uint32_t i = 1; i < nk; i++)  // ascending: the class pairs are added in a fixed order
    for (uint32_t j = i; j > 0 && w[j - 1] > w[j]; j--) {
      const float t = w[j];
      w[j] = w[j - 1];
      w[j - 1] = t;
    }
  cl->nk = nk;
  cl->err = *err;
  for (uint32_t a = 0; a < ST_KMAX; a++) {
    cl->w[a] = a < nk ? w[a] : 0.0f;
    for (uint32_t b = 0; b < ST_KMAX; b++) {
      const float p = (a < nk && b < nk) ? w[a] * w[b] : 0.0f;  // Go's float32 w0 * w1
      cl->prod[a][b] = (double)p;
    }
  }
}

// X[a][c][k] over a x Cp x Kp bytes: one thread per (class, call, 16 keys); threads of a wave take
// consecutive calls, so the W reads (row k, columns c..c+63) coalesce
__global__ __launch_bounds__(256) void k_st_pack(const float* __restrict__ uses, uint32_t nkeys, int32_t C,
                                                 uint32_t Cp, uint32_t Kp, const StClasses* cl, int8_t* X) {
  const uint32_t nk = cl->nk;
  const uint64_t total = (uint64_t)nk * Cp * (Kp / 16);
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = (uint32_t)(t % Cp);
    const uint64_t r = t / Cp;
    const uint32_t k0 = (uint32_t)(r % (Kp / 16)) * 16;
    const uint32_t a = (uint32_t)(r / (Kp / 16));
    const float wa = cl->w[a];
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t k = k0 + j;
      const bool on = (int32_t)c < C && k < nkeys && uses[(size_t)k * C + c] == wa;
      v[j >> 2] |= (on ? 1u : 0u) << (8 * (j & 3));
    }
    *reinterpret_cast<uint4*>(X + ((size_t)a * Cp + c) * Kp + k0) = make_uint4(v[0], v[1], v[2], v[3]);
  }
}

// One 4-wave workgroup per 32x32 tile (rows c0.., columns c1..). The class pairs (a, b) go in groups
// of 16, four per wave, two MFMA chains interleaved; a pair's integer counts n_ab land in LDS, then every
// thread adds n_ab * w_a w_b for its four entries of the tile over the group's pairs in (a, b) order
// (float64, exact products), so the sum is the one-pair-at-a-time sum in that fixed order.
// Operands: lane l holds 16 consecutive keys [16 (l >> 5), +16) of call (l & 31) of the tile, for A
// (rows, class a) and B (columns, class b) alike, so whatever order the instruction gives the 32 keys
// of a step inside its K, A and B agree on it and the step sums the 32 keys. Result registers: column
// l & 31, row (r & 3) + 8 (r >> 2) + 4 (l >> 5) (the gfx950 32x32 C/D map).
// (One wave per tile doing every pair one after another took 75 us at config 1: load latency, chain
// after chain.)
constexpr int ST_GP = 16;  // pairs per LDS group
__global__ __launch_bounds__(256) void k_st_gram(const int8_t* __restrict__ X, int32_t C, uint32_t Cp, uint32_t Kp,
                                                 const StClasses* __restrict__ cl, float* __restrict__ prios) {
  __shared__ int32_t cnt[ST_GP][32 * 32];
  const uint32_t c0 = blockIdx.y * 32, c1 = blockIdx.x * 32;
  const unsigned lane = __lane_id();
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t nk = cl->nk, np = nk * nk;
  const size_t koff = 16 * (lane >> 5);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};  // entries threadIdx.x + 256 e of the tile
  auto chain2 = [&](uint32_t p0, uint32_t p1, v16i& n0, v16i& n1) {
    const int8_t* xa0 = X + ((size_t)(p0 / nk) * Cp + c0 + (lane & 31)) * Kp + koff;
    const int8_t* xb0 = X + ((size_t)(p0 % nk) * Cp + c1 + (lane & 31)) * Kp + koff;
    const uint32_t q1 = p1 < np ? p1 : p0;
    const int8_t* xa1 = X + ((size_t)(q1 / nk) * Cp + c0 + (lane & 31)) * Kp + koff;
    const int8_t* xb1 = X + ((size_t)(q1 % nk) * Cp + c1 + (lane & 31)) * Kp + koff;
    n0 = v16i{};
    n1 = v16i{};
#pragma unroll 4
    for (uint32_t k = 0; k < Kp; k += 32) {
      const v4i a0 = *reinterpret_cast<const v4i*>(xa0 + k);
      const v4i b0 = *reinterpret_cast<const v4i*>(xb0 + k);
      const v4i a1 = *reinterpret_cast<const v4i*>(xa1 + k);
      const v4i b1 = *reinterpret_cast<const v4i*>(xb1 + k);
      n0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, n0, 0, 0, 0);
      n1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, n1, 0, 0, 0);
    }
  };
  auto put = [&](uint32_t slot, const v16i& n) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const uint32_t row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      cnt[slot][row * 32 + (lane & 31)] = n[r];
    }
  };
  for (uint32_t g0 = 0; g0 < np; g0 += ST_GP) {
    for (uint32_t q = 0; q < 4; q += 2) {
      const uint32_t p0 = g0 + 4 * wv + q;
      if (p0 >= np) break;
      v16i n0, n1;
      chain2(p0, p0 + 1, n0, n1);
      put(4 * wv + q, n0);
      if (p0 + 1 < np) put(4 * wv + q + 1, n1);
    }
    __syncthreads();
    const uint32_t gn = min<uint32_t>(ST_GP, np - g0);
    for (uint32_t j = 0; j < gn; j++) {  // (a, b) order
      const double pr = cl->prod[(g0 + j) / nk][(g0 + j) % nk];
#pragma unroll
      for (int e = 0; e < 4; e++) acc[e] += (double)cnt[j][threadIdx.x + 256 * e] * pr;  // exact product
    }
    __syncthreads();
  }
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const uint32_t i = threadIdx.x + 256 * e;
    const uint32_t row = c0 + i / 32, col = c1 + i % 32;
    if ((int32_t)row < C && (int32_t)col < C) prios[(size_t)row * C + col] = row == col ? 0.0f : (float)acc[e];
  }
}

void static_prio_rows_dev(float* prios, int32_t C, hipStream_t s);  // prio.hip

// prios = calcStaticPriorities() of the usage matrix (device pointers), enqueued on s; returns the device
// word whose bits static_prio_check reads (after s has run)
const uint32_t* static_priorities_enqueue(const float* uses, size_t nkeys, int32_t C, float* prios, hipStream_t s) {
  if (C <= 0 || C > 16384) fail(SYZGPU_EINVAL, "C out of range");
  if (nkeys >= (1u << 24)) fail(SYZGPU_EINVAL, "too many usage keys");
  if (!prios || (nkeys && !uses)) fail(SYZGPU_EINVAL, "null pointer");
  Context& c = ctx();
  Scratch& sc = c.scratch;
  const uint32_t Cp = ((uint32_t)C + 31) / 32 * 32;
  const uint32_t Kp = std::max<uint32_t>(32, ((uint32_t)nkeys + 31) / 32 * 32);
  uint32_t* tab = sc.get<uint32_t>("st_tab", ST_KMAX + 2);
  StClasses* cl = sc.get<StClasses>("st_classes", 1);
  int8_t* X = sc.get<int8_t>("st_x", (size_t)ST_KMAX * Cp * Kp);
  ProfScope ps("static_prio", s, (uint64_t)nkeys * C * 4 + (uint64_t)C * C * 8);
  SYZ_HIP(hipMemsetAsync(tab, 0, (ST_KMAX + 2) * 4, s));
  const size_t n = nkeys * (size_t)C;
  if (n) {
    k_st_classes<<<grid_for(n, 256, 1024), 256, 0, s>>>(uses, n, tab, tab + ST_KMAX);
    SYZ_LAUNCHED();
  }
  k_st_prep<<<1, 64, 0, s>>>(tab, tab + ST_KMAX, cl);
  SYZ_LAUNCHED();
  const uint64_t packs = (uint64_t)ST_KMAX * Cp * (Kp / 16);  // an upper bound (nk <= ST_KMAX)
  k_st_pack<<<grid_for(packs, 256, 8192), 256, 0, s>>>(uses, (uint32_t)nkeys, C, Cp, Kp, cl, X);
  SYZ_LAUNCHED();
  k_st_gram<<<dim3(Cp / 32, Cp / 32), 256, 0, s>>>(X, C, Cp, Kp, cl, prios);
  SYZ_LAUNCHED();
  static_prio_rows_dev(prios, C, s);
  return &cl->err;
}

void static_prio_check(uint32_t err) {
  if (err & 2) fail(SYZGPU_EINVAL, "non-finite usage weight");
  if (err & 1) fail(SYZGPU_EINVAL, "more than 8 distinct usage weights");
}

// the same, returning after the error check
void static_priorities_dev(const float* uses, size_t nkeys, int32_t C, float* prios, hipStream_t s) {
  const uint32_t* derr = static_priorities_enqueue(uses, nkeys, C, prios, s);
  uint32_t* h = ctx().pinned.get<uint32_t>(4);
  SYZ_HIP(hipMemcpyAsync(h, derr, 4, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  static_prio_check(h[0]);
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzgpu_static_priorities(const float* uses, size_t nkeys, int32_t C, float* prios) {
  SYZ_API_BODY({
    if (C <= 0 || C > 16384) fail(SYZGPU_EINVAL, "C out of range");
    if (!prios || (nkeys && !uses)) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    const size_t n = nkeys * (size_t)C, CC = (size_t)C * C;
    float* du = C_.scratch.get<float>("sth_uses", n + 1);
    float* dp = C_.scratch.get<float>("sth_prios", CC);
    if (n) SYZ_HIP(hipMemcpyAsync(du, uses, n * 4, hipMemcpyHostToDevice, s));
    static_priorities_dev(du, nkeys, C, dp, s);
    SYZ_HIP(hipMemcpyAsync(prios, dp, CC * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_static_priorities_dev(const float* uses, size_t nkeys, int32_t C, float* prios, void* stream) {
  SYZ_API_BODY({ static_priorities_dev(uses, nkeys, C, prios, (hipStream_t)stream); })
}

}  // extern "C"

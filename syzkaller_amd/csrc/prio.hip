// Dynamic call priorities and the ChoiceTable — prog/prio.go:29-38, 137-192, 202-228.
//
// calcDynamicPrio adds 1.0 for every ordered pair of call *positions* (i0 != i1) of every corpus
// program (prio.go:142-150), so before normalisation
//     dyn[i][j] = float32(min(H(max(i, j)), 2^24)),  i != j;   dyn[i][i] = 0
// with H(k) = #{p : len(p.Calls) > k}: float32 += 1.0 is exact up to 2^24 and then sticks (ties-to-
// even), independent of the order of the adds. A corpus therefore reduces to a histogram of program
// lengths (C+1 int64 — the only data multi-GPU runs exchange). One workgroup per row then does
// normalizePrio (prio.go:158-192) with every float32 op rounded separately (built with
// -ffp-contract=off and IEEE division), the *= static multiply (prio.go:32-36), and the ChoiceTable
// row: run[i][j] = sum over enabled j' <= j of int(prios[i][j'] * 1000) (prio.go:219-225), using Go's
// amd64 float->int conversion (truncation; NaN/out of range -> INT64_MIN) and wrapping int64 sums.
#include <cmath>

#include "pipeline.hpp"

namespace syz {

constexpr int PR_BLOCK = 256;
constexpr int32_t MAX_C = 16384;

__global__ __launch_bounds__(256) void k_len_hist(const uint16_t* prog_len, const uint8_t* sel, size_t n, int32_t C,
                                                  int64_t* hist, int* err) {
  extern __shared__ unsigned long long lh[];
  for (int32_t i = threadIdx.x; i <= C; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  for (size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (size_t)gridDim.x * blockDim.x) {
    if (sel && !sel[r]) continue;
    const int32_t L = prog_len[r];
    if (L > C)
      atomicOr(err, 2);
    else
      atomicAdd(&lh[L], 1ull);
  }
  __syncthreads();
  for (int32_t i = threadIdx.x; i <= C; i += blockDim.x)
    if (lh[i]) atomicAdd((unsigned long long*)&hist[i], lh[i]);
}

// H(k) = sum_{L > k} hist[L], clamped to 2^24 (the float32 accumulator's fixed point), as float, for
// k in [k0, C): a row block of k_prio_row only reads H(max(i, j)) >= H(i), so it builds [i, C) alone.
__device__ __forceinline__ void block_suffix(const int64_t* hist, int32_t C, float* Hf, int64_t* red, int32_t k0 = 0) {
  // process from k0 up: H(k) = total - sum_{k0 < L <= k} hist[L], total = sum_{L > k0} hist[L]
  int64_t carry = 0;
  int64_t total = 0;
  for (int32_t base = k0 + 1; base <= C; base += PR_BLOCK) {
    const int32_t i = base + threadIdx.x;
    total += i <= C ? hist[i] : 0;
  }
  total = block_sum<PR_BLOCK>(total, red);
  for (int32_t base = k0; base < C; base += PR_BLOCK) {
    const int32_t k = base + threadIdx.x;
    const int64_t v = k < C && k > k0 ? hist[k] : 0;
    int64_t tot;
    const int64_t incl = block_excl_scan<PR_BLOCK>(v, red, &tot) + v + carry;
    if (k < C) {
      int64_t H = total - incl;
      if (H > (1ll << 24)) H = 1ll << 24;
      Hf[k] = (float)H;
    }
    carry += tot;
  }
}

__global__ __launch_bounds__(PR_BLOCK) void k_suffix(const int64_t* hist, int32_t C, float* Hf) {
  __shared__ int64_t red[PR_BLOCK / 64 + 1];
  block_suffix(hist, C, Hf, red);
}

__device__ __forceinline__ int64_t go_f32_to_int(float x) {
  if (x != x) return INT64_MIN;
  if (x >= 9223372036854775808.0f || x < -9223372036854775808.0f) return INT64_MIN;
  return (int64_t)x;
}

// mode 0: dynamic from Hf (+ optional static multiply); mode 1: prios given (ChoiceTable only);
// mode 2: calcStaticPriorities' tail on the pair sums in prios_in (static_prio.hip): the diagonal
// becomes the row's maximum (prio.go:124-132), then normalizePrio, written to prios_out (may alias).
// mode 0 with hist: every row block builds H(k), k >= its row, in LDS itself (no separate suffix launch
// on the step's critical path; the same integer sums, so the same floats)
__global__ __launch_bounds__(PR_BLOCK) void k_prio_row(int mode, const float* Hf, const float* static_prios,
                                                       const float* prios_in, int32_t C, const uint8_t* enabled,
                                                       float* prios_out, int64_t* run, uint8_t* present,
                                                       const int64_t* hist) {
  extern __shared__ float Hs[];
  __shared__ int64_t sred[PR_BLOCK / 64 + 1];
  if (mode == 0 && hist) {
    block_suffix(hist, C, Hs, sred, (int32_t)blockIdx.x);
    __syncthreads();
    Hf = Hs;
  }
  __shared__ float rmax[PR_BLOCK / 64 + 1];
  __shared__ float rmin[PR_BLOCK / 64 + 1];
  __shared__ int32_t rnz[PR_BLOCK / 64 + 1];
  __shared__ uint64_t red[PR_BLOCK / 64 + 1];
  const int32_t i = blockIdx.x;
  const size_t row = (size_t)i * C;
  const int w = threadIdx.x >> 6;
  float mx = 0.0f, mn = 1e10f;
  float dg = 0.0f;  // mode 2: the self-priority
  if (mode == 2) {
    float m = 0.0f;  // var max float32; if max < p { max = p } over the whole row (its diagonal is 0)
    for (int32_t j = threadIdx.x; j < C; j += PR_BLOCK) {
      const float p = prios_in[row + j];
      if (m < p) m = p;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const float o = __shfl_xor(m, d, 64);
      m = o > m ? o : m;
    }
    if (__lane_id() == 0) rmax[w] = m;
    __syncthreads();
    for (int k = 0; k < PR_BLOCK / 64; k++) dg = rmax[k] > dg ? rmax[k] : dg;
    __syncthreads();
  }
  auto in_p = [&](int32_t j) -> float {
    if (mode == 0) return (j == i) ? 0.0f : Hf[j > i ? j : i];
    return (j == i) ? dg : prios_in[row + j];
  };
  if (mode != 1) {
    // row statistics of normalizePrio: max, min over non-zero, number of zeros (prio.go:160-173)
    int32_t nz = 0;
    for (int32_t j = threadIdx.x; j < C; j += PR_BLOCK) {
      const float p = in_p(j);
      if (mx < p) mx = p;
      if (p != 0 && mn > p) mn = p;
      if (p == 0) nz++;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const float omx = __shfl_xor(mx, d, 64), omn = __shfl_xor(mn, d, 64);
      mx = omx > mx ? omx : mx;
      mn = omn < mn ? omn : mn;
      nz += __shfl_xor(nz, d, 64);
    }
    if (__lane_id() == 0) {
      rmax[w] = mx;
      rmin[w] = mn;
      rnz[w] = nz;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float a = rmax[0], b = rmin[0];
      int32_t z = rnz[0];
      for (int k = 1; k < PR_BLOCK / 64; k++) {
        a = rmax[k] > a ? rmax[k] : a;
        b = rmin[k] < b ? rmin[k] : b;
        z += rnz[k];
      }
      if (z != 0) {
        const float den = 2.0f * (float)z;  // min /= 2 * float32(nzero)
        b = b / den;
      }
      rmax[PR_BLOCK / 64] = a;
      rmin[PR_BLOCK / 64] = b;
    }
    __syncthreads();
    mx = rmax[PR_BLOCK / 64];
    mn = rmin[PR_BLOCK / 64];
  }
  const bool row_on = !enabled || enabled[i];
  if (present) present[i] = row_on ? 1 : 0;
  uint64_t carry = 0;
  for (int32_t base = 0; base < C; base += PR_BLOCK) {
    const int32_t j = base + threadIdx.x;
    float p = 0.0f;
    if (j < C) {
      if (mode != 1) {
        p = in_p(j);
        if (mx == 0) {
          p = 1.0f;
        } else {
          if (p == 0) p = mn;
          const float t1 = p - mn;
          const float t2 = mx - mn;
          const float t3 = t1 / t2;
          const float t4 = t3 * 0.9f;
          p = t4 + 0.1f;
          if (p > 1) p = 1.0f;
        }
        if (static_prios) p = p * static_prios[row + j];
        if (prios_out) prios_out[row + j] = p;
      } else {
        p = prios_in[row + j];
      }
    }
    if (run) {
      uint64_t t = 0;
      if (j < C && row_on && (!enabled || enabled[j])) t = (uint64_t)go_f32_to_int(p * 1000.0f);
      uint64_t tot;
      const uint64_t incl = block_excl_scan<PR_BLOCK>(t, red, &tot) + t + carry;
      if (j < C) run[row + j] = row_on ? (int64_t)incl : 0;
      carry += tot;
    }
  }
}

void static_prio_rows_dev(float* prios, int32_t C, hipStream_t s) {
  k_prio_row<<<C, PR_BLOCK, 0, s>>>(2, nullptr, nullptr, prios, C, nullptr, prios, nullptr, nullptr, nullptr);
  SYZ_LAUNCHED();
}

void len_hist_dev(const uint16_t* prog_len, const uint8_t* sel, size_t n, int32_t C, int64_t* hist, int* err,
                  hipStream_t s) {
  SYZ_HIP(hipMemsetAsync(hist, 0, (size_t)(C + 1) * 8, s));
  if (n) {
    k_len_hist<<<grid_for(n, 256, 2048), 256, (size_t)(C + 1) * 8, s>>>(prog_len, sel, n, C, hist, err);
    SYZ_LAUNCHED();
  }
}

void prio_choice_dev(const float* static_prios, const int64_t* len_hist, const float* prios_in, int32_t C,
                     const uint8_t* enabled, float* prios_out, int64_t* run, uint8_t* present, hipStream_t s) {
  if (C <= 0 || C > MAX_C) fail(SYZGPU_EINVAL, "C out of range");
  if (prios_in) {
    ProfScope ps("choice_table", s, (uint64_t)C * C * 12);
    k_prio_row<<<C, PR_BLOCK, 0, s>>>(1, nullptr, nullptr, prios_in, C, enabled, nullptr, run, present, nullptr);
    SYZ_LAUNCHED();
    return;
  }
  // SYZGPU_PRIO_SUFFIX=1: the suffix sums as their own launch (A/B reference)
  static const bool sep = dev_env("SYZGPU_PRIO_SUFFIX") != nullptr;
  float* Hf = nullptr;
  if (sep) {
    Hf = ctx().scratch.get<float>("pr_H", C + 1);
    ProfScope ps("prio_suffix", s, (uint64_t)(C + 1) * 12);
    k_suffix<<<1, PR_BLOCK, 0, s>>>(len_hist, C, Hf);
    SYZ_LAUNCHED();
  }
  ProfScope ps("prio_choice", s, (uint64_t)C * C * ((static_prios ? 4 : 0) + (prios_out ? 4 : 0) + (run ? 8 : 0)));
  k_prio_row<<<C, PR_BLOCK, sep ? 0 : (size_t)C * 4, s>>>(0, Hf, static_prios, nullptr, C, enabled, prios_out, run,
                                                          present, sep ? nullptr : len_hist);
  SYZ_LAUNCHED();
}

}  // namespace syz

using namespace syz;

namespace {

int prio_host(const float* static_prios, const uint16_t* prog_len, size_t nprogs, int32_t C, float* out) {
  SYZ_API_BODY({
    if (C <= 0 || C > MAX_C) fail(SYZGPU_EINVAL, "C out of range");
    if (!out || (nprogs && !prog_len)) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    const size_t CC = (size_t)C * C;
    uint16_t* dl = C_.scratch.get<uint16_t>("ph_len", nprogs + 1);
    int64_t* hist = C_.scratch.get<int64_t>("ph_hist", C + 1);
    int* err = C_.scratch.get<int>("ph_err", 2);
    float* dst = static_prios ? C_.scratch.get<float>("ph_static", CC) : nullptr;
    float* dout = C_.scratch.get<float>("ph_out", CC);
    SYZ_HIP(hipMemsetAsync(err, 0, 8, s));
    if (nprogs) SYZ_HIP(hipMemcpyAsync(dl, prog_len, nprogs * 2, hipMemcpyHostToDevice, s));
    if (dst) SYZ_HIP(hipMemcpyAsync(dst, static_prios, CC * 4, hipMemcpyHostToDevice, s));
    len_hist_dev(dl, nullptr, nprogs, C, hist, err, s);
    int* herr = C_.pinned.get<int>(4);
    SYZ_HIP(hipMemcpyAsync(herr, err, 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (*herr) fail(SYZGPU_EINVAL, "len(p.Calls) > C (prog/prio.go:148 would panic)");
    prio_choice_dev(dst, hist, nullptr, C, nullptr, dout, nullptr, nullptr, s);
    SYZ_HIP(hipMemcpyAsync(out, dout, CC * 4, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

}  // namespace

extern "C" {

int syzgpu_dynamic_prio(const uint16_t* prog_len, size_t nprogs, int32_t C, float* out) {
  return prio_host(nullptr, prog_len, nprogs, C, out);
}

int syzgpu_calculate_priorities(const float* static_prios, const uint16_t* prog_len, size_t nprogs, int32_t C,
                                float* out) {
  if (!static_prios) return SYZGPU_EINVAL;
  return prio_host(static_prios, prog_len, nprogs, C, out);
}

int syzgpu_build_choice_table(const float* prios, const uint8_t* enabled, int32_t C, int64_t* run,
                              uint8_t* row_present) {
  SYZ_API_BODY({
    if (C <= 0 || C > MAX_C) fail(SYZGPU_EINVAL, "C out of range");
    if (!prios || !run || !row_present) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    const size_t CC = (size_t)C * C;
    float* dp = C_.scratch.get<float>("ct_prios", CC);
    int64_t* drun = C_.scratch.get<int64_t>("ct_run", CC);
    uint8_t* dpres = C_.scratch.get<uint8_t>("ct_pres", C);
    uint8_t* den = enabled ? C_.scratch.get<uint8_t>("ct_en", C) : nullptr;
    SYZ_HIP(hipMemcpyAsync(dp, prios, CC * 4, hipMemcpyHostToDevice, s));
    if (den) SYZ_HIP(hipMemcpyAsync(den, enabled, C, hipMemcpyHostToDevice, s));
    prio_choice_dev(nullptr, nullptr, dp, C, den, nullptr, drun, dpres, s);
    SYZ_HIP(hipMemcpyAsync(run, drun, CC * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipMemcpyAsync(row_present, dpres, C, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_prio_choice_dev(const float* static_prios, const int64_t* len_hist, int32_t C, const uint8_t* enabled,
                           float* prios, int64_t* run, uint8_t* row_present, void* stream) {
  SYZ_API_BODY({
    if (!len_hist) fail(SYZGPU_EINVAL, "null len_hist");
    prio_choice_dev(static_prios, len_hist, nullptr, C, enabled, prios, run, row_present, (hipStream_t)stream);
  })
}

}  // extern "C"

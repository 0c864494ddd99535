// Design microbenchmarks for the raw Minimize pipeline (dev tooling, not product): rates of the
// memory patterns the candidate designs rely on, on config-4-shaped data (422M sorted PCs in covers
// of ~420, spread over an 8 MB span).
//   hipcc -O3 --offload-arch=gfx950 -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("%s: %s\n", #x, hipGetErrorString(e));                             \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// covers of LEN sorted PCs: pc = LO + prefix of gaps in [1, 2*GAP)
__global__ void k_gen(uint32_t* pcs, size_t n, uint32_t len, uint32_t gap) {
  size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t nc = n / len;
  if (c >= nc) return;
  uint32_t pc = 0x81000000u + (mix((uint32_t)c) % 4096);
  for (uint32_t k = 0; k < len; k++) {
    pc += 1 + mix((uint32_t)(c * 977 + k)) % (2 * gap);
    pcs[c * len + k] = pc;
  }
}

__global__ void k_stream(const uint4* p, size_t n4, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}

// per-PC gather of a u32 table entry (dictionary lookup): table index (pc - lo) >> sh
__global__ void k_gather(const uint4* p, size_t n4, const uint32_t* tab, uint32_t lo, int sh, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc += tab[(v.x - lo) >> sh] + tab[(v.y - lo) >> sh] + tab[(v.z - lo) >> sh] + tab[(v.w - lo) >> sh];
  }
  if (acc == 0x12345678) out[0] = acc;
}

// per-PC gather of one byte
__global__ void k_gather8(const uint4* p, size_t n4, const uint8_t* tab, uint32_t lo, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc += tab[v.x - lo] + tab[v.y - lo] + tab[v.z - lo] + tab[v.w - lo];
  }
  if (acc == 0x12345678) out[0] = acc;
}

// partition of chunks of CH elements into W windows of (pc - lo) >> S, LDS-staged, coalesced runs
template <int W>
__global__ __launch_bounds__(1024) void k_part(const uint32_t* pcs, size_t n, uint32_t lo, int S, uint32_t* out,
                                               uint32_t chunk) {
  extern __shared__ uint32_t sm[];
  uint32_t* hist = sm;            // W
  uint32_t* cur = sm + W;         // W
  uint32_t* buf = sm + 2 * W;     // chunk
  for (size_t c0 = (size_t)blockIdx.x * chunk; c0 < n; c0 += (size_t)gridDim.x * chunk) {
    const uint32_t cnt = (uint32_t)min<size_t>(chunk, n - c0);
    for (int i = threadIdx.x; i < W; i += 1024) hist[i] = 0;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += 1024) atomicAdd(&hist[((pcs[c0 + k] - lo) >> S) & (W - 1)], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {  // serial-ish scan by one wave
      uint32_t run = 0;
      for (int b = 0; b < W; b += 64) {
        uint32_t v = hist[b + threadIdx.x];
        uint32_t x = v;
        for (int d = 1; d < 64; d <<= 1) {
          uint32_t y = __shfl_up(x, d, 64);
          if ((int)threadIdx.x >= d) x += y;
        }
        cur[b + threadIdx.x] = run + x - v;
        run += __shfl(x, 63, 64);
      }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += 1024) {
      const uint32_t pc = pcs[c0 + k];
      const uint32_t w = ((pc - lo) >> S) & (W - 1);
      buf[atomicAdd(&cur[w], 1u)] = ((pc - lo) & ((1u << S) - 1)) | ((k & 63) << 26);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += 1024) out[c0 + k] = buf[k];
    __syncthreads();
  }
}

// scattered (uncoalesced) direct write of the same partition (no LDS staging)
template <int W>
__global__ __launch_bounds__(1024) void k_part_direct(const uint32_t* pcs, size_t n, uint32_t lo, int S,
                                                      uint32_t* out, uint32_t chunk) {
  __shared__ uint32_t hist[W], cur[W];
  for (size_t c0 = (size_t)blockIdx.x * chunk; c0 < n; c0 += (size_t)gridDim.x * chunk) {
    const uint32_t cnt = (uint32_t)min<size_t>(chunk, n - c0);
    for (int i = threadIdx.x; i < W; i += 1024) hist[i] = 0;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += 1024) atomicAdd(&hist[((pcs[c0 + k] - lo) >> S) & (W - 1)], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {
      uint32_t run = 0;
      for (int b = 0; b < W; b += 64) {
        uint32_t v = hist[b + threadIdx.x];
        uint32_t x = v;
        for (int d = 1; d < 64; d <<= 1) {
          uint32_t y = __shfl_up(x, d, 64);
          if ((int)threadIdx.x >= d) x += y;
        }
        cur[b + threadIdx.x] = run + x - v;
        run += __shfl(x, 63, 64);
      }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += 1024) {
      const uint32_t pc = pcs[c0 + k];
      const uint32_t w = ((pc - lo) >> S) & (W - 1);
      out[c0 + atomicAdd(&cur[w], 1u)] = ((pc - lo) & ((1u << S) - 1)) | ((k & 63) << 26);
    }
    __syncthreads();
  }
}

// LDS direct-mapped min table over a window stream (the Pass M inner loop): 32K-entry table
__global__ __launch_bounds__(1024) void k_ldsmin(const uint4* p, size_t n4, size_t per, uint32_t* out) {
  __shared__ uint32_t tab[32768];
  const size_t b = (size_t)blockIdx.x * per, e = min(n4, b + per);
  for (int i = threadIdx.x; i < 32768; i += 1024) tab[i] = 0xFFFFFFFFu;
  __syncthreads();
  for (size_t i = b + threadIdx.x; i < e; i += 1024) {
    uint4 v = p[i];
    uint32_t r = (uint32_t)i >> 6;
    uint32_t a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t id = a[j] & 0x7FFF;
      if (tab[id] > r) atomicMin(&tab[id], r);
    }
  }
  __syncthreads();
  uint32_t acc = 0;
  for (int i = threadIdx.x; i < 32768; i += 1024) acc += tab[i];
  if (acc == 0x12345678) out[0] = acc;
}

int main() {
  const size_t N = (size_t)420 * 1000000;  // 420M PCs, whole covers
  const uint32_t LEN = 420, GAP = 20000;  // ~8 MB span per cover walk
  uint32_t *pcs, *out, *tab, *dst;
  uint8_t* tab8;
  CK(hipMalloc(&pcs, N * 4));
  CK(hipMalloc(&dst, N * 4));
  CK(hipMalloc(&out, 64));
  const size_t span = (size_t)LEN * 2 * GAP + 8192;
  CK(hipMalloc(&tab, span * 4));
  CK(hipMalloc(&tab8, span));
  CK(hipMemset(tab, 1, span * 4));
  CK(hipMemset(tab8, 1, span));
  CK(hipMemset(pcs, 0, N * 4));
  k_gen<<<(N / LEN + 255) / 256, 256>>>(pcs, N, LEN, GAP);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto timeit = [&](const char* name, double bytes, auto fn) {
    fn();
    if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) {
      printf("%s: launch failed\n", name);
      exit(1);
    }
    hipEventRecord(a);
    const int R = 5;
    for (int i = 0; i < R; i++) fn();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= R;
    printf("%-40s %8.3f ms  %8.1f GB/s  %6.2f G elem/s\n", name, ms, bytes / ms / 1e6, N / ms / 1e6);
  };
  const unsigned G = 256 * 8;
  timeit("stream read u32x4", N * 4.0, [&] { k_stream<<<G * 4, 256>>>((const uint4*)pcs, N / 4, out); });
  const uint32_t lo = 0x81000000u;
  // table sizes: span (~16.8M entries) >> sh
  for (int sh : {0, 2, 3, 4, 6}) {
    char nm[64];
    snprintf(nm, sizeof nm, "gather u32 table %.1f MB", (span >> sh) * 4 / 1e6);
    timeit(nm, N * 4.0, [&] { k_gather<<<G * 4, 256>>>((const uint4*)pcs, N / 4, tab, lo, sh, out); });
  }
  timeit("gather u8 bytemap", N * 4.0, [&] { k_gather8<<<G * 4, 256>>>((const uint4*)pcs, N / 4, tab8, lo, out); });
  for (uint32_t ch : {8192u, 16384u, 24576u}) {
    char nm[64];
    snprintf(nm, sizeof nm, "partition LDS-staged W=256 chunk %u", ch);
    timeit(nm, N * 8.0, [&] {
      k_part<256><<<256 * 2, 1024, (2 * 256 + ch) * 4>>>(pcs, N, lo, 15, dst, ch);
    });
    snprintf(nm, sizeof nm, "partition LDS-staged W=1024 chunk %u", ch);
    timeit(nm, N * 8.0, [&] {
      k_part<1024><<<256 * 2, 1024, (2 * 1024 + ch) * 4>>>(pcs, N, lo, 13, dst, ch);
    });
    snprintf(nm, sizeof nm, "partition direct W=256 chunk %u", ch);
    timeit(nm, N * 8.0, [&] { k_part_direct<256><<<256 * 4, 1024>>>(pcs, N, lo, 15, dst, ch); });
  }
  {
    const size_t n4 = N / 4;
    const size_t per = (n4 + 2047) / 2048;
    timeit("lds min direct 32K (2048 items)", N * 4.0, [&] { k_ldsmin<<<2048, 1024>>>((const uint4*)pcs, n4, per, out); });
  }
  return 0;
}

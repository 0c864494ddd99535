// Microbenchmark (dev tooling, not product): HBM read rate of runs of R bytes at random 4-byte-aligned
// offsets of a 1.7 GB buffer — the access shape of the first-occurrence walk over window runs of
// chunk-major elements (R ~ 200 B today) against longer runs and plain streaming.
//   hipcc -O3 --offload-arch=gfx950 -o tools/mb_runs tools/mb_runs.hip && ./tools/mb_runs
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

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

// Each wave reads runs of W words (W <= 64: one dword per lane) at random word offsets, U runs in
// flight; nruns runs in all.
template <int U>
__global__ __launch_bounds__(256) void k_runs(const uint32_t* buf, uint64_t nwords, uint32_t W, uint64_t nruns,
                                              uint32_t* out) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (uint64_t r0 = wave * U; r0 < nruns; r0 += nw * U) {
    uint32_t v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t r = r0 + u;
      const uint64_t off = ((uint64_t)mix((uint32_t)r) * 0x9E37ull + mix((uint32_t)(r >> 32) + 7)) % (nwords - 1024);
      v[u] = 0;
      for (uint32_t k = 0; k < W; k += 64) v[u] ^= k + lane < W ? buf[off + k + lane] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc ^= v[u];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// plain stream of 16-B vectors
__global__ void k_stream(const uint4* p, size_t n4, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}

int main() {
  const uint64_t bytes = 1700ull << 20, nwords = bytes / 4;
  uint32_t *buf, *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 1, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms;
  for (int it = 0; it < 2; it++) {
    CK(hipEventRecord(a));
    k_stream<<<8192, 256>>>((const uint4*)buf, bytes / 16, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
  }
  printf("stream: %.3f ms, %.0f GB/s\n", ms, bytes / (ms * 1e-3) / 1e9);
  const uint32_t Ws[] = {16, 32, 50, 64, 128, 256};
  for (uint32_t W : Ws) {
    const uint64_t nruns = nwords / W;
    for (int grid : {4096, 16384}) {
      for (int it = 0; it < 2; it++) {
        CK(hipEventRecord(a));
        k_runs<8><<<grid, 256>>>(buf, nwords, W, nruns, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
      }
      printf("runs of %3u words (%4u B), U=8, grid %5d: %.3f ms, %.0f GB/s useful\n", W, W * 4, grid, ms,
             nruns * W * 4.0 / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}

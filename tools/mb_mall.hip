// Microbenchmark (dev tooling): does a transpose round trip through a ring buffer small enough for the
// 256 MiB Infinity Cache avoid HBM? Streams S bytes of "PCs" in slabs; per slab a producer kernel
// copies the slab into ring[slab % 2] (a window-major rewrite stand-in) and a consumer kernel reads it
// back. Ring slot sizes from 16 MiB to the whole input: if the cache keeps the ring, small slots run at
// read-only speed + cache bandwidth. Also: pure read of S bytes, pure copy of S bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ a, size_t n4, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n4) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = a[i];
    v.x ^= 1;
    b[i] = v;
  }
}

// scattered-run copy: 64-element runs written to a permuted run position (a transpose stand-in)
__global__ __launch_bounds__(256) void k_copy_runs(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n4,
                                                   uint32_t runs_mask) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const size_t run = i >> 4, inr = i & 15;  // 16 uint4 = 64 u32 per run
    const size_t nr = n4 >> 4;
    const size_t pr = (run * 2654435761ull) % nr;
    uint4 v = a[i];
    v.x ^= 1;
    b[pr * 16 + inr] = v;
  }
}

int main(int argc, char** argv) {
  const size_t S = (argc > 1 ? atoll(argv[1]) : 1700ull) << 20;
  const size_t n4 = S / 16;
  uint4 *src, *ring;
  uint32_t* out;
  CK(hipMalloc(&src, S));
  CK(hipMalloc(&ring, S));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(src, 1, S));
  CK(hipMemset(ring, 0, S));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 256 * 8;
  auto timeit = [&](auto fn) {
    fn();
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
      CK(hipEventRecord(e0));
      fn();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
    }
    return best;
  };
  float t = timeit([&] { k_read<<<grid, 256>>>(src, n4, out); });
  printf("read %zu MiB: %.3f ms  %.2f TB/s\n", S >> 20, t, S / t / 1e9);
  t = timeit([&] { k_copy<<<grid, 256>>>(src, ring, n4); });
  printf("copy %zu MiB: %.3f ms  %.2f TB/s (r+w)\n", S >> 20, t, 2 * S / t / 1e9);
  t = timeit([&] { k_copy_runs<<<grid, 256>>>(src, ring, n4, 0); });
  printf("copy_runs(256B runs permuted) %zu MiB: %.3f ms  %.2f TB/s (r+w)\n", S >> 20, t, 2 * S / t / 1e9);
  const size_t slots[] = {16ull << 20, 32ull << 20, 64ull << 20, 96ull << 20, 128ull << 20, 256ull << 20, S / 2};
  for (size_t slot : slots) {
    if (2 * slot > S) continue;
    const size_t ns = (S + slot - 1) / slot;
    for (int runs = 0; runs < 2; runs++) {
      t = timeit([&] {
        for (size_t k = 0; k < ns; k++) {
          const size_t b = k * slot, len = std::min(slot, S - b);
          uint4* r = ring + (k & 1) * (slot / 16);
          if (runs)
            k_copy_runs<<<grid, 256>>>(src + b / 16, r, len / 16, 0);
          else
            k_copy<<<grid, 256>>>(src + b / 16, r, len / 16);
          k_read<<<grid, 256>>>(r, len / 16, out);
        }
      });
      printf("slab round trip slot %4zu MiB x%zu %s: %.3f ms  (input %.2f TB/s)\n", slot >> 20, ns,
             runs ? "runs" : "seq ", t, S / t / 1e9);
    }
  }
  return 0;
}

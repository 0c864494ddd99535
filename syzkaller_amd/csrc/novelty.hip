// syz-fuzzer's new-coverage check over a batch (syz-fuzzer/fuzzer.go:446-470 execute; the same
// rule as syz-manager NewInput, manager.go:609-616):
//   for each cover k, in order:  diff := Difference(Difference(cov_k, maxCover[g_k]), flakes)
//                                if diff != {} { maxCover[g_k] = Union(maxCover[g_k], diff); new }
//
// Exact batch reformulation: a cover whose diff is empty adds nothing, so before
// cover k the table is maxCover0[g] u (every earlier cover of g minus flakes). Cover k is new iff one
// of its PCs - not 0xFFFFFFFF (foreach drops it, cover.go:81-102), not a flake, not in maxCover0[g]
// - occurs first, among the covers of g, in cover k. With items (g<<32|pc, rank) laid out in rank
// order (maxCover0 entries rank 0, cover k rank k+1) a STABLE sort by key puts every key's first
// occurrence at the head of its run, so one pass over run heads decides every key:
//   head rank 0         -> the PC was in maxCover0[g]: output
//   head rank k+1       -> unless pc is 0xFFFFFFFF or a flake: cover k is new, the PC is output
// The runs come out sorted by (g, pc), so the updated tables are an ordered compaction. A table that
// took at least one Union loses a 0xFFFFFFFF entry it had (Union also goes through foreach).
#include <algorithm>

#include "pipeline.hpp"

namespace syz {

void radix_sort_pairs(uint64_t*& keys, uint32_t*& vals, uint64_t*& ktmp, uint32_t*& vtmp, size_t n, int end_bit,
                      hipStream_t s);

__global__ void k_nov_items_mc(const uint32_t* mc, const uint64_t* mc_off, uint32_t G, uint64_t total, uint64_t* keys,
                               uint32_t* vals, int* err) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = (uint32_t)upper_bound_dev<uint64_t>(mc_off, 0, G + 1, j) - 1;
    const uint32_t pc = mc[j];
    if (j > mc_off[g] && mc[j - 1] >= pc) atomicOr(err, 1);  // maxCover tables must be canonical
    keys[j] = ((uint64_t)g << 32) | pc;
    vals[j] = 0;
  }
}

// one wave per cover
__global__ __launch_bounds__(256) void k_nov_items_cov(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                                       size_t n, uint32_t G, uint64_t base, uint64_t* keys,
                                                       uint32_t* vals, int* err) {
  const size_t k = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (k >= n) return;
  const uint32_t g = group[k];
  if (g >= G) {
    if (__lane_id() == 0) atomicOr(err, 2);
    return;
  }
  const uint64_t b = off[k], e = off[k + 1];
  for (uint64_t j = b + __lane_id(); j < e; j += 64) {
    const uint32_t pc = pcs[j];
    if (j > b && pcs[j - 1] >= pc) atomicOr(err, 4);  // covers must be canonical (executor.cc:572-585)
    keys[base + j] = ((uint64_t)g << 32) | pc;
    vals[base + j] = (uint32_t)(k + 1);
  }
}

__device__ __forceinline__ bool in_sorted(const uint32_t* a, uint64_t n, uint32_t v) {
  const uint64_t p = lower_bound_dev<uint32_t>(a, 0, n, v);
  return p < n && a[p] == v;
}

__global__ void k_nov_mark(const uint64_t* keys, const uint32_t* vals, uint64_t ni, const uint32_t* flakes,
                           uint64_t nflakes, uint8_t* is_new, uint8_t* updated, uint8_t* flag, uint64_t* sentpos,
                           uint32_t* nsent) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ni; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = keys[i];
    uint8_t f = 0;
    if (i == 0 || keys[i - 1] != key) {
      const uint32_t r = vals[i];
      const uint32_t pc = (uint32_t)key;
      if (r == 0) {
        f = 1;
        if (pc == SENT) sentpos[atomicAdd(nsent, 1u)] = i;
      } else if (pc != SENT && !in_sorted(flakes, nflakes, pc)) {
        is_new[r - 1] = 1;
        updated[key >> 32] = 1;
        f = 1;
      }
    }
    flag[i] = f;
  }
}

__global__ void k_nov_sent(const uint64_t* keys, const uint64_t* sentpos, const uint32_t* nsent,
                           const uint8_t* updated, uint8_t* flag) {
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < *nsent; t += gridDim.x * blockDim.x) {
    const uint64_t i = sentpos[t];
    if (updated[keys[i] >> 32]) flag[i] = 0;
  }
}

__global__ void k_nov_out(const uint64_t* keys, const uint8_t* flag, const uint64_t* pos, uint64_t ni, uint32_t* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ni; i += (uint64_t)gridDim.x * blockDim.x)
    if (flag[i]) out[pos[i]] = (uint32_t)keys[i];
}

// gfirst[g] = first sorted index whose group is >= g (ni if none), g in [0, G]
__global__ void k_group_first(const uint64_t* keys, uint64_t ni, uint32_t G, uint64_t* gfirst) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= ni; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t lo = i == 0 ? 0 : (keys[i - 1] >> 32) + 1;
    const uint64_t hi = i == ni ? G : (keys[i] >> 32);
    for (uint64_t g = lo; g <= hi && g <= G; g++) gfirst[g] = i;
  }
}

__global__ void k_gather_pos(const uint64_t* pos, const uint64_t* gfirst, uint32_t G, uint64_t* out_off) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g <= G; g += gridDim.x * blockDim.x)
    out_off[g] = pos[gfirst[g]];
}

static int key_bits(uint32_t G) {
  int b = 0;
  while (b < 32 && (1ull << b) < G) b++;
  return 32 + b;
}

void novelty_batch(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n, uint32_t G,
                   const uint32_t* mc, const uint64_t* mc_off, const uint32_t* flakes, size_t nflakes,
                   uint8_t* is_new, uint32_t* out_mc, size_t out_cap, uint64_t* out_mc_off) {
  Context& c = ctx();
  Scratch& sc = c.scratch;
  hipStream_t s = c.stream;
  if (G == 0) fail(SYZGPU_EINVAL, "ngroups must be > 0");
  if (!off || !mc_off || !out_mc_off || (n && (!group || !is_new))) fail(SYZGPU_EINVAL, "null pointer");
  if (off[0] != 0 || mc_off[0] != 0) fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
  if (n >= 0xFFFFFFF0ull) fail(SYZGPU_EINVAL, "too many covers in one batch");
  for (size_t i = 1; i < nflakes; i++)
    if (flakes[i - 1] >= flakes[i]) fail(SYZGPU_EINVAL, "flakes must be canonical (strictly increasing)");
  const uint64_t L = off[n], M = mc_off[G], ni = L + M;
  uint32_t* d_pcs = sc.get<uint32_t>("nv_pcs", L + 1);
  uint64_t* d_off = sc.get<uint64_t>("nv_off", n + 1);
  uint32_t* d_grp = sc.get<uint32_t>("nv_grp", n + 1);
  uint32_t* d_mc = sc.get<uint32_t>("nv_mc", M + 1);
  uint64_t* d_mco = sc.get<uint64_t>("nv_mco", G + 1);
  uint32_t* d_fl = sc.get<uint32_t>("nv_fl", nflakes + 1);
  int* err = sc.get<int>("nv_err", 2);
  uint64_t* keys = sc.get<uint64_t>("nv_keys", ni + 1);
  uint32_t* vals = sc.get<uint32_t>("nv_vals", ni + 1);
  uint64_t* ktmp = sc.get<uint64_t>("nv_ktmp", ni + 1);
  uint32_t* vtmp = sc.get<uint32_t>("nv_vtmp", ni + 1);
  uint8_t* d_new = sc.get<uint8_t>("nv_new", n + 1);
  uint8_t* upd = sc.get<uint8_t>("nv_upd", G + 1);
  uint8_t* flag = sc.get<uint8_t>("nv_flag", ni + 1);
  uint64_t* pos = sc.get<uint64_t>("nv_pos", ni + 1);
  uint64_t* sentpos = sc.get<uint64_t>("nv_sentpos", G + 1);
  uint32_t* nsent = sc.get<uint32_t>("nv_nsent", 1);
  uint64_t* gfirst = sc.get<uint64_t>("nv_gfirst", G + 1);
  uint64_t* d_ooff = sc.get<uint64_t>("nv_ooff", G + 1);
  uint32_t* d_out = sc.get<uint32_t>("nv_out", ni + 1);
  if (L) SYZ_HIP(hipMemcpyAsync(d_pcs, pcs, L * 4, hipMemcpyHostToDevice, s));
  SYZ_HIP(hipMemcpyAsync(d_off, off, (n + 1) * 8, hipMemcpyHostToDevice, s));
  if (n) SYZ_HIP(hipMemcpyAsync(d_grp, group, n * 4, hipMemcpyHostToDevice, s));
  if (M) SYZ_HIP(hipMemcpyAsync(d_mc, mc, M * 4, hipMemcpyHostToDevice, s));
  SYZ_HIP(hipMemcpyAsync(d_mco, mc_off, (G + 1) * 8, hipMemcpyHostToDevice, s));
  if (nflakes) SYZ_HIP(hipMemcpyAsync(d_fl, flakes, nflakes * 4, hipMemcpyHostToDevice, s));
  SYZ_HIP(hipMemsetAsync(err, 0, 8, s));
  SYZ_HIP(hipMemsetAsync(d_new, 0, n + 1, s));
  SYZ_HIP(hipMemsetAsync(upd, 0, G + 1, s));
  SYZ_HIP(hipMemsetAsync(nsent, 0, 4, s));
  {
    ProfScope ps("novelty_items", s, ni * 16);
    if (M) {
      k_nov_items_mc<<<grid_for(M, 256, 16384), 256, 0, s>>>(d_mc, d_mco, G, M, keys, vals, err);
      SYZ_LAUNCHED();
    }
    if (n) {
      k_nov_items_cov<<<(unsigned)((n * 64 + 255) / 256), 256, 0, s>>>(d_pcs, d_off, d_grp, n, G, M, keys, vals, err);
      SYZ_LAUNCHED();
    }
  }
  {
    ProfScope ps("novelty_sort", s, ni * 12 * 3);
    radix_sort_pairs(keys, vals, ktmp, vtmp, ni, key_bits(G), s);
  }
  {
    ProfScope ps("novelty_mark", s, ni * 13);
    if (ni) {
      k_nov_mark<<<grid_for(ni, 256, 65536), 256, 0, s>>>(keys, vals, ni, d_fl, nflakes, d_new, upd, flag, sentpos,
                                                        nsent);
      SYZ_LAUNCHED();
      k_nov_sent<<<grid_for(G, 256, 64), 256, 0, s>>>(keys, sentpos, nsent, upd, flag);
      SYZ_LAUNCHED();
    }
  }
  exclusive_scan_u8(flag, pos, ni, s);
  if (ni) {
    k_nov_out<<<grid_for(ni, 256, 65536), 256, 0, s>>>(keys, flag, pos, ni, d_out);
    SYZ_LAUNCHED();
  }
  k_group_first<<<grid_for(ni + 1, 256, 65536), 256, 0, s>>>(keys, ni, G, gfirst);
  SYZ_LAUNCHED();
  k_gather_pos<<<grid_for(G + 1, 256, 1024), 256, 0, s>>>(pos, gfirst, G, d_ooff);
  SYZ_LAUNCHED();
  int herr[2];
  SYZ_HIP(hipMemcpyAsync(herr, err, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipMemcpyAsync(out_mc_off, d_ooff, (G + 1) * 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (herr[0] & 1) fail(SYZGPU_EINVAL, "maxCover tables must be canonical (strictly increasing)");
  if (herr[0] & 2) fail(SYZGPU_EINVAL, "group id >= ngroups");
  if (herr[0] & 4) fail(SYZGPU_EINVAL, "covers must be canonical (strictly increasing)");
  const uint64_t total = out_mc_off[G];
  if (total > out_cap) fail(SYZGPU_ECAPACITY, "out_mc capacity too small");
  if (total) SYZ_HIP(hipMemcpyAsync(out_mc, d_out, total * 4, hipMemcpyDeviceToHost, s));
  if (n) SYZ_HIP(hipMemcpyAsync(is_new, d_new, n, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
}

}  // namespace syz

extern "C" int syzgpu_novelty_batch(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                                    uint32_t ngroups, const uint32_t* mc, const uint64_t* mc_off,
                                    const uint32_t* flakes, size_t nflakes, uint8_t* is_new, uint32_t* out_mc,
                                    size_t out_cap, uint64_t* out_mc_off) {
  SYZ_API_BODY({
    syz::novelty_batch(pcs, off, group, n, ngroups, mc, mc_off, flakes, nflakes, is_new, out_mc, out_cap,
                       out_mc_off);
  })
}

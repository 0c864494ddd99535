// Internal interfaces between the kernels of libsyzgpu.so.
#pragma once
#include <functional>

#include "common.hpp"
#include "plan_host.hpp"

namespace syz {


// gosort.hip: the element at sorted position r of the groups' ranges is el[perm[r]]
// (GS_T_SEG, GS_U32_LEN_LIMIT, Seg, Pack, gosort_segments: plan_host.hpp)
struct GosortPlan {
  size_t n = 0;
  uint32_t nsmall = 0, npacks = 0, nbig = 0;
  uint64_t big_total = 0;  // elements in the groups that start the global levels
  uint64_t big_max = 0;    // elements in the largest of them
  mutable uint32_t rounds_hint = 0;  // global rounds the last run of this plan needed (issued up front)
  mutable bool may_bounce = true;    // false: every cover length fits the u32 sort element (< 2^19)
  Seg* small = nullptr;
  Pack* packs = nullptr;
  Seg* big = nullptr;
  size_t cap_small = 0, cap_packs = 0, cap_big = 0;  // (grow-only across re-plans)
  GosortPlan() = default;
  GosortPlan(const GosortPlan&) = delete;
  GosortPlan& operator=(const GosortPlan&) = delete;
  ~GosortPlan();
};
void gosort_plan(GosortPlan& P, const std::vector<uint64_t>& hstart, uint32_t ngroups, hipStream_t s);
// small_done(q) is enqueued on stream q once the packed (small) call groups are sorted, big_done(q)
// once the big ones are; both run before gosort_run's streams join, so per-class consumers overlap
// with the other class's sort.
void gosort_run(uint64_t* el, uint32_t* perm, size_t n, const GosortPlan& P, hipStream_t s,
                const std::function<void(hipStream_t)>& small_done = {},
                const std::function<void(hipStream_t)>& big_done = {});
void gosort_groups(uint64_t* el, uint32_t* perm, size_t n, const std::vector<uint64_t>& hstart, uint32_t ngroups,
                   hipStream_t s);

// radix.hip: stable LSD sort of (u64 key, u32 value) pairs by key bits [0, end_bit), RADIX_BITS per pass
constexpr int RADIX_BITS = 8;
void radix_sort_pairs(uint64_t*& keys, uint32_t*& vals, uint64_t*& ktmp, uint32_t*& vtmp, size_t n, int end_bit,
                      hipStream_t s);
void radix_sort_pairs(uint32_t*& keys, uint32_t*& vals, uint32_t*& ktmp, uint32_t*& vtmp, size_t n, int end_bit,
                      hipStream_t s);

// setops.hip
uint64_t setop_batch_dev(int op, const uint32_t* a, const uint64_t* aoff, uint64_t na, const uint32_t* b,
                         const uint64_t* boff, uint64_t nb, uint32_t npairs, uint32_t* out, uint64_t out_cap,
                         uint64_t* out_off_dev, hipStream_t s);
void canonicalize_batch_dev(uint32_t* pcs, const uint64_t* off, const uint64_t* host_off, size_t ncov,
                            uint64_t* out_len, hipStream_t s);
// the same with the covers classed on the device (no host offsets)
void canonicalize_batch_dev2(uint32_t* pcs, const uint64_t* off, size_t ncov, uint64_t* out_len, hipStream_t s);

// prio.hip
void len_hist_dev(const uint16_t* prog_len, const uint8_t* sel, size_t n, int32_t C, int64_t* hist, int* err,
                  hipStream_t s);
// calcStaticPriorities (static_prio.hip): enqueue only, and the check of its device error word
const uint32_t* static_priorities_enqueue(const float* uses, size_t nkeys, int32_t C, float* prios, hipStream_t s);
void static_prio_check(uint32_t err);
void prio_choice_dev(const float* static_prios, const int64_t* len_hist, const float* prios_in, int32_t C,
                     const uint8_t* enabled, float* prios_out, int64_t* run, uint8_t* present, hipStream_t s);

}  // namespace syz

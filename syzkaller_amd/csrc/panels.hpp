// The raw-cover Minimize pipeline (panels.hip) and the pieces of minimize.hip it shares.
#pragma once
#include <array>
#include <memory>
#include <mutex>
#include <vector>

#include "plan_host.hpp"
#include "store.hpp"

namespace syz {

constexpr uint32_t MAX_GROUPS_PM = 4096;


struct PSlab {
  uint64_t elem;      // first element (4-aligned: the slab's passes leave as 16-byte vectors)
  uint64_t t0;        // first tile (index into the job's tile sequence)
  uint32_t m0, nmem;  // first member (partition index), members spanned
  uint32_t nt, g;     // tiles, call group
  uint32_t j, pad;    // slab index inside its call group
};

// The slab form's layout of one job (slab_dev.hpp), device arrays in the lane's scratch under a name
// prefix. slab_plan (host): blocks, slab bounds, D rows; the caller stages hsg / hgblock / hbgroup to the
// device and sets dsg / dgblock / dbgroup; slab_build (device): tiles, their prefix, the slabs, per-group
// first slab and element; then k_slab (P) and for_slab_window (M).
struct SlabJob : SlabPlan {  // the host plan (plan_host.hpp slab_plan) and its device arrays
  const SGroup* dsg = nullptr;
  const uint32_t* dgblock = nullptr;
  const uint32_t* dbgroup = nullptr;
  uint64_t* tpos = nullptr;
  uint64_t* cstart = nullptr;  // cstart[B] = slabs
  PSlab* slabs = nullptr;
  uint32_t* gslab = nullptr;
  uint64_t* gebase = nullptr;
  uint32_t* D = nullptr;
  uint32_t* elems = nullptr;
  uint64_t ecap = 0;         // elements the buffer holds
  uint32_t* wtot = nullptr;  // per (call, window) totals, when asked for
};
void slab_build(SlabJob& J, const char* prefix, const uint32_t* mlen, const uint64_t* mpos, size_t nmem,
                const uint64_t* gstart, hipStream_t s, bool tiles_done = false);
// the members' tile prefix alone (slab_build's first step, which needs no plan): returns tpos
uint64_t* slab_tiles(const uint32_t* mlen, size_t nmem, const char* prefix, hipStream_t s);

struct RawMinArgs {
  const uint32_t* pcs;
  const uint64_t* off;
  const uint32_t* group;
  const uint16_t* prog_len;  // may be null (no histogram then)
  size_t n;
  uint32_t G;
  const uint32_t* key_lo = nullptr;  // host, per group: this rank's PC range [key_lo, key_hi] of it
  const uint32_t* key_hi = nullptr;  // (null: whole groups)
  hipStream_t s = nullptr;
};
struct RawEndArgs {
  int32_t C = 0;
  const uint8_t* count_hist = nullptr;  // host, per group: counted in len_hist (null: all)
  uint8_t* selected = nullptr;          // device, n bytes in entry order
  int64_t* len_hist = nullptr;          // device, C+1
  int64_t* out_idx = nullptr;           // device, kept entries group-major in selection order
  uint64_t* group_out_off = nullptr;    // device, G+1
  hipStream_t s = nullptr;
  bool defer_check = false;             // leave the len(p.Calls) > C check to the caller (minimize_raw_end_check)
};

// One minimizeCorpus job (the raw path): its selection lives here between begin and end, so a
// multi-GPU step can exchange the selection of split call groups in between, and concurrent callers
// with their own jobs never see each other's state.
// plan_layout's plan for one layout (the key), kept by the job for the next step on the same layout
struct SlabPlanCache {
  std::vector<uint64_t> key;
  SlabJob SJ;  // host parts; dsg / dgblock / dbgroup point into dstage
  size_t icount[2][3] = {{0, 0, 0}, {0, 0, 0}};
  std::array<std::array<size_t, 3>, 2> ifirst{};
  uint64_t item_pcs[2][3] = {{0, 0, 0}, {0, 0, 0}};
  size_t o_gb = 0, o_bg = 0, o_it = 0, o_exp = 0;  // staging offsets (o_exp: k_gpack's expected words)
  uint64_t cpcs[2] = {0, 0}, cent[2] = {0, 0};  // PCs / entries of the small and big call groups
  uint32_t lo = 0, hi = 0;
  size_t n = 0;
  Grow<uint8_t> dstage;  // SGroup[G], gblock[G + 1], bgroup[B + 1], items, expected words
};

struct MinJob {
  std::recursive_mutex mu;
  size_t n = 0;
  uint32_t G = 0;
  bool begun = false;
  bool may_bounce = true;  // a cover too long for the Go sort's u32 element (begin's length scan)
  const uint32_t* group = nullptr;     // caller's device buffers (valid from begin to end)
  const uint16_t* prog_len = nullptr;
  Grow<uint64_t> gstart;
  Grow<uint32_t> selbits;  // kept bit per global rank (Go-sort position), n / 32 + 2 words
  Grow<uint32_t> ent_of_rank, rank_of_member, xg;
  Grow<uint64_t> xo;
  Grow<uint8_t> count_hist;
  std::vector<uint64_t> hstart, xkey;
  std::shared_ptr<GosortPlan> plan;  // Go-sort plan of the last layout (keeps its rounds hint)
  std::shared_ptr<SlabPlanCache> pcache;  // plan_layout's plan of the last layout
  bool nospec = false;                    // begin_once: this call redoes a speculation that missed
  bool spec_ok = false;                   // the last planned layout was the cached one: speculate next call
  uint64_t spec_hits = 0, spec_misses = 0;
  std::vector<uint64_t> plan_key;
  uint64_t stats_total_pcs = 0;
  size_t stats_items_direct = 0, stats_items_hash = 0;
  hipEvent_t done = nullptr;  // begin's last work (M) on its stream: end / exchange / fetch wait for it
  ~MinJob() {
    if (done) (void)hipEventDestroy(done);
  }
};

void minimize_raw_begin(MinJob& J, const RawMinArgs& a);
void minimize_raw_xchg(MinJob& J, const uint32_t* groups, const uint64_t* offsets, uint32_t ng, uint8_t* buf,
                       int import, hipStream_t s);
void minimize_raw_end(MinJob& J, const RawEndArgs& e);
void minimize_raw_end_check(int err);  // the deferred check of end's device error word (mz_err)
void minimize_raw_fetch(MinJob& J, int64_t* out_idx, uint64_t* group_out_off);
// group-major kept list (device) from a rank bitmap
void sel_compact_dev(const uint32_t* selbits, const uint32_t* ent_of_rank, const uint64_t* gstart, size_t n, uint32_t G,
                     int64_t* out_idx, uint64_t* group_out_off, hipStream_t s);

// minimize.hip
// group_partition_dev's optional extra outputs (k_grp_scatter)
struct PartOut {
  uint64_t* gstart = nullptr;          // (set by group_partition_dev)
  uint32_t* rank_of_member = nullptr;  // identity ranks: rank_of_member[m] = m, ent_of_rank[m] = members[m]
  uint32_t* ent_of_rank = nullptr;
  uint32_t* mlen = nullptr;            // member lengths (whole covers)
};
void group_partition_dev(const uint32_t* group, const uint64_t* off, size_t n, uint32_t G, uint64_t* gstart,
                         uint32_t* members, uint64_t* el, int* err, hipStream_t s, PartOut po = PartOut{});
void rank_init_dev(const uint32_t* members, size_t n, uint32_t* rank_of_member, uint32_t* ent_of_rank, hipStream_t s);
void ranks_packs(const uint64_t* el, const uint32_t* perm, const GosortPlan& P, const uint32_t* members,
                 uint32_t* rank_of_member, uint32_t* ent_of_rank, hipStream_t q);
void ranks_big(const uint64_t* el, const uint32_t* perm, const GosortPlan& P, const uint32_t* members,
               uint32_t* rank_of_member, uint32_t* ent_of_rank, hipStream_t q);

}  // namespace syz

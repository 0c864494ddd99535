// Multi-GPU minimizeCorpus behind the C ABI (SURVEY.md §7 and §8b `syzgpu_init(ndev)`, §8e): ONE
// process drives a sub-job per device, so a Go manager built with the syzgpu tag uses every GPU of its
// node through syzgpu_mgz_* alone, with no torch.distributed and no second process.
//
// The split is the one bench.py runs over torch.distributed (syzkaller_amd/sharding.py),
// restated here so the library owns it:
//   * call groups go to sub-jobs whole (each call's Minimize is independent, manager.go:523-527); a group
//     heavier than a sub-job's share is split by PC value (plan_parts / split_bounds below), and each
//     holder minimizes its PC range only (RawMinArgs key_lo / key_hi, panels.hip);
//   * between begin and end the holders of split groups exchange their selections: an input is kept iff
//     some PC of it first occurs at it, so the parts' selections OR to the whole one. Every sub-job
//     exports one byte per entry of the split groups it holds into its buffer, the buffers go to every
//     device by peer copies (xGMI between devices, a device copy on one device), and a MAX kernel folds
//     them before the import (the RCCL MAX all-reduce of bench.py, done inside the library);
//   * each group's primary counts it in the kept-length histogram; the histograms are summed the same
//     way on the first device, which computes calcStaticPriorities + CalculatePriorities +
//     BuildChoiceTable (prio.go:29-38, 202-228) once;
//   * the kept list is assembled on the host from each group's primary, group-major (the order of
//     syzgpu_minimize_grouped).
// Each sub-job runs on a host thread of its own that holds a lane of its device (LaneGuard(dev)); the
// threads meet at barriers between the phases. A device may appear more than once (the one-GPU test
// runs two sub-jobs on device 0).
#include <algorithm>
#include <condition_variable>
#include <numeric>
#include <thread>

#include "panels.hpp"
#include "pipeline.hpp"

namespace syz {

// (the key-space plan, kp::plan_parts / kp::split_bounds: plan_host.cpp)

// ---- device helpers -----------------------------------------------------------------------------------
__global__ void k_mg_max_u8(uint8_t* dst, const uint8_t* src, uint64_t bytes, uint32_t nsrc) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < bytes; i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t m = 0;
    for (uint32_t k = 0; k < nsrc; k++) m = max(m, src[(uint64_t)k * bytes + i]);
    dst[i] = m;
  }
}
__global__ void k_mg_sum_i64(int64_t* dst, const int64_t* src, uint32_t n, uint32_t nsrc) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int64_t s = 0;
    for (uint32_t k = 0; k < nsrc; k++) s += src[(uint64_t)k * n + i];
    dst[i] = s;
  }
}

// A reusable barrier for the sub-job threads of one call. A phase's failure is recorded before the
// barrier, so after it every thread sees it and they all stop at the same point.
class PhaseBarrier {
 public:
  explicit PhaseBarrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      gen_++;
      cv_.notify_all();
      return;
    }
    cv_.wait(lk, [&] { return gen_ != gen; });
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  uint64_t gen_ = 0;
};

struct MgShard {
  int dev = 0;
  std::vector<uint64_t> ids;  // global ids of the entries this sub-job holds, ascending
  size_t n = 0;
  Grow<uint32_t> pcs, grp;
  Grow<uint64_t> off, goff;
  Grow<uint16_t> plen;
  Grow<uint8_t> sel, xbuf, xgather;
  Grow<int64_t> hist, hgather, out;
  Grow<float> uses, stat, prios;
  Grow<int64_t> run;
  Grow<uint8_t> rowp;
  std::vector<uint32_t> key_lo, key_hi, xg;
  std::vector<uint64_t> xo;
  std::vector<uint8_t> count;  // the groups this sub-job counts in the histogram (their primary)
  bool parts = false;          // holds a part of a split group
  std::unique_ptr<MinJob> job{new MinJob()};
  std::vector<int64_t> h_out;  // this call's kept list (local ids, group-major) and group offsets
  std::vector<uint64_t> h_goff;
};

struct MultiJob {
  std::mutex mu;  // one call at a time per job
  std::vector<std::unique_ptr<MgShard>> sh;
  uint32_t G = 0;
  size_t n = 0;
  bool loaded = false;
  kp::Plan plan;
  std::vector<uint32_t> xgroups;  // split groups, ascending; xoff: their byte offsets in the exchange buffer
  std::vector<uint64_t> xoff;
  uint64_t xbytes = 0;
};

// Runs f(r) for every sub-job on a thread of its own holding a lane of the sub-job's device; the first
// failure is rethrown after every thread has stopped. f gets the barrier to meet the others between phases
// and a flag that tells it another thread failed (then it returns at once).
template <class F>
static void mg_run(MultiJob& M, F f) {
  const int R = (int)M.sh.size();
  PhaseBarrier bar(R);
  std::mutex emu;
  bool failed = false;
  int code = SYZGPU_OK;
  std::string msg;
  auto note = [&](int c, const std::string& m) {
    std::lock_guard<std::mutex> lk(emu);
    if (!failed) {
      failed = true;
      code = c;
      msg = m;
    }
  };
  // phase(): run one step of f's work; false when this or another thread failed (after the barrier)
  auto body = [&](int r) {
    auto step = [&](auto&& g) -> bool {
      try {
        g();
      } catch (const Error& e) {
        note(e.code, e.msg);
      } catch (const std::exception& e) {
        note(SYZGPU_EINTERNAL, e.what());
      }
      bar.wait();
      std::lock_guard<std::mutex> lk(emu);
      return !failed;
    };
    std::unique_ptr<LaneGuard> lg;
    if (!step([&] { lg.reset(new LaneGuard(M.sh[r]->dev)); })) return;
    f(r, step);
  };
  std::vector<std::thread> th;
  for (int r = 0; r < R; r++) th.emplace_back(body, r);
  for (auto& t : th) t.join();
  if (failed) fail(code, msg);
}

static void mg_create(MultiJob& M, const int* devices, int ndev) {
  if (!devices || ndev <= 0 || ndev > 64) fail(SYZGPU_EINVAL, "1..64 devices");
  for (int i = 0; i < ndev; i++) {
    auto s = std::make_unique<MgShard>();
    s->dev = devices[i];
    M.sh.push_back(std::move(s));
  }
  // peer access between the distinct devices (the exchange's copies go over xGMI)
  mg_run(M, [&](int r, auto&& step) {
    step([&] {
      for (int i = 0; i < ndev; i++) {
        const int d = devices[i];
        if (d == M.sh[r]->dev) continue;
        int ok = 0;
        SYZ_HIP(hipDeviceCanAccessPeer(&ok, M.sh[r]->dev, d));
        if (!ok) continue;
        const hipError_t e = hipDeviceEnablePeerAccess(d, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) SYZ_HIP(e);
        (void)hipGetLastError();
      }
    });
  });
}

static void mg_load(MultiJob& M, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                    const uint16_t* prog_len, size_t n, uint32_t G, uint32_t split_largest) {
  if (G == 0 || G > MAX_GROUPS_PM) fail(SYZGPU_EINVAL, "ngroups out of range (1..4096)");
  if (!off || (n && (!group || !prog_len)) || (n && off[n] && !pcs)) fail(SYZGPU_EINVAL, "null pointer");
  if (off[0] != 0) fail(SYZGPU_EINVAL, "off[0] must be 0");
  const int R = (int)M.sh.size();
  std::vector<int64_t> E(G, 0);
  std::vector<double> P(G, 0.0);
  for (size_t e = 0; e < n; e++) {
    if (group[e] >= G) fail(SYZGPU_EINVAL, "group id >= ngroups");
    if (off[e + 1] < off[e]) fail(SYZGPU_EINVAL, "offsets must not decrease");
    E[group[e]]++;
    P[group[e]] += (double)(off[e + 1] - off[e]);
  }
  M.plan = kp::plan_parts(E, P, R, split_largest);
  M.G = G;
  M.n = n;
  M.xgroups.clear();
  M.xoff.clear();
  M.xbytes = 0;
  std::vector<std::vector<uint64_t>> bounds(G);
  for (uint32_t g = 0; g < G; g++)
    if (M.plan.ranks[g].size() > 1) {
      M.xgroups.push_back(g);
      M.xoff.push_back(M.xbytes);
      M.xbytes += (uint64_t)E[g];
      bounds[g] = kp::split_bounds(pcs, off, group, n, g, M.plan.ranks[g].size());
    }
  for (int r = 0; r < R; r++) {
    MgShard& S = *M.sh[r];
    S.key_lo.assign(G, 0);
    S.key_hi.assign(G, 0xFFFFFFFFu);
    S.count.assign(G, 0);
    S.xg.clear();
    S.xo.clear();
    S.parts = false;
    std::vector<uint8_t> held(G, 0);
    for (uint32_t g = 0; g < G; g++) {
      const auto& h = M.plan.ranks[g];
      const auto it = std::find(h.begin(), h.end(), r);
      if (it == h.end()) continue;
      held[g] = 1;
      S.count[g] = h[0] == r;
      if (h.size() > 1) {
        const size_t j = (size_t)(it - h.begin());
        S.key_lo[g] = (uint32_t)bounds[g][j];
        S.key_hi[g] = (uint32_t)(bounds[g][j + 1] - 1);
        S.parts = true;
      }
    }
    for (size_t i = 0; i < M.xgroups.size(); i++)
      if (held[M.xgroups[i]]) {
        S.xg.push_back(M.xgroups[i]);
        S.xo.push_back(M.xoff[i]);
      }
    S.ids.clear();
    for (size_t e = 0; e < n; e++)
      if (held[group[e]]) S.ids.push_back(e);
    S.n = S.ids.size();
  }
  // each sub-job's corpus: its entries' covers, in corpus order, uploaded by its own thread
  mg_run(M, [&](int r, auto&& step) {
    step([&] {
      MgShard& S = *M.sh[r];
      const size_t m = S.n;
      std::vector<uint64_t> lo(m + 1, 0);
      std::vector<uint32_t> lg(m);
      std::vector<uint16_t> ll(m);
      for (size_t i = 0; i < m; i++) {
        const uint64_t e = S.ids[i];
        lo[i + 1] = lo[i] + (off[e + 1] - off[e]);
        lg[i] = group[e];
        ll[i] = prog_len[e];
      }
      std::vector<uint32_t> lp(lo[m]);
      for (size_t i = 0; i < m; i++) {
        const uint64_t e = S.ids[i];
        std::copy(pcs + off[e], pcs + off[e + 1], lp.begin() + lo[i]);
      }
      hipStream_t s = ctx().stream;
      S.pcs.ensure(lo[m] + 1);
      S.off.ensure(m + 1);
      S.grp.ensure(m + 1);
      S.plen.ensure(m + 1);
      if (lo[m]) SYZ_HIP(hipMemcpyAsync(S.pcs.p, lp.data(), lo[m] * 4, hipMemcpyHostToDevice, s));
      SYZ_HIP(hipMemcpyAsync(S.off.p, lo.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
      if (m) {
        SYZ_HIP(hipMemcpyAsync(S.grp.p, lg.data(), m * 4, hipMemcpyHostToDevice, s));
        SYZ_HIP(hipMemcpyAsync(S.plen.p, ll.data(), m * 2, hipMemcpyHostToDevice, s));
      }
      S.sel.ensure(m + 1);
      S.out.ensure(m + 1);
      S.goff.ensure(G + 1);
      if (M.xbytes) {
        S.xbuf.ensure(M.xbytes);
        S.xgather.ensure(M.xbytes * M.sh.size());
      }
      SYZ_HIP(hipStreamSynchronize(s));  // (host temporaries)
    });
  });
  M.loaded = true;
}

struct MgOut {
  int32_t C;
  const float* uses;
  size_t nkeys;
  int64_t *out_idx, *len_hist, *run;
  uint64_t* group_out_off;
  float* prios;
  uint8_t* row_present;
};

static void mg_minimize(MultiJob& M, const MgOut& o) {
  if (!M.loaded) fail(SYZGPU_EINVAL, "load a corpus first");
  if (o.C <= 0 || !o.out_idx || !o.group_out_off || !o.len_hist) fail(SYZGPU_EINVAL, "null pointer or C <= 0");
  const bool prio = o.prios || o.run;
  if (prio && (!o.uses || !o.prios || !o.run)) fail(SYZGPU_EINVAL, "priorities need uses, prios and run");
  const int R = (int)M.sh.size();
  const uint32_t G = M.G;
  const int32_t C = o.C;
  std::vector<int64_t> hist(C + 1, 0);
  mg_run(M, [&](int r, auto&& step) {
    MgShard& S = *M.sh[r];
    hipStream_t s = nullptr;
    // begin: this sub-job's groups (and PC ranges of split ones); its split groups' selection out
    if (!step([&] {
          s = ctx().stream;
          S.hist.ensure(C + 1);
          RawMinArgs a{S.pcs.p, S.off.p, S.grp.p, S.plen.p, S.n, G};
          if (S.parts) {
            a.key_lo = S.key_lo.data();
            a.key_hi = S.key_hi.data();
          }
          a.s = s;
          minimize_raw_begin(*S.job, a);
          if (M.xbytes) {
            SYZ_HIP(hipMemsetAsync(S.xbuf.p, 0, M.xbytes, s));
            if (!S.xg.empty())
              minimize_raw_xchg(*S.job, S.xg.data(), S.xo.data(), (uint32_t)S.xg.size(), S.xbuf.p, 0, s);
          }
          SYZ_HIP(hipStreamSynchronize(s));
        }))
      return;
    // the exchange: every sub-job's buffer to this device, MAX-folded, imported; then end
    if (!step([&] {
          if (M.xbytes) {
            for (int k = 0; k < R; k++)
              SYZ_HIP(hipMemcpyPeerAsync(S.xgather.p + (uint64_t)k * M.xbytes, S.dev, M.sh[k]->xbuf.p, M.sh[k]->dev,
                                         M.xbytes, s));
            k_mg_max_u8<<<grid_for(M.xbytes, 256, 4096), 256, 0, s>>>(S.xbuf.p, S.xgather.p, M.xbytes, (uint32_t)R);
            SYZ_LAUNCHED();
            if (!S.xg.empty())
              minimize_raw_xchg(*S.job, S.xg.data(), S.xo.data(), (uint32_t)S.xg.size(), S.xbuf.p, 1, s);
          }
          RawEndArgs e;
          e.C = C;
          e.count_hist = S.count.data();
          e.selected = S.sel.p;
          e.len_hist = S.hist.p;
          e.out_idx = S.out.p;
          e.group_out_off = S.goff.p;
          e.s = s;
          minimize_raw_end(*S.job, e);  // (waits for the stream: the len(p.Calls) > C check)
          S.h_goff.resize(G + 1);
          SYZ_HIP(hipMemcpyAsync(S.h_goff.data(), S.goff.p, (G + 1) * 8, hipMemcpyDeviceToHost, s));
          SYZ_HIP(hipStreamSynchronize(s));
          S.h_out.resize(S.h_goff[G]);
          if (S.h_goff[G])
            SYZ_HIP(hipMemcpyAsync(S.h_out.data(), S.out.p, S.h_goff[G] * 8, hipMemcpyDeviceToHost, s));
          SYZ_HIP(hipStreamSynchronize(s));
        }))
      return;
    // the histograms summed on the first sub-job's device; the priorities there
    step([&] {
      if (r != 0) return;
      S.hgather.ensure((size_t)(C + 1) * R);
      for (int k = 0; k < R; k++)
        SYZ_HIP(hipMemcpyPeerAsync(S.hgather.p + (size_t)k * (C + 1), S.dev, M.sh[k]->hist.p, M.sh[k]->dev,
                                   (size_t)(C + 1) * 8, s));
      k_mg_sum_i64<<<grid_for(C + 1, 256, 64), 256, 0, s>>>(S.hist.p, S.hgather.p, (uint32_t)(C + 1), (uint32_t)R);
      SYZ_LAUNCHED();
      SYZ_HIP(hipMemcpyAsync(hist.data(), S.hist.p, (size_t)(C + 1) * 8, hipMemcpyDeviceToHost, s));
      if (prio) {
        const size_t cc = (size_t)C * C;
        S.uses.ensure(o.nkeys * C + 1);
        S.stat.ensure(cc);
        S.prios.ensure(cc);
        S.run.ensure(cc);
        S.rowp.ensure(C + 1);
        if (o.nkeys) SYZ_HIP(hipMemcpyAsync(S.uses.p, o.uses, o.nkeys * C * 4, hipMemcpyHostToDevice, s));
        const uint32_t* dserr = static_priorities_enqueue(S.uses.p, o.nkeys, C, S.stat.p, s);
        prio_choice_dev(S.stat.p, S.hist.p, nullptr, C, nullptr, S.prios.p, S.run.p, S.rowp.p, s);
        uint32_t herr = 0;
        SYZ_HIP(hipMemcpyAsync(&herr, dserr, 4, hipMemcpyDeviceToHost, s));
        SYZ_HIP(hipMemcpyAsync(o.prios, S.prios.p, cc * 4, hipMemcpyDeviceToHost, s));
        SYZ_HIP(hipMemcpyAsync(o.run, S.run.p, cc * 8, hipMemcpyDeviceToHost, s));
        if (o.row_present) SYZ_HIP(hipMemcpyAsync(o.row_present, S.rowp.p, C, hipMemcpyDeviceToHost, s));
        SYZ_HIP(hipStreamSynchronize(s));
        static_prio_check(herr);
      }
      SYZ_HIP(hipStreamSynchronize(s));
    });
  });
  // the kept list: each group from its primary, local ids mapped to corpus ids, group-major
  uint64_t pos = 0;
  o.group_out_off[0] = 0;
  for (uint32_t g = 0; g < G; g++) {
    const auto& h = M.plan.ranks[g];
    if (!h.empty()) {
      const MgShard& S = *M.sh[h[0]];
      for (uint64_t i = S.h_goff[g]; i < S.h_goff[g + 1]; i++) o.out_idx[pos++] = (int64_t)S.ids[S.h_out[i]];
    }
    o.group_out_off[g + 1] = pos;
  }
  std::copy(hist.begin(), hist.end(), o.len_hist);
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzgpu_mgz_create(const int* devices, int ndev, syzgpu_mgz** out) {
  try {
    if (!out) fail(SYZGPU_EINVAL, "null pointer");
    auto M = std::make_unique<MultiJob>();
    mg_create(*M, devices, ndev);
    *out = reinterpret_cast<syzgpu_mgz*>(M.release());
    return SYZGPU_OK;
  } catch (const Error& e) {
    set_last_error(e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return SYZGPU_EINTERNAL;
  }
}

int syzgpu_mgz_destroy(syzgpu_mgz* job) {
  if (!job) return SYZGPU_OK;
  MultiJob* M = reinterpret_cast<MultiJob*>(job);
  { std::lock_guard<std::mutex> lk(M->mu); }
  // each sub-job's buffers are freed on its device; the caller's current device is restored
  int cur = 0;
  const bool had = hipGetDevice(&cur) == hipSuccess;
  for (auto& s : M->sh) {
    (void)hipSetDevice(s->dev);
    s.reset();
  }
  if (had) (void)hipSetDevice(cur);
  delete M;
  return SYZGPU_OK;
}

#define SYZ_MG_BODY(...)                               \
  try {                                                \
    if (!job) fail(SYZGPU_EINVAL, "null job");         \
    MultiJob& M = *reinterpret_cast<MultiJob*>(job);   \
    std::lock_guard<std::mutex> lk_(M.mu);             \
    __VA_ARGS__;                                       \
    check_faults();                                    \
    return SYZGPU_OK;                                  \
  } catch (const Error& e) {                           \
    set_last_error(e.msg);                             \
    return e.code;                                     \
  } catch (const std::bad_alloc&) {                    \
    set_last_error("host allocation failed");          \
    return SYZGPU_ENOMEM;                              \
  } catch (const std::exception& e) {                  \
    set_last_error(e.what());                          \
    return SYZGPU_EINTERNAL;                           \
  }

int syzgpu_mgz_load(syzgpu_mgz* job, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                    const uint16_t* prog_len, size_t n, uint32_t ngroups, uint32_t split_largest) {
  SYZ_MG_BODY(mg_load(M, pcs, off, group, prog_len, n, ngroups, split_largest))
}

int syzgpu_mgz_minimize_prio(syzgpu_mgz* job, int32_t C, const float* uses, size_t nkeys, int64_t* out_idx,
                             uint64_t* group_out_off, int64_t* len_hist, float* prios, int64_t* run,
                             uint8_t* row_present) {
  SYZ_MG_BODY(mg_minimize(M, MgOut{C, uses, nkeys, out_idx, len_hist, run, group_out_off, prios, row_present}))
}

int syzgpu_mgz_info(syzgpu_mgz* job, uint64_t* info, size_t cap) {
  SYZ_MG_BODY({
    if (!info) fail(SYZGPU_EINVAL, "null pointer");
    std::vector<uint64_t> v{(uint64_t)M.sh.size(), M.G, M.n, M.xgroups.size(), M.xbytes};
    for (auto& s : M.sh) v.push_back(s->n);
    for (size_t i = 0; i < cap && i < v.size(); i++) info[i] = v[i];
  })
}

// The key-space plan alone (no device): ranks_out[g * nranks + j] = the sub-job holding part j of group g
// (-1 past its parts), cost_out[r] = the modelled step of sub-job r (µs)
int syzgpu_plan_parts(const int64_t* entries, const double* pcs, uint32_t ngroups, int nranks, uint32_t split_largest,
                      int32_t* ranks_out, double* cost_out) {
  try {
    if (!entries || !pcs || !ranks_out || nranks <= 0) fail(SYZGPU_EINVAL, "null pointer or nranks <= 0");
    const std::vector<int64_t> E(entries, entries + ngroups);
    const std::vector<double> P(pcs, pcs + ngroups);
    const kp::Plan p = kp::plan_parts(E, P, nranks, split_largest);
    for (uint32_t g = 0; g < ngroups; g++)
      for (int j = 0; j < nranks; j++)
        ranks_out[(size_t)g * nranks + j] = j < (int)p.ranks[g].size() ? p.ranks[g][j] : -1;
    if (cost_out)
      for (int r = 0; r < nranks; r++) cost_out[r] = p.cost[r];
    return SYZGPU_OK;
  } catch (const Error& e) {
    set_last_error(e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return SYZGPU_EINTERNAL;
  }
}

// split_bounds of group g into k parts (no device): bounds_out[k + 1]
int syzgpu_plan_split_bounds(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n, uint32_t g,
                             uint32_t k, uint64_t* bounds_out) {
  try {
    if (!off || !group || !bounds_out || k == 0) fail(SYZGPU_EINVAL, "null pointer or k == 0");
    const std::vector<uint64_t> b = kp::split_bounds(pcs, off, group, n, g, k);
    std::copy(b.begin(), b.end(), bounds_out);
    return SYZGPU_OK;
  } catch (const Error& e) {
    set_last_error(e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return SYZGPU_EINTERNAL;
  }
}

}  // extern "C"

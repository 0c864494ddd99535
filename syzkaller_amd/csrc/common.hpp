// Shared runtime pieces of libsyzgpu.so: error handling, the per-device context with grow-only
// scratch buffers, and wave64 / workgroup primitives used by every kernel.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/syzgpu.h"

namespace syz {

constexpr uint32_t SENT = 0xFFFFFFFFu;  // cover/cover.go:17

struct Error {
  int code;
  std::string msg;
};

[[noreturn]] void fail(int code, const std::string& msg);
void set_last_error(const std::string& msg);

#define SYZ_HIP(expr)                                                                            \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      ::syz::fail(e_ == hipErrorOutOfMemory ? SYZGPU_ENOMEM : SYZGPU_EHIP,                       \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                            \
  } while (0)

#define SYZ_LAUNCHED() SYZ_HIP(hipGetLastError())

// Grow-only device scratch, keyed by name. Never shrinks within a context; freed at shutdown.
class Scratch {
 public:
  void* get(const std::string& name, size_t bytes);
  template <class T>
  T* get(const std::string& name, size_t count) {
    return static_cast<T*>(get(name, count * sizeof(T) + 16));
  }
  // A buffer whose users return it to all-`fill` bytes before they finish (sparse clean-up instead
  // of a full memset per call). It is filled on (re)allocation, and again when the previous user
  // did not hand it back with put_clean (an error path left it dirty).
  void* get_clean(const std::string& name, size_t bytes, int fill, hipStream_t s);
  template <class T>
  T* get_clean(const std::string& name, size_t count, int fill, hipStream_t s) {
    return static_cast<T*>(get_clean(name, count * sizeof(T) + 16, fill, s));
  }
  void put_clean(const std::string& name) { bufs_[name].clean = true; }
  void release();
  ~Scratch() { release(); }

 private:
  struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    bool clean = false;
  };
  std::map<std::string, Buf> bufs_;
};

// Pinned host staging for small D2H readbacks.
class Pinned {
 public:
  void* get(size_t bytes);
  template <class T>
  T* get(size_t count) {
    return static_cast<T*>(get(count * sizeof(T) + 16));
  }
  ~Pinned();

 private:
  void* p_ = nullptr;
  size_t bytes_ = 0;
};

// A lane: everything one API call works with (streams, scratch, pinned staging, captured graphs).
// Calls hold a lane for their duration; concurrent callers (goroutines, fuzzer procs under coverMu's
// read lock, fuzzer.go:448-456) get different lanes and run concurrently on the device. A thread gets
// the lane it used last when that one is free, so per-thread state (syzgpu_minimize_grouped_fetch)
// survives between its calls; state shared across calls on different threads lives in handles.
struct MinJob;
struct Context {
  int device = -1;
  uint64_t gen = 0;
  hipStream_t stream = nullptr;  // library-owned stream for host-pointer entry points
  Scratch scratch;
  Pinned pinned;
  Pinned pinned_err;  // the raw Minimize's P flags (panels.hip launch_step)
  Pinned pinned_plan;          // the Go sort's plan staging (gosort_plan)
  hipEvent_t ev_plan = nullptr;  // its copies are done
  // the last minimize of this lane (for syzgpu_minimize_grouped_fetch): which thread ran it, on
  // which job; fetch on another thread or after the lane served someone else reports EINVAL
  std::thread::id last_thread;
  const MinJob* last_job = nullptr;
  std::shared_ptr<MinJob> own_job;  // the lane's job for the one-call entry points
  hipStream_t side = nullptr;         // second stream: independent work overlapped with the main one
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipStream_t cap = nullptr;           // capture stream for the gosort round graph
  hipGraphExec_t gl_exec[2][4] = {};  // [start parity][rounds - 1]: global-round graphs
  std::vector<const void*> gl_key;
  unsigned long long* gr_host = nullptr;  // host-mapped progress word of the global rounds
  unsigned long long* gr_dev = nullptr;   // its device address
  uint32_t gr_epoch = 0;
  uint32_t gr_resident = 0;  // workgroups of k_gr_persist resident at once (occupancy x CUs)
  hipStream_t part = nullptr;  // the raw Minimize's transpose pass, beside the Go sort
  hipEvent_t ev_part0 = nullptr, ev_part1 = nullptr;
  hipEvent_t ev_psmall = nullptr;  // P's slabs of the small call groups are cut
  hipEvent_t ev_spin = nullptr;    // stream_wait_spin's marker
  std::vector<hipEvent_t> ev_cnt, ev_sct;  // per batch: count done, scatter done
  int ncu = 0;  // compute units of the device
  // single-pass scans (scan.hpp): per tag and stream, the flag buffer, the tiles it was cleared for, the epoch
  std::unordered_map<std::string, std::pair<void*, std::pair<size_t, uint32_t>>> scan_epoch;
  std::shared_ptr<struct GosortPlan> raw_plan;  // Go-sort plan of the last raw corpus layout
  std::vector<uint64_t> raw_plan_key;
};

// The lane held by the calling thread (inside SYZ_API_BODY); lazily init(0); throws ENODEV. Lanes belong
// to one device each: the process's device by default, another one for the sub-jobs of a multi-device
// job (multi.hip), each run on a thread of its own holding a lane of its device.
Context& ctx();
// The lane's side stream and its fork / join events, created on first use.
inline void ensure_side(Context& c) {
  if (c.side) return;
  SYZ_HIP(hipStreamCreateWithFlags(&c.side, hipStreamNonBlocking));
  SYZ_HIP(hipEventCreateWithFlags(&c.ev_fork, hipEventDisableTiming));
  SYZ_HIP(hipEventCreateWithFlags(&c.ev_join, hipEventDisableTiming));
}
// The calling thread's next (outermost) API call runs on lane c (of generation gen), waiting for it if another thread holds
// it (a lane that no longer exists is ignored): for entries whose result lives on the lane of an earlier
// call (syzgpu_minimize_grouped_fetch). Lane affinity alone is not enough: the thread's lane may be busy
// with another thread's call (a finalizer, a multi-device job's sub-job) when the fetch arrives.
void want_lane(Context* c, uint64_t gen);  // gen: c->gen when c was used
// RAII: hold a lane for the calling thread (nested API calls reuse it).
struct LaneGuard {
  explicit LaneGuard(int device = -1);  // -1: the process's device (syzgpu_init); else a lane of that device
  ~LaneGuard();
  LaneGuard(const LaneGuard&) = delete;
  LaneGuard& operator=(const LaneGuard&) = delete;
};

// Kernel timing (bench roofline). Records named events around launches when enabled.
struct Prof {
  bool on = false;
  bool serial = false;  // (syzgpu_profile_enable(2)) the raw minimize's passes one after another, so each
                        // scope times its kernels alone (the bench's per-kernel pass)
  std::string only;  // when non-empty, only scopes of this name are recorded
  bool match(const char* name) const { return only.empty() || only == name; }
  struct Rec {
    std::string name;
    hipEvent_t a, b;
    uint64_t bytes;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  void reset();
  size_t begin(const char* name, hipStream_t s, uint64_t bytes);
  void end(size_t rec, hipStream_t s);
};
Prof& prof();

struct ProfScope {
  hipStream_t s;
  bool on;
  size_t rec = 0;
  ProfScope(const char* name, hipStream_t st, uint64_t bytes) : s(st), on(prof().on && prof().match(name)) {
    if (on) rec = prof().begin(name, s, bytes);
  }
  void end() {  // (early, before the scope closes)
    if (on) prof().end(rec, s);
    on = false;
  }
  ~ProfScope() { end(); }
};

// Developer switches (A/B variants that lost, timing-only debug modes, some of which give wrong results):
// read from the environment only in the variant and dbg builds (-DSYZ_DEV_KNOBS, Makefile `variant` /
// `dbg`). The production library always takes the default, so a manager that inherits one of these
// variables gets the shipped behaviour. The runtime options the production library reads are listed in
// INTEGRATION.md ("Environment"); none of them changes a result.
inline const char* dev_env(const char* name) {
#ifdef SYZ_DEV_KNOBS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// The process's device fault word: host-mapped, so a kernel that detects an internal failure it has no
// other way to report (scan.hpp's look-back timeout or 2^56 overflow) sets a bit that the host reads
// without a device wait. Every entry point checks it on return (SYZ_API_BODY); once set, calls fail
// with SYZGPU_EINTERNAL (sticky, like a device error).
constexpr uint32_t FAULT_SCAN_WAIT = 1, FAULT_SCAN_RANGE = 2;
uint32_t* fault_word_dev();  // its device address (allocated on first use)
void check_faults();         // fail(SYZGPU_EINTERNAL) when a bit is set

// ---- device-wide scans (scan.hpp, runtime.hip) ----------------------------------------------------------
// out[i] = sum(in[0..i)), out[n] = total. in may be uint8_t / uint32_t / uint64_t.
void exclusive_scan_u8(const uint8_t* in, uint64_t* out, size_t n, hipStream_t s);
// tag: a distinct scratch name for scans that may run on another stream at the same time
void exclusive_scan_u32(const uint32_t* in, uint64_t* out, size_t n, hipStream_t s, const char* tag = "");

// Host-side phase timing for development (SYZGPU_PHASE_TIMING=1: each mark drains the stream and
// prints the wall time since the previous mark to stderr); off, a mark costs nothing.
struct PhaseTimer {
  bool on;
  const char* what;
  std::chrono::steady_clock::time_point t;
  explicit PhaseTimer(const char* w) : on(dev_env("SYZGPU_PHASE_TIMING") != nullptr), what(w), t(std::chrono::steady_clock::now()) {}
  void mark(const char* name, hipStream_t s) {
    if (!on) return;
    (void)hipStreamSynchronize(s);
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "[phase] %s.%s %.3f ms\n", what, name, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};
// host-side time between points (SYZGPU_HOST_TIMING=1; no stream waits, unlike PhaseTimer)
struct HostTimer {
  bool on;
  const char* what;
  std::chrono::steady_clock::time_point t;
  explicit HostTimer(const char* w) : on(dev_env("SYZGPU_HOST_TIMING") != nullptr), what(w), t(std::chrono::steady_clock::now()) {}
  void mark(const char* name) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "[host] %s.%s %.1f us\n", what, name, std::chrono::duration<double, std::micro>(n - t).count());
    t = n;
  }
};
void exclusive_scan_u64(const uint64_t* in, uint64_t* out, size_t n, hipStream_t s);
// Waits for everything issued to s so far by polling an event (no blocking wait: the host turns around
// in microseconds when the plan it waits for is short); falls back to a blocking wait after 50 ms.
void stream_wait_spin(hipStream_t s);
void event_wait_spin(hipEvent_t e);  // the same on an event already recorded

inline unsigned grid_for(size_t n, unsigned block, unsigned cap = 1u << 20) {
  size_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ---- device primitives ---------------------------------------------------------------------
__device__ __forceinline__ unsigned lane64() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  const unsigned l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Compiler + LDS ordering point between lanes of one wave (ds ops of a wave retire in order).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <class T>
__device__ __forceinline__ T wave_incl_scan(T x) {
  const unsigned l = __lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T y = __shfl_up(x, d, 64);
    if (l >= (unsigned)d) x += y;
  }
  return x;
}

// 32-bit inclusive wave64 scan on DPP (row_shr within 16-lane rows, then row_bcast:15 / :31):
// seven VALU steps instead of six LDS-latency shuffles.
template <int CTRL, int ROW, int BANK>
__device__ __forceinline__ uint32_t dpp_add(uint32_t x) {
  return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW, BANK, false);
}
template <>
__device__ __forceinline__ uint32_t wave_incl_scan<uint32_t>(uint32_t v) {
  uint32_t x = v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);             // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x113, 0xF, 0xF, false);             // row_shr:3
  x = dpp_add<0x114, 0xF, 0xE>(x);  // row_shr:4, lanes 4..15 of each row
  x = dpp_add<0x118, 0xF, 0xC>(x);  // row_shr:8, lanes 8..15
  x = dpp_add<0x142, 0xA, 0xF>(x);  // row_bcast:15 into rows 1 and 3
  x = dpp_add<0x143, 0xC, 0xF>(x);  // row_bcast:31 into rows 2 and 3
  return x;
}

// Inclusive wave64 max-scan of int32 on the same DPP sequence (disabled / out-of-row lanes read
// INT_MIN, the identity).
template <int CTRL, int ROW, int BANK>
__device__ __forceinline__ int32_t dpp_max(int32_t x) {
  const int32_t y = __builtin_amdgcn_update_dpp((int)0x80000000, x, CTRL, ROW, BANK, false);
  return x > y ? x : y;
}
__device__ __forceinline__ int32_t wave_incl_max(int32_t v) {
  int32_t x = v;
  const int32_t a = __builtin_amdgcn_update_dpp((int)0x80000000, v, 0x111, 0xF, 0xF, false);
  const int32_t b = __builtin_amdgcn_update_dpp((int)0x80000000, v, 0x112, 0xF, 0xF, false);
  const int32_t c = __builtin_amdgcn_update_dpp((int)0x80000000, v, 0x113, 0xF, 0xF, false);
  x = x > a ? x : a;
  x = x > b ? x : b;
  x = x > c ? x : c;
  x = dpp_max<0x114, 0xF, 0xE>(x);
  x = dpp_max<0x118, 0xF, 0xC>(x);
  x = dpp_max<0x142, 0xA, 0xF>(x);
  x = dpp_max<0x143, 0xC, 0xF>(x);
  return x;
}

template <class T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

template <class T>
__device__ __forceinline__ T wave_min(T x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    T y = __shfl_xor(x, d, 64);
    x = y < x ? y : x;
  }
  return x;
}

// Folds every thread's [lo, hi] into span[0] (min) and span[1] (max): reduced across the workgroup
// first, and each atomic skipped when the running span already covers the block's value (same-address
// atomics from every wave of a large grid serialize). Every thread of the block must call it.
template <int BLOCK>
__device__ __forceinline__ void block_span_update(uint32_t lo, uint32_t hi, uint32_t* span) {
  __shared__ uint32_t red[2][BLOCK / 64];
  lo = wave_min(lo);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t y = __shfl_xor(hi, d, 64);
    hi = y > hi ? y : hi;
  }
  if (__lane_id() == 0) {
    red[0][threadIdx.x >> 6] = lo;
    red[1][threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < BLOCK / 64; i++) {
      lo = min(lo, red[0][i]);
      hi = max(hi, red[1][i]);
    }
    if (lo < __hip_atomic_load(&span[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&span[0], lo);
    if (hi > __hip_atomic_load(&span[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&span[1], hi);
  }
}

// Exclusive scan across a workgroup of BLOCK threads. lds needs BLOCK/64 + 1 slots. Every thread
// reads the (at most 16) wave totals itself: two barriers, no serial pass.
template <int BLOCK, class T>
__device__ __forceinline__ T block_excl_scan(T v, T* lds, T* total) {
  constexpr int W = BLOCK / 64;
  const int w = threadIdx.x >> 6;
  const T x = wave_incl_scan(v);
  if (__lane_id() == 63) lds[w] = x;
  __syncthreads();
  T pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < W; i++) {
    const T t = lds[i];
    pre += i < w ? t : T(0);
    tot += t;
  }
  *total = tot;
  __syncthreads();  // lds reusable
  return x - v + pre;
}

template <int BLOCK, class T>
__device__ __forceinline__ T block_sum(T v, T* lds) {
  T tot;
  block_excl_scan<BLOCK>(v, lds, &tot);
  return tot;
}

template <int BLOCK, class T>
__device__ __forceinline__ T block_min(T v, T* lds) {
  const int w = threadIdx.x >> 6;
  T x = wave_min(v);
  if (__lane_id() == 0) lds[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    T m = lds[0];
    for (int i = 1; i < BLOCK / 64; i++) m = lds[i] < m ? lds[i] : m;
    lds[BLOCK / 64] = m;
  }
  __syncthreads();
  T r = lds[BLOCK / 64];
  __syncthreads();
  return r;
}

// First index in [lo, hi) with a[i] >= v / > v.
template <class T>
__device__ __forceinline__ uint64_t lower_bound_dev(const T* a, uint64_t lo, uint64_t hi, T v) {
  while (lo < hi) {
    uint64_t m = lo + ((hi - lo) >> 1);
    if (a[m] < v)
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}
template <class T>
__device__ __forceinline__ uint64_t upper_bound_dev(const T* a, uint64_t lo, uint64_t hi, T v) {
  while (lo < hi) {
    uint64_t m = lo + ((hi - lo) >> 1);
    if (a[m] <= v)
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

}  // namespace syz

// Entry-point wrapper: runs body under the context lock, converts exceptions to status codes.
#define SYZ_API_BODY(...)                                                                        \
  try {                                                                                          \
    ::syz::LaneGuard lane_;                                                                      \
    ::syz::Context& C_ = ::syz::ctx();                                                           \
    (void)C_;                                                                                    \
    __VA_ARGS__;                                                                                 \
    ::syz::check_faults();                                                                       \
    return SYZGPU_OK;                                                                            \
  } catch (const ::syz::Error& e) {                                                              \
    ::syz::set_last_error(e.msg);                                                                \
    return e.code;                                                                               \
  } catch (const std::bad_alloc&) {                                                              \
    ::syz::set_last_error("host allocation failed");                                             \
    return SYZGPU_ENOMEM;                                                                        \
  } catch (const std::exception& e) {                                                            \
    ::syz::set_last_error(e.what());                                                             \
    return SYZGPU_EINTERNAL;                                                                     \
  }

#include <chrono>
// Context, error state, scratch memory, profiling and the device-wide scans.
#include <condition_variable>
#include <cstdio>
#include <cstdlib>

#include "common.hpp"
#include "scan.hpp"
#include "store.hpp"

namespace syz {

static thread_local std::string g_last_error;

void set_last_error(const std::string& msg) { g_last_error = msg; }

[[noreturn]] void fail(int code, const std::string& msg) { throw Error{code, msg}; }

void* Scratch::get(const std::string& name, size_t bytes) {
  Buf& b = bufs_[name];
  if (b.bytes >= bytes && b.p) return b.p;
  if (b.p) SYZ_HIP(hipFree(b.p));
  b.p = nullptr;
  b.bytes = 0;
  size_t want = bytes < 256 ? 256 : bytes;
  want += want / 8;  // headroom for slightly larger next calls
  SYZ_HIP(hipMalloc(&b.p, want));
  b.bytes = want;
  return b.p;
}

void* Scratch::get_clean(const std::string& name, size_t bytes, int fill, hipStream_t s) {
  void* old = bufs_[name].p;
  void* p = get(name, bytes);
  Buf& b = bufs_[name];
  if (p != old || !b.clean) SYZ_HIP(hipMemsetAsync(p, fill, b.bytes, s));
  b.clean = false;
  return p;
}

void Scratch::release() {
  for (auto& kv : bufs_)
    if (kv.second.p) (void)hipFree(kv.second.p);
  bufs_.clear();
}

void* Pinned::get(size_t bytes) {
  if (bytes_ >= bytes && p_) return p_;
  if (p_) (void)hipHostFree(p_);
  p_ = nullptr;
  // headroom: a plan staged every call grows by a few bytes as the corpus grows, and each regrowth is a
  // free + pinned allocation (hundreds of microseconds on the step's critical path)
  const size_t want = bytes + bytes / 2 + 256;
  SYZ_HIP(hipHostMalloc(&p_, want, hipHostMallocDefault));
  bytes_ = want;
  return p_;
}

Pinned::~Pinned() {
  if (p_) (void)hipHostFree(p_);
}

// ---- lanes -------------------------------------------------------------------------------------------
static std::mutex g_mu;                 // device choice and the lane pool
static std::condition_variable g_cv;
static int g_device = -1;
static uint64_t g_gen = 1;              // bumped by syzgpu_shutdown: lanes of older generations are gone
static std::vector<Context*> g_lanes;
static std::vector<bool> g_busy;
static thread_local Context* t_lane = nullptr;  // held for the current API call
static thread_local int t_depth = 0;
static thread_local Context* t_last = nullptr;   // affinity: the lane this thread used last
static thread_local uint64_t t_last_gen = 0;
static thread_local Context* t_want = nullptr;    // want_lane: the next call runs on this lane (waits for it)
static thread_local uint64_t t_want_gen = 0;

void want_lane(Context* c, uint64_t gen) {  // (c is not dereferenced: it may be gone)
  t_want = c;
  t_want_gen = gen;
}

static size_t max_lanes() {  // per device
  static const size_t v = [] {
    const char* e = getenv("SYZGPU_LANES");
    const long x = e ? atol(e) : 8;
    return (size_t)(x < 1 ? 1 : x > 64 ? 64 : x);
  }();
  return v;
}

static std::vector<int> g_checked;  // devices found to be gfx950 (g_mu held)

static void check_device(int dev) {  // g_mu held
  for (int d : g_checked)
    if (d == dev) return;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) fail(SYZGPU_ENODEV, "no HIP device available");
  if (dev < 0 || dev >= n) fail(SYZGPU_ENODEV, "device index out of range");
  hipDeviceProp_t prop;
  SYZ_HIP(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    fail(SYZGPU_ENODEV, std::string("libsyzgpu is built for gfx950 only, found ") + prop.gcnArchName);
  g_checked.push_back(dev);
}

static void pick_device(int dev) {  // g_mu held
  check_device(dev);
  g_device = dev;
}

static Context* new_lane(int dev) {  // g_mu held
  check_device(dev);
  SYZ_HIP(hipSetDevice(dev));
  std::unique_ptr<Context> c(new Context());
  c->device = dev;
  c->gen = g_gen;
  SYZ_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  g_lanes.push_back(c.get());
  g_busy.push_back(false);
  return c.release();
}

LaneGuard::LaneGuard(int device) {
  if (t_depth++ > 0) {
    if (device >= 0 && t_lane && t_lane->device != device) {
      t_depth--;
      fail(SYZGPU_EINTERNAL, "nested call on another device");
    }
    return;
  }
  // a requested lane (want_lane), for this call only
  Context* const want_req = t_want;
  const uint64_t want_gen = t_want_gen;
  t_want = nullptr;
  std::unique_lock<std::mutex> lk(g_mu);
  try {
    if (g_device < 0) pick_device(device >= 0 ? device : 0);
    const int dev = device >= 0 ? device : g_device;
    // the requested lane, when it still exists: wait for it, whatever else is free
    Context* const want = want_req && want_gen == g_gen ? want_req : nullptr;
    for (;;) {
      size_t pick = g_lanes.size(), mine = 0, wanted = g_lanes.size();
      for (size_t i = 0; i < g_lanes.size(); i++)
        if (g_lanes[i]->device == dev) {
          mine++;
          if (!g_busy[i] && g_lanes[i] == t_last && t_last_gen == g_gen) pick = i;
          if (g_lanes[i] == want) wanted = i;
        }
      if (wanted < g_lanes.size()) {
        if (g_busy[wanted]) {
          g_cv.wait(lk);
          continue;
        }
        pick = wanted;
      }
      if (pick == g_lanes.size())
        for (size_t i = 0; i < g_lanes.size(); i++)
          if (!g_busy[i] && g_lanes[i]->device == dev) {
            pick = i;
            break;
          }
      if (pick == g_lanes.size() && mine < max_lanes()) {
        new_lane(dev);
        pick = g_lanes.size() - 1;
      }
      if (pick < g_lanes.size()) {
        g_busy[pick] = true;
        t_lane = g_lanes[pick];
        t_last = t_lane;
        t_last_gen = g_gen;
        break;
      }
      g_cv.wait(lk);
    }
  } catch (...) {
    t_depth--;
    throw;
  }
  SYZ_HIP(hipSetDevice(t_lane->device));
}

LaneGuard::~LaneGuard() {
  if (--t_depth > 0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t i = 0; i < g_lanes.size(); i++)
    if (g_lanes[i] == t_lane) g_busy[i] = false;
  t_lane = nullptr;
  g_cv.notify_all();  // (waiters may want lanes of different devices)
}

Context& ctx() {
  if (!t_lane) fail(SYZGPU_EINTERNAL, "no lane held (library entry point without SYZ_API_BODY)");
  return *t_lane;
}

static void free_lane(Context* c) {
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  c->own_job.reset();
  c->scratch.release();
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->part) (void)hipStreamDestroy(c->part);
  if (c->cap) (void)hipStreamDestroy(c->cap);
  for (hipEvent_t e : {c->ev_fork, c->ev_join, c->ev_part0, c->ev_part1, c->ev_psmall, c->ev_spin, c->ev_plan})
    if (e) (void)hipEventDestroy(e);
  for (auto& row : c->gl_exec)
    for (auto& g : row)
      if (g) (void)hipGraphExecDestroy(g);
  if (c->gr_host) (void)hipHostFree(c->gr_host);
  delete c;
}

Prof& prof() {
  static Prof p;
  return p;
}

static std::mutex g_prof_mu;

void Prof::reset() {
  recs.clear();
  used = 0;
}

size_t Prof::begin(const char* name, hipStream_t s, uint64_t bytes) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (used + 2 > pool.size()) {
    for (int i = 0; i < 64; i++) {
      hipEvent_t e;
      SYZ_HIP(hipEventCreate(&e));
      pool.push_back(e);
    }
  }
  Rec r{name, pool[used], pool[used + 1], bytes};
  used += 2;
  SYZ_HIP(hipEventRecord(r.a, s));
  recs.push_back(r);
  return recs.size() - 1;
}

void Prof::end(size_t rec, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  SYZ_HIP(hipEventRecord(recs[rec].b, s));
}

// ---- the device fault word (common.hpp) -----------------------------------------------------------------
static std::mutex g_fault_mu;
static uint32_t* g_fault_host = nullptr;
static uint32_t* g_fault_dev = nullptr;

uint32_t* fault_word_dev() {
  std::lock_guard<std::mutex> lk(g_fault_mu);
  if (!g_fault_dev) {
    void* h = nullptr;
    SYZ_HIP(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
    std::memset(h, 0, 64);
    void* d = nullptr;
    SYZ_HIP(hipHostGetDevicePointer(&d, h, 0));
    g_fault_host = static_cast<uint32_t*>(h);
    g_fault_dev = static_cast<uint32_t*>(d);
  }
  return g_fault_dev;
}

void check_faults() {
  const uint32_t* h = g_fault_host;
  if (!h) return;
  const uint32_t f = __atomic_load_n(h, __ATOMIC_RELAXED);
  if (f & FAULT_SCAN_WAIT) fail(SYZGPU_EINTERNAL, "device scan: a look-back never completed (results void)");
  if (f & FAULT_SCAN_RANGE) fail(SYZGPU_EINTERNAL, "device scan: a prefix reached 2^56 (results void)");
}

// ---- device-wide exclusive scans (scan.hpp) ------------------------------------------------------------
__global__ void k_scan_zero(uint64_t* out0, uint64_t* out1) {
  out0[0] = 0;
  if (out1) out1[0] = 0;
}

ScanState scan_state(const char* tag, size_t tiles, int nv, hipStream_t s) {
  if (tiles >= 0xFFFFFFFFull) fail(SYZGPU_EINVAL, "scan too long");
  Context& c = ctx();
  // per tag and stream: scans on other streams never share a ticket or words
  char sk[32];
  snprintf(sk, sizeof sk, "_%p", (void*)s);
  const std::string key = std::string("scan1_") + tag + sk;
  const size_t words = 32 + tiles * nv;  // [0, 32): the ticket's line
  uint64_t* buf = c.scratch.get<uint64_t>(key, words);
  auto& ep = c.scan_epoch[key];
  // a new or grown buffer (its memory may hold anything, the ticket too), or the epochs ran out: cleared
  if (ep.first != buf || ep.second.first < words || ep.second.second >= 63) {
    SYZ_HIP(hipMemsetAsync(buf, 0, words * 8, s));
    ep = {buf, {words, 0u}};
  }
  ep.second.second++;
  return ScanState{buf + 32, reinterpret_cast<uint32_t*>(buf), ep.second.second, fault_word_dev()};
}

uint64_t* scan_scratch(const char* tag, int depth, size_t words) {
  char k[96];
  snprintf(k, sizeof k, "scan2_%s.%d", tag, depth);
  return ctx().scratch.get<uint64_t>(k, words);
}

template <class T>
struct LoadFn {
  const T* in;
  __device__ void operator()(size_t i, uint64_t* v) const { v[0] = (uint64_t)in[i]; }
};

void exclusive_scan_u8(const uint8_t* in, uint64_t* out, size_t n, hipStream_t s) {
  scan_f<1>(LoadFn<uint8_t>{in}, n, out, nullptr, s, "u8");
}
void exclusive_scan_u32(const uint32_t* in, uint64_t* out, size_t n, hipStream_t s, const char* tag) {
  scan_f<1>(LoadFn<uint32_t>{in}, n, out, nullptr, s, tag);
}
void stream_wait_spin(hipStream_t s) {
  Context& c = ctx();
  if (!c.ev_spin) SYZ_HIP(hipEventCreateWithFlags(&c.ev_spin, hipEventDisableTiming));
  SYZ_HIP(hipEventRecord(c.ev_spin, s));
  event_wait_spin(c.ev_spin);
}

// Spins for 200 us (the step's short read-backs come back within it), then polls with the thread
// yielding its core to the manager's other threads for up to 5 ms, then blocks.
void event_wait_spin(hipEvent_t e) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) return;
    if (r != hipErrorNotReady) SYZ_HIP(r);
    const auto dt = std::chrono::steady_clock::now() - t0;
    if (dt > std::chrono::milliseconds(5)) break;
    if (dt > std::chrono::microseconds(200))
      std::this_thread::yield();
    else
      __builtin_ia32_pause();
  }
  SYZ_HIP(hipEventSynchronize(e));
}

void exclusive_scan_u64(const uint64_t* in, uint64_t* out, size_t n, hipStream_t s) {
  scan_f<1>(LoadFn<uint64_t>{in}, n, out, nullptr, s, "u64");
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzgpu_init(int device) {
  try {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_device >= 0) {
      if (g_device == device) return SYZGPU_OK;
      fail(SYZGPU_EINVAL, "already initialised on another device");
    }
    pick_device(device);
    return SYZGPU_OK;
  } catch (const Error& e) {
    set_last_error(e.msg);
    return e.code;
  }
}

// Frees every lane; no call may be in flight (handles created before stay valid: they own their
// device memory).
int syzgpu_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (Context* c : g_lanes) free_lane(c);
  g_lanes.clear();
  g_busy.clear();
  g_device = -1;
  g_gen++;
  return SYZGPU_OK;
}

int syzgpu_device_count(int* n) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return SYZGPU_OK;
}

size_t syzgpu_last_error(char* buf, size_t cap) {
  const std::string& m = g_last_error;
  if (buf && cap) {
    size_t k = m.size() < cap - 1 ? m.size() : cap - 1;
    std::memcpy(buf, m.data(), k);
    buf[k] = 0;
  }
  return m.size();
}

const char* syzgpu_version(void) { return "syzgpu 0.1 gfx950"; }

int syzgpu_profile_enable(int on) {
  prof().on = on != 0;
  prof().serial = on == 2;
  prof().reset();
  return SYZGPU_OK;
}

int syzgpu_debug_fail_grow(int k) {
  syz::grow_fail_countdown().store(k > 0 ? k : 0);
  return SYZGPU_OK;
}

int syzgpu_profile_only(const char* name) {
  prof().only = name ? name : "";
  return SYZGPU_OK;
}

size_t syzgpu_profile_read(char (*names)[48], float* ms, uint64_t* bytes, size_t cap) {
  Prof& p = prof();
  size_t k = 0;
  for (auto& r : p.recs) {
    if (k >= cap) break;
    float t = 0;
    if (hipEventSynchronize(r.b) != hipSuccess) continue;
    if (hipEventElapsedTime(&t, r.a, r.b) != hipSuccess) continue;
    std::snprintf(names[k], 48, "%s", r.name.c_str());
    ms[k] = t;
    bytes[k] = r.bytes;
    k++;
  }
  p.reset();
  return k;
}

}  // extern "C"

// Seeded synthetic corpus generator (bench / test input only; not part of the product path).
//
// prog.Generate is Go and produces no covers (covers come from kcov inside a VM), so the corpora
// that feed the benchmark configs (BASELINE.json) are synthesised with the shape SURVEY.md §8d fixes:
//   group g        ~ Zipf(s) over G calls                  (manager groups by CallName, manager.go:514)
//   |cov|          ~ lognormal(median, sigma), [1, 16383]   (kCoverSize limit, executor.cc:48,563)
//   PCs            60% from a shared "hot" region (power-law), 40% from a group-private slice,
//                  scattered as 0x81000000 + 4*perm(idx); sorted + deduplicated like executor.cc:572-585
//   len(p.Calls)   1 + Geometric(p), clipped to [1, prog_len_max] (only input CalculatePriorities reads)
// Every random draw is a pure function of (seed, entry, draw#) — independent of thread count.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/syzgpu_synth.h"

namespace {

inline uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() { return splitmix(s++); }
  double uniform() { return ((next() >> 11) + 0.5) * (1.0 / 9007199254740992.0); }  // (0,1)
};

struct Layout {
  std::vector<double> group_cdf;
  std::vector<uint64_t> priv_start, priv_size;
  uint64_t hot_size = 0;
  uint64_t perm_a = 1, perm_b = 0;
};

uint64_t gcd(uint64_t a, uint64_t b) {
  while (b) {
    uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

bool make_layout(const syzgpu_synth_params* p, Layout* L) {
  if (p->ngroups == 0 || p->npcs < 16) return false;
  const uint32_t G = p->ngroups;
  std::vector<double> w(G);
  double tot = 0;
  for (uint32_t g = 0; g < G; g++) tot += (w[g] = std::pow(double(g + 1), -p->zipf_s));
  L->group_cdf.resize(G);
  double acc = 0;
  for (uint32_t g = 0; g < G; g++) L->group_cdf[g] = (acc += w[g] / tot);
  L->group_cdf[G - 1] = 1.0;
  L->hot_size = std::max<uint64_t>(1, uint64_t(double(p->npcs) * p->hot_space));
  if (L->hot_size >= p->npcs) L->hot_size = p->npcs / 2;
  const uint64_t priv_total = p->npcs - L->hot_size;
  L->priv_start.resize(G);
  L->priv_size.resize(G);
  // group-private slices proportional to the group's weight, contiguous, covering priv_total
  acc = 0;
  uint64_t prev = 0;
  for (uint32_t g = 0; g < G; g++) {
    acc += w[g] / tot;
    uint64_t end = (g + 1 == G) ? priv_total : uint64_t(acc * double(priv_total));
    if (end < prev) end = prev;
    L->priv_start[g] = L->hot_size + prev;
    L->priv_size[g] = end - prev;
    prev = end;
  }
  // affine bijection over [0, npcs) to scatter PC indices
  uint64_t a = (uint64_t(p->npcs) * 2654435761ull / 1000003ull) | 1;
  a %= p->npcs;
  if (a < 2) a = 2;
  while (gcd(a, p->npcs) != 1) a++;
  L->perm_a = a;
  L->perm_b = splitmix(p->seed ^ 0xABCDEF) % p->npcs;
  return true;
}

inline uint32_t pc_of(const syzgpu_synth_params* p, const Layout& L, uint64_t idx) {
  uint64_t v = (L.perm_a * idx + L.perm_b) % p->npcs;
  return uint32_t(0x81000000ull + 4ull * v);
}

template <class F>
void parallel_for(uint64_t n, int nthreads, F f) {
  if (nthreads <= 1 || n < 1024) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  uint64_t chunk = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; t++) {
    uint64_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo >= hi) break;
    th.emplace_back([=] { f(lo, hi); });
  }
  for (auto& t : th) t.join();
}

}  // namespace

extern "C" void syzgpu_synth_default_params(syzgpu_synth_params* p, uint64_t seed, uint64_t n,
                                            uint32_t ngroups, uint32_t npcs) {
  std::memset(p, 0, sizeof(*p));
  p->seed = seed;
  p->n = n;
  p->ngroups = ngroups;
  p->npcs = npcs;
  p->zipf_s = 1.1;
  p->len_median = 256.0;
  p->len_sigma = 1.0;
  p->len_max = 16383;
  p->hot_frac = 0.6;
  p->hot_space = 0.3;
  p->hot_exponent = 3.0;
  p->prog_len_max = 40;
  p->prog_len_p = 0.3;
}

extern "C" int syzgpu_synth_layout(const syzgpu_synth_params* p, uint32_t* group, uint64_t* off,
                                   uint16_t* prog_len) {
  Layout L;
  if (!make_layout(p, &L)) return 1;
  off[0] = 0;
  for (uint64_t e = 0; e < p->n; e++) {
    Rng r(splitmix(p->seed * 0x100000001B3ull + e));
    double u = r.uniform();
    uint32_t g = uint32_t(std::lower_bound(L.group_cdf.begin(), L.group_cdf.end(), u) -
                          L.group_cdf.begin());
    if (g >= p->ngroups) g = p->ngroups - 1;
    group[e] = g;
    // lognormal length via Box-Muller
    double u1 = r.uniform(), u2 = r.uniform();
    double z = std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    double lf = std::exp(std::log(p->len_median) + p->len_sigma * z);
    uint64_t len = lf < 1.0 ? 1 : (lf > p->len_max ? p->len_max : uint64_t(lf));
    uint64_t pool = L.hot_size + L.priv_size[g];
    if (len > pool) len = pool;
    off[e + 1] = off[e] + len;
    if (prog_len) {
      double v = std::floor(std::log(r.uniform()) / std::log(1.0 - p->prog_len_p));
      uint64_t pl = 1 + (v > 1e6 ? 1000000 : uint64_t(v));
      if (pl > p->prog_len_max) pl = p->prog_len_max;
      prog_len[e] = uint16_t(pl);
    }
  }
  return 0;
}

extern "C" int syzgpu_synth_fill_ids(const syzgpu_synth_params* p, const uint64_t* ids, const uint32_t* group,
                                     const uint64_t* off, uint64_t n, uint32_t* pcs, int nthreads) {
  Layout L;
  if (!make_layout(p, &L)) return 1;
  parallel_for(n, nthreads, [&](uint64_t lo, uint64_t hi) {
    std::vector<uint32_t> buf;
    for (uint64_t k = lo; k < hi; k++) {
      const uint64_t e = ids ? ids[k] : k;  // global entry id: seeds the draws
      const uint32_t g = group[k];
      const uint64_t len = off[k + 1] - off[k];
      Rng r(splitmix((p->seed ^ 0x5EED5EEDull) * 0x100000001B3ull + e));
      buf.clear();
      uint64_t attempts = 0;
      while (buf.size() < len && attempts < 64) {
        attempts++;
        uint64_t need = len - buf.size();
        for (uint64_t i = 0; i < need; i++) {
          uint64_t idx;
          if (L.priv_size[g] == 0 || r.uniform() < p->hot_frac) {
            double x = std::pow(r.uniform(), p->hot_exponent);
            idx = uint64_t(x * double(L.hot_size));
            if (idx >= L.hot_size) idx = L.hot_size - 1;
          } else {
            idx = L.priv_start[g] + (r.next() % L.priv_size[g]);
          }
          buf.push_back(pc_of(p, L, idx));
        }
        std::sort(buf.begin(), buf.end());
        buf.erase(std::unique(buf.begin(), buf.end()), buf.end());
      }
      // pool exhausted by rejection: pad deterministically from the group's private slice / hot set
      for (uint64_t k = 0; buf.size() < len && k < L.hot_size + L.priv_size[g]; k++) {
        uint64_t idx = k < L.priv_size[g] ? L.priv_start[g] + k : k - L.priv_size[g];
        uint32_t pc = pc_of(p, L, idx);
        if (!std::binary_search(buf.begin(), buf.end(), pc)) {
          buf.insert(std::upper_bound(buf.begin(), buf.end(), pc), pc);
        }
      }
      std::memcpy(pcs + off[k], buf.data(), len * sizeof(uint32_t));
    }
  });
  return 0;
}

extern "C" int syzgpu_synth_fill(const syzgpu_synth_params* p, const uint32_t* group,
                                 const uint64_t* off, uint32_t* pcs, int nthreads) {
  return syzgpu_synth_fill_ids(p, nullptr, group, off, p->n, pcs, nthreads);
}

// ---- serialized programs (prog.Serialize's text shape, prog/encoding.go:19-117) -------------------
namespace {
const char* const kCallNames[] = {
    "mmap", "openat$dir", "open", "close", "read", "write", "ioctl$sock_SIOCGIFINDEX", "socket$inet6_tcp",
    "bind$inet6", "connect$inet6", "sendmsg$netlink", "recvmsg", "setsockopt$inet_tcp_int", "getsockopt",
    "epoll_create1", "epoll_ctl$EPOLL_CTL_ADD", "pipe2", "dup3", "fcntl$setflags", "getpid", "clone",
    "ptrace$peek", "keyctl$join", "add_key$user", "bpf$PROG_LOAD", "perf_event_open", "io_setup",
    "io_submit", "memfd_create", "fallocate", "write$binfmt_elf64", "syz_open_dev$tty1"};
const char* const kArgs[] = {"0x0", "0x1", "0xffffffffffffffff", "&(0x7f0000000000)='./file0\\x00'",
                             "&(0x7f0000001000/0x1000)=nil", "0x3", "&(0x7f0000002000)={0x2, 0x4e20}",
                             "&(0x7f0000003000)=\"a5ff\"", "0x40", "0x8912"};

void prog_text(uint64_t seed, uint64_t i, uint32_t ncalls, std::string& s) {
  Rng r(splitmix(seed * 0x100000001B3ull + i));
  s.clear();
  if (r.uniform() < 0.1) s += "# https://syzkaller.appspot.com/bug?id=" + std::to_string(r.next() % 100000) + "\n";
  for (uint32_t c = 0; c < ncalls; c++) {
    if (r.uniform() < 0.03) s += r.uniform() < 0.5 ? "\n" : "#\n";
    if (r.uniform() < 0.5) s += "r" + std::to_string(c) + " = ";
    s += kCallNames[r.next() % (sizeof(kCallNames) / sizeof(kCallNames[0]))];
    s += "(";
    const int nargs = (int)(r.next() % 7);
    for (int a = 0; a < nargs; a++) {
      if (a) s += ", ";
      if (c > 0 && r.uniform() < 0.15)
        s += "r" + std::to_string(r.next() % c);
      else
        s += kArgs[r.next() % (sizeof(kArgs) / sizeof(kArgs[0]))];
    }
    s += ")";
    if (r.uniform() < 0.02) s += "\r";
    if (c + 1 < ncalls || r.uniform() < 0.9) s += "\n";
  }
}
}  // namespace

extern "C" int syzgpu_synth_prog_text(uint64_t seed, const uint16_t* prog_len, uint64_t n, uint64_t* off,
                                      uint8_t* data, int nthreads) {
  if (!prog_len || !off) return 1;
  if (!data) {  // sizes pass: off[0..n]
    std::vector<uint64_t> len(n);
    parallel_for(n, nthreads, [&](uint64_t b, uint64_t e) {
      std::string s;
      for (uint64_t i = b; i < e; i++) {
        prog_text(seed, i, prog_len[i], s);
        len[i] = s.size();
      }
    });
    off[0] = 0;
    for (uint64_t i = 0; i < n; i++) off[i + 1] = off[i] + len[i];
    return 0;
  }
  parallel_for(n, nthreads, [&](uint64_t b, uint64_t e) {
    std::string s;
    for (uint64_t i = b; i < e; i++) {
      prog_text(seed, i, prog_len[i], s);
      std::memcpy(data + off[i], s.data(), s.size());
    }
  });
  return 0;
}

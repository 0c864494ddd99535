// Driver of the host-side planners (syzkaller_amd/csrc/plan_host.cpp) under AddressSanitizer +
// UndefinedBehaviorSanitizer (tests/test_sanitizers.py, `make -C syzkaller_amd san`): seeded random
// layouts (empty and one-entry call groups, group counts up to MAX_GROUPS, PC spans up to 2^32, key
// parts) through plan_windows, slab_plan, plan_items, gosort_segments and the multi-device plan, with
// each result's invariants checked. Prints "ok".
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <stdexcept>

#include "plan_host.hpp"

namespace syz {
[[noreturn]] void fail(int code, const std::string& msg) { throw std::runtime_error(std::to_string(code) + ": " + msg); }
}  // namespace syz

using namespace syz;

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

struct Layout {
  uint32_t G;
  std::vector<uint64_t> hstart, hpcs;
  uint64_t span;
  uint32_t lo;
};

static Layout random_layout(std::mt19937_64& r) {
  Layout L;
  const uint32_t pick = (uint32_t)(r() % 4);
  L.G = pick == 0 ? 1 + (uint32_t)(r() % 4) : pick == 1 ? 1 + (uint32_t)(r() % 300) : 1 + (uint32_t)(r() % 4096);
  L.hstart.assign(L.G + 1, 0);
  L.hpcs.assign(L.G, 0);
  const double s = 0.5 + (double)(r() % 100) / 50.0;  // Zipf-ish skew
  const uint64_t scale = 1 + r() % 400000;
  for (uint32_t g = 0; g < L.G; g++) {
    uint64_t n = (uint64_t)((double)scale / std::pow((double)(g + 1), s));
    if (r() % 10 == 0) n = r() % 2;  // empty and one-entry groups
    L.hstart[g + 1] = L.hstart[g] + n;
    L.hpcs[g] = n * (1 + r() % 900);
  }
  const uint32_t sb = 10 + (uint32_t)(r() % 23);
  L.span = sb >= 32 ? (1ull << 32) : (1ull << sb) + r() % (1ull << sb);
  if (L.span > (1ull << 32)) L.span = 1ull << 32;
  L.lo = (uint32_t)(r() % ((1ull << 32) - L.span + 1));
  return L;
}

static void check_windows(const Layout& L, const std::vector<PGroup>& pg) {
  CHECK(pg.size() == L.G);
  for (uint32_t g = 0; g < L.G; g++) {
    const PGroup& p = pg[g];
    CHECK(p.S >= DS && p.S <= 32);
    CHECK(p.W >= 1);
    CHECK((uint64_t)p.W == std::max<uint64_t>(1, (L.span + (1ull << p.S) - 1) >> p.S));
    CHECK(p.mode <= PMODE_PACKED);
    if (p.mode == PMODE_PACKED) CHECK(p.S <= PSMAX);
    if (p.mode == PMODE_DIRECT) CHECK(p.S == DS);
  }
}

static void check_slabs(const Layout& L, const std::vector<PGroup>& pg, const SlabPlan& J) {
  CHECK(J.hsg.size() == L.G && J.hgblock.size() == L.G + 1 && J.hbgroup.size() == J.B);
  uint64_t d = 0, x = 0, bound = 0, pcs = 0;
  for (uint32_t g = 0; g < L.G; g++) {
    const SGroup& s = J.hsg[g];
    CHECK(s.dbase == d && s.xbase == x && s.S == pg[g].S && s.W == pg[g].W);
    CHECK(s.memb >= 1 && s.memb <= SL_MEMB);
    const uint64_t ng = L.hstart[g + 1] - L.hstart[g];
    CHECK(J.hgblock[g + 1] - J.hgblock[g] == (ng + s.memb - 1) / s.memb);
    for (uint32_t b = J.hgblock[g]; b < J.hgblock[g + 1]; b++) CHECK(J.hbgroup[b] == g);
    // a block's slabs fit the group's D row: tiles <= PCs / 64 + members
    CHECK((uint64_t)s.stride * SL_TILES >= L.hpcs[g] / 64 + ng);
    d += (uint64_t)(s.W + 1) * s.stride;
    x += s.stride * slab_pad(s.W);
    bound += s.stride;
    pcs += L.hpcs[g];
  }
  CHECK(J.dtotal == d && J.xtotal == x && J.slab_bound == bound && J.total_pcs == pcs);
}

static void check_items(const Layout& L, const std::vector<PGroup>& pg, const ItemPlan& P, const uint32_t* klo,
                        const uint32_t* khi, uint32_t lo, uint32_t hi) {
  size_t tot = 0;
  for (int b = 0; b < 2; b++)
    for (int m = 0; m < 3; m++) {
      CHECK(P.ifirst[b][m] == tot);
      tot += P.icount[b][m];
    }
  CHECK(tot == P.items.size());
  std::set<std::pair<uint32_t, uint32_t>> seen;
  for (int b = 0; b < 2; b++)
    for (int m = 0; m < 3; m++)
      for (size_t i = P.ifirst[b][m]; i < P.ifirst[b][m] + P.icount[b][m]; i++) {
        const PItem it = P.items[i];
        CHECK(it.g < L.G && it.w < pg[it.g].W && (int)pg[it.g].mode == m);
        CHECK((L.hstart[it.g + 1] - L.hstart[it.g] > GS_T_SEG) == (b == 1));
        CHECK(L.hpcs[it.g] > 0);
        if (klo) {  // a key part walks only the windows of its range
          const uint64_t a = ((uint64_t)std::max(klo[it.g], lo) - lo) >> pg[it.g].S;
          const uint64_t z = ((uint64_t)std::min(khi[it.g], hi) - lo) >> pg[it.g].S;
          CHECK(it.w >= a && it.w <= z);
        }
        CHECK(seen.insert({it.g, it.w}).second);
      }
  if (!klo) {
    size_t want = 0;
    for (uint32_t g = 0; g < L.G; g++)
      if (L.hpcs[g]) want += pg[g].W;
    CHECK(want == P.items.size());
  }
}

static void check_segments(const Layout& L, const std::vector<Seg>& small, const std::vector<Pack>& packs,
                           const std::vector<Seg>& big) {
  // packs and big groups tile [0, n) in order
  struct R {
    uint64_t lo, hi;
  };
  std::vector<R> rs;
  for (const Pack& p : packs) rs.push_back({p.plo, p.phi});
  for (const Seg& s : big) rs.push_back({s.lo, s.hi});
  std::sort(rs.begin(), rs.end(), [](const R& a, const R& b) { return a.lo < b.lo; });
  uint64_t cov = 0;
  for (const R& r : rs) {
    CHECK(r.lo == cov && r.hi > r.lo);
    cov = r.hi;
  }
  CHECK(cov == L.hstart[L.G]);
  for (const Pack& p : packs) {
    CHECK(p.phi - p.plo <= GS_T_SEG && p.sbeg <= p.send && p.send <= small.size());
    for (uint32_t k = p.sbeg; k < p.send; k++) CHECK(small[k].lo >= p.plo && small[k].hi <= p.phi);
  }
  for (const Seg& s : small) CHECK(s.hi - s.lo > 1 && s.hi - s.lo <= GS_T_SEG && s.depth == go_max_depth(s.hi - s.lo));
  for (const Seg& s : big) CHECK(s.hi - s.lo > GS_T_SEG && s.depth == go_max_depth(s.hi - s.lo));
}

int main() {
  std::mt19937_64 r(20261018);
  int nplans = 0;
  for (int it = 0; it < 400; it++) {
    const Layout L = random_layout(r);
    std::vector<PGroup> pg;
    plan_windows(L.span, L.hpcs.data(), L.hstart.data(), L.G, pg);
    check_windows(L, pg);
    SlabPlan J;
    try {
      slab_plan(J, L.hstart, L.hpcs.data(), pg, L.G, (it & 1) != 0);
    } catch (const std::runtime_error&) {
      continue;  // a layout past the 32-bit element offsets is rejected (EINVAL), not planned
    }
    check_slabs(L, pg, J);
    const uint32_t hi = (uint32_t)(L.lo + (L.span - 1));
    ItemPlan P;
    plan_items(L.hstart, L.hpcs, L.hpcs.data(), pg, L.G, nullptr, nullptr, L.lo, hi, P);
    check_items(L, pg, P, nullptr, nullptr, L.lo, hi);
    // key parts: a random sub-range of every group
    std::vector<uint32_t> klo(L.G), khi(L.G);
    for (uint32_t g = 0; g < L.G; g++) {
      const uint64_t a = L.lo + r() % L.span, b = L.lo + r() % L.span;
      klo[g] = (uint32_t)std::min(a, b);
      khi[g] = (uint32_t)std::max(a, b);
      if (r() % 8 == 0) klo[g] = 0, khi[g] = 0xFFFFFFFFu;
    }
    plan_items(L.hstart, L.hpcs, L.hpcs.data(), pg, L.G, klo.data(), khi.data(), L.lo, hi, P);
    check_items(L, pg, P, klo.data(), khi.data(), L.lo, hi);
    std::vector<Seg> small, big;
    std::vector<Pack> packs;
    if (L.hstart[L.G] < 0xFFFFFFF0ull) {
      gosort_segments(L.hstart, L.G, small, packs, big);
      check_segments(L, small, packs, big);
    }
    // the multi-device plan over 1..8 sub-jobs
    std::vector<int64_t> E(L.G);
    std::vector<double> Pc(L.G);
    for (uint32_t g = 0; g < L.G; g++) {
      E[g] = (int64_t)(L.hstart[g + 1] - L.hstart[g]);
      Pc[g] = (double)L.hpcs[g];
    }
    const int R = 1 + (int)(r() % 8);
    const kp::Plan kpl = kp::plan_parts(E, Pc, R, (it % 5 == 0) ? (uint32_t)(1 + r() % 9) : 0u);
    CHECK(kpl.ranks.size() == L.G && kpl.cost.size() == (size_t)R);
    for (uint32_t g = 0; g < L.G; g++) {
      const auto& h = kpl.ranks[g];
      CHECK(E[g] == 0 ? h.empty() : !h.empty());
      CHECK(h.size() <= (size_t)R);
      std::set<int> u(h.begin(), h.end());
      CHECK(u.size() == h.size());
      for (int x : h) CHECK(x >= 0 && x < R);
    }
    nplans++;
  }
  // split bounds over a small random corpus
  for (int it = 0; it < 50; it++) {
    const uint32_t G = 1 + (uint32_t)(r() % 5);
    const size_t n = r() % 3000;
    std::vector<uint32_t> group(n), pcs;
    std::vector<uint64_t> off(n + 1, 0);
    for (size_t e = 0; e < n; e++) {
      group[e] = (uint32_t)(r() % G);
      const size_t len = r() % 50;
      uint32_t pc = (uint32_t)(r() % 1000);
      for (size_t k = 0; k < len; k++) pcs.push_back(pc += 1 + (uint32_t)(r() % 1000));
      off[e + 1] = pcs.size();
    }
    for (uint32_t g = 0; g < G; g++) {
      const size_t k = 1 + r() % 8;
      const std::vector<uint64_t> b = kp::split_bounds(pcs.data(), off.data(), group.data(), n, g, k);
      CHECK(b.size() == k + 1 && b.front() == 0 && b.back() == (1ull << 32));
      for (size_t j = 1; j < b.size(); j++) CHECK(b[j] > b[j - 1]);
    }
  }
  std::printf("ok %d layouts\n", nplans);
  return 0;
}

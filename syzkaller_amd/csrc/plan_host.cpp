// Host-side planners (plan_host.hpp): plain C++, compiled into libsyzgpu.so and, under ASan + UBSan, into
// the planner test driver (tests/planner_san.cpp).
#include "plan_host.hpp"

#include <algorithm>
#include <numeric>

namespace syz {

// ---- windows: panels.hip's per-call window size ---------------------------------------------------------
void plan_windows(uint64_t span, const uint64_t* gpcs, const uint64_t* gstart, uint32_t G, std::vector<PGroup>& pg) {
  pg.assign(G, PGroup{});
  auto nwin = [&](uint32_t S) { return (span + (1ull << S) - 1) >> S; };
  uint32_t smin = DS;
  while (smin < 32 && nwin(smin) > WMAX) smin++;
  const uint64_t w15 = nwin(DS);
  for (uint32_t g = 0; g < G; g++) {
    const uint64_t E = gpcs[g];
    PGroup& p = pg[g];
    if (smin == DS && E >= (uint64_t)DENSE * w15) {
      p.S = DS;
      p.W = (uint32_t)w15;
      p.mode = PMODE_DIRECT;
      continue;
    }
    // sparse: the widest window (<= 2^SMAX addresses) that still gives about HTARGET PCs per window;
    // a group of < 2^13 entries whose windows fit 2^19 addresses takes the packed table (2x the PCs)
    const bool small = gstart[g + 1] - gstart[g] < (1u << PK_RBITS);
    const uint64_t tgt = small ? PHTARGET : HTARGET;
    const uint64_t want = std::max<uint64_t>(1, std::min<uint64_t>(WMAX, (E + tgt - 1) / tgt));
    uint32_t S = std::max(smin, DS);
    while (S < SMAX && nwin(S + 1) >= want) S++;
    if (S > SMAX) S = SMAX;
    if (small && S > PSMAX && nwin(PSMAX) <= WMAX) S = PSMAX;
    p.S = S;
    p.W = (uint32_t)std::max<uint64_t>(1, nwin(S));
    p.mode = small && S <= PSMAX ? PMODE_PACKED : PMODE_HASH;
  }
}

// ---- slabs: blocks of members, D rows, element-slot bounds -----------------------------------------------
void slab_plan(SlabPlan& J, const std::vector<uint64_t>& hstart, const uint64_t* hpcs, const std::vector<PGroup>& hpg,
               uint32_t G, bool want_wtot) {
  J.G = G;
  J.hsg.assign(G, SGroup{});
  J.hgblock.assign(G + 1, 0);
  J.hbgroup.clear();
  J.slab_bound = J.dtotal = J.wtotal = J.total_pcs = J.xtotal = 0;
  J.wmax = 1;
  for (uint32_t g = 0; g < G; g++) {
    const uint64_t ng = hstart[g + 1] - hstart[g];
    const uint32_t S = hpg[g].S, W = hpg[g].W;
    // a member's tag fits 32 - S bits, and the all-ones tag is never a member's (SL_NONE: padding)
    const uint32_t memb = S <= 23 ? SL_MEMB : (1u << (32 - S)) - 1;
    const uint64_t nb = (ng + memb - 1) / memb;
    J.hgblock[g + 1] = J.hgblock[g] + (uint32_t)nb;
    J.hbgroup.insert(J.hbgroup.end(), nb, g);
    // slabs of a block: ceil(tiles / SL_TILES); tiles <= PCs / 64 + members
    const uint64_t stride = (hpcs[g] / 64 + ng) / SL_TILES + nb + 1;
    // a group's element offsets (D) are 32-bit
    if (hpcs[g] + stride * slab_pad(W) + 8 >= (1ull << 32)) fail(SYZGPU_EINVAL, "a call group with 2^32 or more PCs");
    // per-window totals (wtot) only for the hashed groups of a job that asks for them
    const bool wt = want_wtot && hpg[g].mode == PMODE_HASH;
    J.hsg[g] = SGroup{J.dtotal, S, W, (uint32_t)stride, memb, wt ? (uint32_t)J.wtotal : SG_NO_WTOT, 0, J.xtotal};
    J.wmax = std::max(J.wmax, W);
    J.xtotal += stride * slab_pad(W);
    J.dtotal += (uint64_t)(W + 1) * stride;
    if (wt) J.wtotal += W;
    J.slab_bound += stride;
    J.total_pcs += hpcs[g];
  }
  if (J.wtotal >= (1ull << 32) || J.slab_bound >= (1ull << 31)) fail(SYZGPU_EINVAL, "too many slabs");
  J.B = J.hgblock[G];
}

// ---- M's work items ----------------------------------------------------------------------------------------
void plan_items(const std::vector<uint64_t>& hstart, const std::vector<uint64_t>& hpcs, const uint64_t* hsl,
                const std::vector<PGroup>& hpg, uint32_t G, const uint32_t* key_lo, const uint32_t* key_hi,
                uint32_t lo, uint32_t hi, ItemPlan& P) {
  P = ItemPlan{};
  const auto is_big = [&](uint32_t g) { return hstart[g + 1] - hstart[g] > GS_T_SEG; };
  std::vector<uint32_t> order(G);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t x, uint32_t y) { return hpcs[x] / hpg[x].W > hpcs[y] / hpg[y].W; });
  std::vector<uint32_t> iw0(G, 0), iw1(G, 0);
  for (uint32_t g : order) {
    if (!hpcs[g]) continue;
    uint32_t w0 = 0, w1 = hpg[g].W;
    if (key_lo) {
      const uint32_t klo = std::max(key_lo[g], lo), khi = std::min(key_hi[g], hi);
      if (klo > khi) continue;
      w0 = (klo - lo) >> hpg[g].S;
      w1 = std::min<uint32_t>(hpg[g].W, ((khi - lo) >> hpg[g].S) + 1);
    }
    iw0[g] = w0;
    iw1[g] = w1;
    P.icount[is_big(g) ? 1 : 0][hpg[g].mode] += w1 - w0;
    P.item_pcs[is_big(g) ? 1 : 0][hpg[g].mode] += hsl[g];
  }
  size_t nitems = 0;
  for (int big = 0; big < 2; big++)
    for (int m = 0; m < 3; m++) {
      P.ifirst[big][m] = nitems;
      nitems += P.icount[big][m];
    }
  P.items.resize(nitems);
  std::array<std::array<size_t, 3>, 2> at = P.ifirst;
  for (uint32_t g : order) {
    size_t& k = at[is_big(g) ? 1 : 0][hpg[g].mode];
    for (uint32_t w = iw0[g]; w < iw1[g]; w++) P.items[k++] = PItem{g, w};
  }
  for (uint32_t g = 0; g < G; g++) {
    P.cpcs[is_big(g) ? 1 : 0] += hsl[g];
    P.cent[is_big(g) ? 1 : 0] += hstart[g + 1] - hstart[g];
  }
}

// ---- the Go sort's segments and packs ------------------------------------------------------------------------
// Packs of consecutive small call groups: at most GS_T_SEG elements (the LDS sorter's capacity), and at
// most n / GS_PACK_DIV so that a small corpus still spreads over many workgroups (config 1's 10k entries
// in one pack: one workgroup, 184 us). The packs and the big groups tile [0, n): the entries of one-entry
// groups between them belong to a pack's range (or to a pack of no segments), so the pack ranks pass
// gives them their rank (their position) too.
void gosort_segments(const std::vector<uint64_t>& hstart, uint32_t ngroups, std::vector<Seg>& small,
                     std::vector<Pack>& packs, std::vector<Seg>& big) {
  small.clear();
  packs.clear();
  big.clear();
  constexpr uint32_t T_SEG = GS_T_SEG;
  const uint64_t n_all = hstart[ngroups];
  const uint64_t pack_cap = std::min<uint64_t>(T_SEG, std::max<uint64_t>(64, n_all / GS_PACK_DIV));
  uint64_t cov = 0;  // [0, cov) is covered by a pack or a big group
  auto cover_to = [&](uint64_t x) {  // one-entry groups' entries [cov, x)
    if (cov >= x) return;
    if (!packs.empty() && packs.back().phi == cov && x - packs.back().plo <= T_SEG) {
      packs.back().phi = (uint32_t)x;
    } else {
      for (; cov < x; cov = std::min<uint64_t>(x, cov + T_SEG))
        packs.push_back(Pack{(uint32_t)cov, (uint32_t)std::min<uint64_t>(x, cov + T_SEG), (uint32_t)small.size(),
                             (uint32_t)small.size()});
    }
    cov = x;
  };
  for (uint32_t g = 0; g < ngroups; g++) {
    const uint32_t lo = (uint32_t)hstart[g], hi = (uint32_t)hstart[g + 1];
    if (hi - lo <= 1) continue;
    const Seg sg{lo, hi, go_max_depth(hi - lo), 0};
    if (hi - lo > T_SEG) {
      cover_to(lo);
      big.push_back(sg);
      cov = hi;
      continue;
    }
    if (!packs.empty() && packs.back().phi == cov && hi - packs.back().plo <= pack_cap) {
      packs.back().phi = hi;
      packs.back().send++;
    } else {
      if (hi - cov > T_SEG) cover_to(lo);
      packs.push_back(Pack{(uint32_t)cov, hi, (uint32_t)small.size(), (uint32_t)small.size() + 1});
    }
    small.push_back(sg);
    cov = hi;
  }
  cover_to(n_all);
}

// ---- the multi-device job's key-space plan: syzkaller_amd/sharding.py plan_parts / _assign /
// split_bounds, restated with the same cost model and tie-breaking (tests/test_multi.py compares them) ------
namespace kp {
constexpr int64_t SMALL_GROUP = 8192;
constexpr double LAT_REF_US = 290.0;   // the Go sort's dependent rounds once a rank holds a big group
constexpr double US_PER_PC = 4.26e-6;  // per streamed PC (transpose + first-occurrence tables)
constexpr double US_PER_ENTRY = 1.24e-3;
constexpr double SMALL_PC_FRACTION = 0.3;

static double sort_latency_us(int64_t n) { return n <= SMALL_GROUP ? 0.0 : LAT_REF_US; }

static Plan assign(const std::vector<int64_t>& E, const std::vector<double>& P, const std::vector<int64_t>& k, int R) {
  const size_t G = E.size();
  std::vector<double> lat(G), w(G);
  for (size_t g = 0; g < G; g++) {
    lat[g] = sort_latency_us(E[g]);
    const double f = E[g] > SMALL_GROUP ? 1.0 : SMALL_PC_FRACTION;
    w[g] = US_PER_PC * P[g] * f / (double)std::max<int64_t>(k[g], 1) + US_PER_ENTRY * (double)E[g];
  }
  struct Item {
    double c;
    uint32_t g, j;
  };
  std::vector<Item> items;
  for (size_t g = 0; g < G; g++)
    if (E[g] > 0)
      for (int64_t j = 0; j < k[g]; j++) items.push_back(Item{lat[g] + w[g], (uint32_t)g, (uint32_t)j});
  std::sort(items.begin(), items.end(), [](const Item& a, const Item& b) {
    if (a.c != b.c) return a.c > b.c;
    if (a.g != b.g) return a.g < b.g;
    return a.j < b.j;
  });
  std::vector<double> cl(R, 0.0), cw(R, 0.0);
  Plan p;
  p.ranks.assign(G, {});
  for (const Item& it : items) {
    int best = -1;
    double bc = 0;
    for (int r = 0; r < R; r++) {
      const auto& h = p.ranks[it.g];
      if (std::find(h.begin(), h.end(), r) != h.end()) continue;
      const double c = std::max(cl[r], lat[it.g]) + cw[r] + w[it.g];
      if (best < 0 || c < bc - 1e-9) {
        best = r;
        bc = c;
      }
    }
    if (best < 0) fail(SYZGPU_EINTERNAL, "plan: more parts than sub-jobs");
    p.ranks[it.g].push_back(best);
    cl[best] = std::max(cl[best], lat[it.g]);
    cw[best] += w[it.g];
  }
  p.cost.resize(R);
  for (int r = 0; r < R; r++) p.cost[r] = cl[r] + cw[r];
  return p;
}

// start with whole groups, then double the part count of the heaviest group on the bottleneck rank while
// the modelled step (max over ranks) improves; split_largest > 1 forces the largest group into that many
// parts instead (rehearsals and tests)
Plan plan_parts(const std::vector<int64_t>& E, const std::vector<double>& P, int R, uint32_t split_largest,
                int max_rounds) {
  const size_t G = E.size();
  std::vector<int64_t> k(G, 1);
  if (split_largest > 1 && G) {
    const size_t g = (size_t)(std::max_element(E.begin(), E.end()) - E.begin());
    k[g] = std::min<int64_t>(split_largest, R);
    return assign(E, P, k, R);
  }
  Plan cur = assign(E, P, k, R);
  for (int round = 0; round < max_rounds; round++) {
    const int r = (int)(std::max_element(cur.cost.begin(), cur.cost.end()) - cur.cost.begin());
    int64_t pick = -1;
    double pv = 0;
    for (size_t g = 0; g < G; g++) {
      const auto& h = cur.ranks[g];
      if (std::find(h.begin(), h.end(), r) == h.end() || k[g] >= R || E[g] <= SMALL_GROUP) continue;
      const double v = sort_latency_us(E[g]) + US_PER_PC * P[g] / (double)k[g];
      if (pick < 0 || v > pv) {  // (ties: the smaller group id, as max(key=(v, -g)))
        pick = (int64_t)g;
        pv = v;
      }
    }
    if (pick < 0) break;
    std::vector<int64_t> k2(k);
    k2[pick] = std::min<int64_t>(R, k[pick] * 2);
    Plan nxt = assign(E, P, k2, R);
    if (*std::max_element(nxt.cost.begin(), nxt.cost.end()) >=
        *std::max_element(cur.cost.begin(), cur.cost.end()) - 1e-6)
      break;
    k = k2;
    cur = nxt;
  }
  return cur;
}

// PC-value bounds of a split group's k parts: k + 1 values [0, ..., 2^32] at equal-count quantiles of a
// sample of the group's PCs (every 16th entry of the group in corpus order), a pure function of the
// group's covers
std::vector<uint64_t> split_bounds(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                                   uint32_t g, size_t k) {
  std::vector<uint64_t> sample;
  size_t seen = 0;
  for (size_t e = 0; e < n; e++) {
    if (group[e] != g) continue;
    if (seen++ % 16) continue;
    sample.insert(sample.end(), pcs + off[e], pcs + off[e + 1]);
  }
  std::vector<uint64_t> b{0};
  if (!sample.empty()) {
    std::sort(sample.begin(), sample.end());
    for (size_t j = 1; j < k; j++)
      b.push_back(std::max<uint64_t>(b.back() + 1, sample[std::min(sample.size() - 1, sample.size() * j / k)]));
  } else {
    for (size_t j = 1; j < k; j++) b.push_back((1ull << 32) * j / k);
  }
  b.push_back(1ull << 32);
  return b;
}
}  // namespace kp

}  // namespace syz

// Host-side planners of the raw Minimize pipeline (panels.hip), the Go sort (gosort.hip) and the
// multi-device job (multi.hip), in plain C++ with no HIP dependency: the library compiles them
// (plan_host.cpp), and tests/test_sanitizers.py builds the same file with g++ under ASan + UBSan and
// drives it over random layouts (tests/planner_san.cpp). Everything here is a pure function of a layout.
#pragma once
#include <array>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/syzgpu.h"

namespace syz {

[[noreturn]] void fail(int code, const std::string& msg);

// ---- window planning (panels_dev.hpp's kernels use the same constants) --------------------------------
constexpr uint32_t WMAX = 1024;  // windows per call group
#ifndef SYZ_DS
#define SYZ_DS 14
#endif
constexpr uint32_t DS = SYZ_DS;  // direct-mode window bits: a 2^DS-entry u32 min table
constexpr uint32_t SMAX = 26;    // 32 - 6 tag bits
#ifndef SYZ_HTARGET
#define SYZ_HTARGET 8192
#endif
constexpr uint32_t HTARGET = SYZ_HTARGET;        // PCs per window a sparse call's window size aims at
constexpr uint32_t DENSE = 8192u >> (15 - DS);    // PCs per window (per 32K addresses: 8192) above which a call is direct
constexpr uint32_t PK_RBITS = 13;                 // packed sparse windows: offset << 13 | rank in the group
constexpr uint32_t PSMAX = 32 - PK_RBITS;         // window bits a packed slot holds
#ifndef SYZ_PK_BITS
#define SYZ_PK_BITS 13
#endif
constexpr uint32_t PHS_BITS = SYZ_PK_BITS;  // 13: 32 KB packed tables
constexpr uint32_t PHS = 1u << PHS_BITS;
constexpr uint32_t PHTARGET = PHS;  // packed windows aim at as many PCs as the table's slots

enum { PMODE_DIRECT = 0, PMODE_HASH = 1, PMODE_PACKED = 2 };

struct PGroup {             // per call group: window bits, windows, table kind
  uint32_t S, W, mode, rb;  // rb: first region of the group (region form: rb + segment * W + window)
};
struct PItem {  // one (call group, window) min-rank table
  uint32_t g, w;
};

// ---- slabs (slab_dev.hpp) ----------------------------------------------------------------------------
#ifndef SYZ_SL_BLOCK
#define SYZ_SL_BLOCK 512
#endif
#ifndef SYZ_SL_TPW
#define SYZ_SL_TPW 32
#endif
constexpr int SL_BLOCK = SYZ_SL_BLOCK;
constexpr int SL_WAVES = SL_BLOCK / 64;
constexpr int SL_TPW = SYZ_SL_TPW;
constexpr uint32_t SL_TILES = (uint32_t)SL_TPW * SL_WAVES;  // tiles per slab (<= 64 PCs each)
constexpr uint32_t SL_MEMB = 512;                              // members per slab at most

constexpr uint32_t SG_NO_WTOT = 0xFFFFFFFFu;  // SGroup.wbase of a group without per-window totals
struct SGroup {    // per call group, slab form
  uint64_t dbase;  // first D entry
  uint32_t S, W;   // window bits, windows
  uint32_t stride; // D row length (>= the group's slabs)
  uint32_t memb;   // members per block: min(SL_MEMB, 2^(32 - S))
  uint32_t wbase;  // first per-window total (wtot, when P is asked for them), else SG_NO_WTOT
  uint32_t pad;    // bit 0: a big call group (the Go sort's global rounds; P's second launch)
  uint64_t xbase;  // element slots of the padding of the groups before (a slab's runs are padded to
                   // 4 elements: it takes its PCs + 3 W + 4 slots at most)
};

// slots of padding a slab of a call with W windows may take (k_sl_slabs' spacing)
constexpr uint64_t slab_pad(uint32_t W) { return 3ull * W + 4; }

// The host part of a slab layout: per-group SGroup, blocks of members, bounds of the device arrays.
struct SlabPlan {
  uint32_t G = 0, B = 0;
  uint32_t wmax = 1;  // the widest call's windows (P's LDS staging is sized for it)
  uint64_t slab_bound = 0, dtotal = 0, wtotal = 0, total_pcs = 0, xtotal = 0;
  std::vector<SGroup> hsg;
  std::vector<uint32_t> hgblock, hbgroup;
};

// window size per call group (span: the PC span of the job; gpcs: PCs each group holds)
void plan_windows(uint64_t span, const uint64_t* gpcs, const uint64_t* gstart, uint32_t G, std::vector<PGroup>& pg);
// hpcs: PCs each call group's members hold (their slices); S, W from hpg
void slab_plan(SlabPlan& J, const std::vector<uint64_t>& hstart, const uint64_t* hpcs, const std::vector<PGroup>& hpg,
               uint32_t G, bool want_wtot);

// M's work items: (call, window), by class (big groups: sorted by the Go sort's global rounds) and
// table kind, largest expected window first; a key part only its windows
struct ItemPlan {
  std::vector<PItem> items;
  size_t icount[2][3] = {{0, 0, 0}, {0, 0, 0}};
  std::array<std::array<size_t, 3>, 2> ifirst{};
  uint64_t item_pcs[2][3] = {{0, 0, 0}, {0, 0, 0}};
  uint64_t cpcs[2] = {0, 0}, cent[2] = {0, 0};  // PCs / entries of the small and big call groups
};
void plan_items(const std::vector<uint64_t>& hstart, const std::vector<uint64_t>& hpcs, const uint64_t* hsl,
                const std::vector<PGroup>& hpg, uint32_t G, const uint32_t* key_lo, const uint32_t* key_hi,
                uint32_t lo, uint32_t hi, ItemPlan& out);

// ---- the Go sort's plan (gosort.hip) -------------------------------------------------------------------
constexpr uint32_t GS_T_SEG = 8192;                // call groups above this many entries start the global rounds
constexpr uint64_t GS_U32_LEN_LIMIT = 1ull << 19;  // cover lengths the packed u32 sort element holds
#ifndef SYZ_GS_PACK_DIV
#define SYZ_GS_PACK_DIV 1024
#endif
constexpr uint64_t GS_PACK_DIV = SYZ_GS_PACK_DIV;  // pack size cap: n / GS_PACK_DIV elements

struct Seg {
  uint32_t lo, hi;
  int32_t depth;  // remaining sort.Sort maxDepth budget at this recursion node
  uint32_t pad;
};
struct Pack {
  uint32_t plo, phi;    // element range in el[] (whole segments)
  uint32_t sbeg, send;  // its segments in the segment array
};
// sort.Sort's maxDepth for n elements (Go sort.go: 2 * ceil(lg(n + 1))); constexpr: device code uses it too
constexpr int32_t go_max_depth(uint64_t n) {
  int32_t depth = 0;
  for (uint64_t i = n; i > 0; i >>= 1) depth++;
  return depth * 2;
}
// the groups above GS_T_SEG (big: the global rounds) and the packs of the others (LDS sorter), the packs
// and big groups tiling [0, n)
void gosort_segments(const std::vector<uint64_t>& hstart, uint32_t ngroups, std::vector<Seg>& small,
                     std::vector<Pack>& packs, std::vector<Seg>& big);

// ---- the multi-device job's key-space plan (multi.hip; syzkaller_amd/sharding.py restated) --------------
namespace kp {
struct Plan {
  std::vector<std::vector<int>> ranks;  // ranks[g]: holders of group g's parts, the primary first
  std::vector<double> cost;             // modelled step per rank (µs)
};
Plan plan_parts(const std::vector<int64_t>& E, const std::vector<double>& P, int R, uint32_t split_largest = 0,
                int max_rounds = 24);
std::vector<uint64_t> split_bounds(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                                   uint32_t g, size_t k);
}  // namespace kp

}  // namespace syz

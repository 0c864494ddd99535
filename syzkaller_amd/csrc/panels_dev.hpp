// Device code shared by the raw-cover pipelines: minimizeCorpus (panels.hip) and the new-coverage
// check on windows (novelty_win.hip): window planning constants, the walk's scan and the min-table
// helpers. The transpose (P) and the window walk (M) are slab_dev.hpp.
#pragma once
#include "panels.hpp"

namespace syz {

#ifndef SYZ_PBM_WORDS
#define SYZ_PBM_WORDS 6144
#endif
#ifndef SYZ_DIRECT_RB
#define SYZ_DIRECT_RB 16
#endif
#ifndef SYZ_DIRECT_WPE
#define SYZ_DIRECT_WPE 1
#endif
constexpr uint32_t PBM_WORDS = SYZ_PBM_WORDS;  // LDS winner bitmap of the direct kernel
// (WMAX, DS, SMAX, DENSE, HTARGET, PK_RBITS, PSMAX, PHS, PHTARGET: plan_host.hpp)
constexpr int PP_BLOCK = 1024;
constexpr int PP_WAVES = PP_BLOCK / 64;
constexpr int PP_U = 4;     // 64-PC tiles per wave in flight in k_part's passes
#ifndef SYZ_HS_BITS
#define SYZ_HS_BITS 13
#endif
constexpr uint32_t HS_BITS = SYZ_HS_BITS;
constexpr uint32_t HS = 1u << HS_BITS;  // open-addressing slots of a sparse-window table (8 B each)
#ifndef SYZ_HCAP
#define SYZ_HCAP 16384
#endif
constexpr uint32_t HCAP = SYZ_HCAP;  // PCs per round of a sparse window: twice the slots, i.e. the table
                                     // fills only if no PC repeats (then the probe limit redoes the
                                     // window in more rounds); a tighter cap reads most windows twice
constexpr uint32_t HPROBE = 128; // a longer probe run means the table is full after all
constexpr uint32_t HBM_WORDS = 2048;  // LDS winner bitmap of the sparse kernel (65536 ranks per pass)
// packed sparse windows (call groups of < 8192 entries): one u32 per slot, offset << 13 | rank in the
// group (PK_RBITS, PHS_BITS: plan_host.hpp)
#ifndef SYZ_PK_BLOCK
#define SYZ_PK_BLOCK 512
#endif
constexpr int PK_BLOCK = SYZ_PK_BLOCK;     // 32 KB packed tables in 512-thread workgroups, four per CU
constexpr uint32_t PHCAP = 2 * PHS;       // PCs per round of a packed window



// elements the element buffer needs for `pcs` PCs in at most `chunks` chunks (k_chunks' alignment)
inline uint64_t elem_bound(uint64_t pcs, uint64_t chunks) { return pcs + 4 * chunks + 8; }

// The second source of the new-coverage check (novelty_win.hip): members with an entry id >= n1 are
// maxCover tables (mc/mc_off, table e - n1), the others covers; every list must be strictly increasing
// (err 1 for a table, 4 for a cover), which P checks as it reads: lane neighbours in a tile, tile
// neighbours through LDS, and a member's first PC in a chunk against its previous one.
struct NovSrc {
  const uint32_t* mc = nullptr;
  const uint64_t* mc_off = nullptr;
  uint32_t n1 = 0xFFFFFFFFu;
};

// ---- M walk, packed form ------------------------------------------------------------------------------
// A walk with one wave instruction per run leaves lanes idle on short runs and pays per-run bookkeeping
// (profiles/r03_pmin_base: ~0.9 VALU wave instructions per element). Here the workgroup takes up to PK_RUNS runs of the window at once (one per
// thread: desc pair, chunk start, member block), numbers their elements with one workgroup scan, and
// the waves then stream the concatenation in 64-element blocks — every lane of every load holds an
// element whichever run it belongs to, and every wave has blocks whether the window has thousands of
// short runs (dense calls) or a handful of long ones (sparse calls). A block's runs come from two LDS
// maps built per batch: the run holding the block's first element, and a bitmask of the runs that
// start inside the block, so a lane's run is that run plus a mbcnt of the mask. The ranks of a block's
// elements are one gather from rank_of_member (the member blocks of a block's runs: a few hundred bytes,
// L2-resident); PK_U blocks are in flight per wave. f(offset, rank) is called for every lane, with
// rank RANK_NONE for lanes past the window (a min table ignores it). IDENT: the rank is the member's
// position (novelty).
constexpr uint32_t PK_RUNS = 1024;      // runs per batch (one per thread of a 1024-thread workgroup)
constexpr uint32_t PK_NBLK = 256;       // 64-element blocks per element window of a batch
constexpr uint32_t PK_EW = 64 * PK_NBLK;
// LDS words the walk needs (callers may alias them with their emit bitmap)
constexpr uint32_t PK_SCRATCH_WORDS = 2 * PK_RUNS + 3 * PK_NBLK;
#ifndef SYZ_PK_U
#define SYZ_PK_U 4
#endif

// Workgroup exclusive scan of a run length and of "non-empty" at once: pre = elements of the runs
// before this one, k = non-empty runs before it, T = all elements. Wave totals are summed in a rolled
// loop (the unrolled block_excl_scan holds every wave total in registers). lds: 2 * waves words.
__device__ __forceinline__ void pk_scan(uint32_t len, uint32_t* lds, uint32_t& pre, uint32_t& k, uint32_t& T) {
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t inc = wave_incl_scan<uint32_t>(len);
  const uint64_t bal = __ballot(len != 0);
  const uint32_t kin = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
  if (__lane_id() == 63) {
    lds[2 * w] = inc;
    lds[2 * w + 1] = (uint32_t)__popcll(bal);
  }
  __syncthreads();
  uint32_t p = 0, q = 0, tp = 0;
#pragma unroll 1
  for (int i = 0; i < nw; i++) {
    const uint32_t a = lds[2 * i], b = lds[2 * i + 1];
    if (i < w) {
      p += a;
      q += b;
    }
    tp += a;
  }
  __syncthreads();
  pre = inc - len + p;
  k = kin + q;
  T = tp;
}

}  // namespace syz

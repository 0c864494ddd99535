// Device-resident sets of program signatures (hash.Sig = sha1.Sum, hash/hash.go:13-15): the hub's
// corpus map[hash.Sig]*Input with each input's seq (syz-hub/state/state.go:23-26, 211-228), a manager's
// map[hash.Sig]bool (state.go:30-40, 211-218) and the manager's PersistentSet (syz-manager/
// persistent.go:91-102, pruned by minimizeCorpus, manager.go:541-553).
//
// Open addressing with linear probing over 2^k slots, kept at most half full. A slot is claimed with one
// 64-bit CAS of (batch round << 32 | batch item + 1); the claimer then writes the full 20-byte key.
// A prober compares against the key of an earlier batch's slot (published by the kernel boundary) or,
// for a slot claimed in the current batch, against the claiming item's own input signature, which
// is always visible - so one launch resolves a whole batch with no waits on another lane's store and
// exact 160-bit comparisons. In a batch, the FIRST item (batch order, atomicMin) of a new signature
// is the one reported as added: the Go loop (state.go:211-228) inserts on the first occurrence and
// finds the entry for the later ones. Erase keeps the slot (a tombstone keeps probe chains intact);
// inserting the signature again revives it.
#include <algorithm>
#include <cstring>
#include <memory>

#include "pipeline.hpp"

namespace syz {

constexpr int SG_BLOCK = 256;
constexpr uint32_t SG_PENDING = 0, SG_NEW = 1, SG_FOUND = 2;

struct SigSet {
  std::recursive_mutex mu;  // one call on a set at a time
  uint64_t cap = 0, mask = 0, live = 0, used = 0;  // used: slots ever claimed (live + tombstones)
  uint32_t round = 1;                               // the next insert batch
  uint64_t* tag = nullptr;   // 0 = empty, else (round << 32 | item + 1) of the claim
  uint32_t* key = nullptr;   // 5 words per slot
  uint32_t* claim = nullptr; // batch round of the claim or of the last revival
  uint32_t* owner = nullptr; // first batch item of a signature new in its batch (~0 when free/erased)
  uint64_t* seq = nullptr;
  uint32_t* dead = nullptr;
  void alloc(uint64_t c) {
    cap = c;
    mask = c - 1;
    SYZ_HIP(hipMalloc(&tag, c * 8));
    SYZ_HIP(hipMalloc(&key, c * 20));
    SYZ_HIP(hipMalloc(&claim, c * 4));
    SYZ_HIP(hipMalloc(&owner, c * 4));
    SYZ_HIP(hipMalloc(&seq, c * 8));
    SYZ_HIP(hipMalloc(&dead, c * 4));
    hipStream_t s = ctx().stream;  // stream-ordered: another thread's graph capture may be running
    SYZ_HIP(hipMemsetAsync(tag, 0, c * 8, s));
    SYZ_HIP(hipMemsetAsync(claim, 0, c * 4, s));
    SYZ_HIP(hipMemsetAsync(owner, 0xFF, c * 4, s));
    SYZ_HIP(hipMemsetAsync(dead, 0, c * 4, s));
    SYZ_HIP(hipStreamSynchronize(s));
  }
  void free_all() {
    for (void* p : {(void*)tag, (void*)key, (void*)claim, (void*)owner, (void*)seq, (void*)dead})
      if (p) (void)hipFree(p);
    tag = nullptr, key = nullptr, claim = nullptr, owner = nullptr, seq = nullptr, dead = nullptr;
  }
  ~SigSet() { free_all(); }
};

struct SigView {  // kernel arguments
  uint64_t mask;
  uint64_t* tag;
  uint32_t* key;
  uint32_t* claim;
  uint32_t* owner;
  uint64_t* seq;
  uint32_t* dead;
};

__device__ __forceinline__ void sig_load(const uint32_t* sigs, uint64_t i, uint32_t (&w)[5]) {
#pragma unroll
  for (int q = 0; q < 5; q++) w[q] = sigs[5 * i + q];
}
__device__ __forceinline__ uint64_t sig_home(const uint32_t (&w)[5], uint64_t mask) {
  return (((uint64_t)w[3] << 32) | w[2]) & mask;
}
__device__ __forceinline__ bool sig_eq(const uint32_t* k, const uint32_t (&w)[5]) {
  return k[0] == w[0] && k[1] == w[1] && k[2] == w[2] && k[3] == w[3] && k[4] == w[4];
}

// A batch of inserts in one launch. state[i]: SG_NEW (claimed a slot) / SG_FOUND (the signature has a
// slot) / SG_PENDING (masked out); slot_of[i]: the slot.
__global__ __launch_bounds__(SG_BLOCK) void k_sig_insert(SigView T, const uint32_t* __restrict__ sigs,
                                                         const uint8_t* __restrict__ mask, uint64_t n,
                                                         uint32_t round, uint64_t seqv,
                                                         const uint64_t* __restrict__ seqs, uint8_t* state,
                                                         uint64_t* slot_of) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    state[i] = SG_PENDING;
    if (mask && !mask[i]) continue;
    uint32_t w[5];
    sig_load(sigs, i, w);
    const uint64_t mine = ((uint64_t)round << 32) | (uint64_t)(i + 1);
    uint64_t s = sig_home(w, T.mask);
    for (uint64_t probes = 0; probes <= T.mask; probes++, s = (s + 1) & T.mask) {
      uint64_t cur = __hip_atomic_load(&T.tag[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == 0) {
        cur = atomicCAS((unsigned long long*)&T.tag[s], 0ull, (unsigned long long)mine);
        if (cur == 0) {  // claimed: the key becomes visible to later batches at the kernel boundary
#pragma unroll
          for (int q = 0; q < 5; q++) T.key[5 * s + q] = w[q];
          T.claim[s] = round;
          T.seq[s] = seqs ? seqs[i] : seqv;
          T.dead[s] = 0;
          atomicMin(&T.owner[s], (uint32_t)i);
          state[i] = SG_NEW;
          slot_of[i] = s;
          break;
        }
      }
      const bool this_batch = (uint32_t)(cur >> 32) == round;
      const uint32_t* k = this_batch ? sigs + 5 * ((cur & 0xFFFFFFFFull) - 1) : T.key + 5 * s;
      if (!sig_eq(k, w)) continue;
      if (this_batch || T.dead[s]) atomicMin(&T.owner[s], (uint32_t)i);
      state[i] = SG_FOUND;
      slot_of[i] = s;
      break;
    }
  }
}

// Revivals of erased signatures (their first batch item), then the added flags: the first batch item of
// each signature claimed or revived in this batch.
__global__ void k_sig_revive(SigView T, const uint64_t* slot_of, const uint8_t* state, const uint8_t* mask, uint64_t n,
                             uint32_t round, uint64_t seqv, const uint64_t* seqs) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if ((mask && !mask[i]) || state[i] != SG_FOUND) continue;
    const uint64_t s = slot_of[i];
    if (T.dead[s] && T.owner[s] == (uint32_t)i) {
      T.dead[s] = 0;
      T.claim[s] = round;
      T.seq[s] = seqs ? seqs[i] : seqv;
    }
  }
}

// Counts go through a block reduction and one atomic per block: same-address atomics serialize in
// the L2 (per-wave atomics cost 0.39 ms for a 1M-item batch).
__global__ __launch_bounds__(SG_BLOCK) void k_sig_added(SigView T, const uint64_t* slot_of, const uint8_t* state,
                                                        const uint8_t* mask, uint64_t n, uint32_t round,
                                                        uint8_t* added, unsigned long long* nnew) {
  __shared__ uint32_t red[SG_BLOCK / 64 + 1];
  uint32_t ca = 0, cn = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t a = 0;
    const uint8_t st = state[i];
    if (!(mask && !mask[i]) && st != SG_PENDING) {
      const uint64_t s = slot_of[i];
      a = T.claim[s] == round && T.owner[s] == (uint32_t)i;
    }
    if (added) added[i] = a;
    ca += a;
    cn += st == SG_NEW;  // slots claimed (not revived)
  }
  ca = block_sum<SG_BLOCK>(ca, red);
  cn = block_sum<SG_BLOCK>(cn, red);
  if (threadIdx.x == 0) {
    if (ca) atomicAdd(&nnew[0], (unsigned long long)ca);
    if (cn) atomicAdd(&nnew[1], (unsigned long long)cn);
  }
}

// lookups (mode 0), erases (mode 1)
__global__ __launch_bounds__(SG_BLOCK) void k_sig_find(SigView T, const uint32_t* __restrict__ sigs, uint64_t n,
                                                       int mode, uint8_t* found, uint64_t* seq_out,
                                                       unsigned long long* nerased) {
  uint32_t ce = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t w[5];
    sig_load(sigs, i, w);
    uint64_t s = sig_home(w, T.mask);
    uint8_t f = 0;
    uint64_t q = 0;
    for (uint64_t probes = 0; probes <= T.mask; probes++, s = (s + 1) & T.mask) {
      if (T.tag[s] == 0) break;
      if (!sig_eq(T.key + 5 * s, w)) continue;
      if (mode == 0) {
        f = !T.dead[s];
        if (f) q = T.seq[s];
      } else if (!T.dead[s]) {
        f = atomicExch(&T.dead[s], 1u) == 0;  // duplicates in one erase batch: one of them erases
        if (f) T.owner[s] = 0xFFFFFFFFu;      // a later batch that revives it takes its first item as owner
      }
      break;
    }
    if (found) found[i] = f;
    if (seq_out) seq_out[i] = q;
    ce += mode == 1 && f;
  }
  if (mode == 1) {  // one atomic per block
    __shared__ uint32_t red[SG_BLOCK / 64 + 1];
    ce = block_sum<SG_BLOCK>(ce, red);
    if (threadIdx.x == 0 && ce) atomicAdd(nerased, (unsigned long long)ce);
  }
}

// live entries in slot order (state.go iterates its map: any order is the reference's)
__global__ void k_sig_live_flag(SigView T, uint64_t cap, uint8_t* flag) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x)
    flag[s] = T.tag[s] != 0 && !T.dead[s];
}
__global__ void k_sig_live_emit(SigView T, uint64_t cap, const uint8_t* flag, const uint64_t* pos, uint32_t* out,
                                uint64_t* seq_out) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x)
    if (flag[s]) {
      const uint64_t p = pos[s];
#pragma unroll
      for (int q = 0; q < 5; q++) out[5 * p + q] = T.key[5 * s + q];
      if (seq_out) seq_out[p] = T.seq[s];
    }
}

static SigView view(SigSet& S) { return SigView{S.mask, S.tag, S.key, S.claim, S.owner, S.seq, S.dead}; }

static uint64_t pow2_at_least(uint64_t x) {
  uint64_t c = 1024;
  while (c < x) c <<= 1;
  return c;
}

static void sig_check_ptr(const void* p) {
  if ((uintptr_t)p & 3) fail(SYZGPU_EINVAL, "signatures must be 4-byte aligned");
}

// live entries -> out (5 words each) and seq_out; returns their number (<= cap written)
static uint64_t sigset_export(SigSet& S, uint32_t* out, uint64_t* seq_out, uint64_t cap, hipStream_t s) {
  Scratch& sc = ctx().scratch;
  uint8_t* flag = sc.get<uint8_t>("sg_flag", S.cap + 1);
  uint64_t* pos = sc.get<uint64_t>("sg_pos", S.cap + 1);
  k_sig_live_flag<<<grid_for(S.cap, 256, 8192), 256, 0, s>>>(view(S), S.cap, flag);
  SYZ_LAUNCHED();
  exclusive_scan_u8(flag, pos, S.cap, s);
  uint64_t m = 0;
  SYZ_HIP(hipMemcpyAsync(&m, pos + S.cap, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  if (m <= cap && m) {
    k_sig_live_emit<<<grid_for(S.cap, 256, 8192), 256, 0, s>>>(view(S), S.cap, flag, pos, out, seq_out);
    SYZ_LAUNCHED();
  }
  return m;
}

static uint64_t sigset_insert(SigSet& S, const uint32_t* sigs, const uint8_t* mask, uint64_t n, uint64_t seqv,
                              const uint64_t* seqs, uint8_t* added, hipStream_t s);

// a table kept at most half full (tombstones count: they are only reclaimed here)
static void sigset_reserve(SigSet& S, uint64_t more, hipStream_t s) {
  if ((S.used + more) * 2 <= S.cap) return;
  const uint64_t nc = pow2_at_least(4 * (S.live + more));
  Scratch& sc = ctx().scratch;
  uint32_t* keys = sc.get<uint32_t>("sg_grow_k", 5 * S.live + 5);
  uint64_t* seqs = sc.get<uint64_t>("sg_grow_s", S.live + 1);
  const uint64_t m = sigset_export(S, keys, seqs, S.live, s);
  SYZ_HIP(hipStreamSynchronize(s));
  S.free_all();
  const uint32_t round = S.round;
  S.alloc(nc);
  S.round = round;
  S.live = S.used = 0;
  if (m) sigset_insert(S, keys, nullptr, m, 0, seqs, nullptr, s);
}

static uint64_t sigset_insert(SigSet& S, const uint32_t* sigs, const uint8_t* mask, uint64_t n, uint64_t seqv,
                              const uint64_t* seqs, uint8_t* added, hipStream_t s) {
  if (!n) return 0;
  sigset_reserve(S, n, s);
  Scratch& sc = ctx().scratch;
  uint8_t* state = sc.get<uint8_t>("sg_state", n + 1);
  uint64_t* slot_of = sc.get<uint64_t>("sg_slot", n + 1);
  unsigned long long* nnew = sc.get<unsigned long long>("sg_nnew", 2);
  const uint32_t round = S.round++;
  const unsigned grid = grid_for(n, SG_BLOCK, 8192);
  ProfScope ps("sig_insert", s, n * 20 + n * 28);  // the batch's signatures + one slot touched per item
  k_sig_insert<<<grid, SG_BLOCK, 0, s>>>(view(S), sigs, mask, n, round, seqv, seqs, state, slot_of);
  SYZ_LAUNCHED();
  k_sig_revive<<<grid, 256, 0, s>>>(view(S), slot_of, state, mask, n, round, seqv, seqs);
  SYZ_LAUNCHED();
  SYZ_HIP(hipMemsetAsync(nnew, 0, 16, s));
  k_sig_added<<<grid_for(n, SG_BLOCK, 256), SG_BLOCK, 0, s>>>(view(S), slot_of, state, mask, n, round, added, nnew);
  SYZ_LAUNCHED();
  uint64_t h[2] = {0, 0};
  SYZ_HIP(hipMemcpyAsync(h, nnew, 16, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  S.live += h[0];
  S.used += h[1];
  return h[0];
}

static uint64_t sigset_find(SigSet& S, const uint32_t* sigs, uint64_t n, int mode, uint8_t* found, uint64_t* seq_out,
                            hipStream_t s) {
  if (!n) return 0;
  unsigned long long* ne = ctx().scratch.get<unsigned long long>("sg_nerase", 2);
  SYZ_HIP(hipMemsetAsync(ne, 0, 8, s));
  if (S.cap) {
    k_sig_find<<<grid_for(n, SG_BLOCK, mode == 1 ? 512 : 8192), SG_BLOCK, 0, s>>>(view(S), sigs, n, mode, found,
                                                                                    seq_out, ne);
    SYZ_LAUNCHED();
  } else if (found) {
    SYZ_HIP(hipMemsetAsync(found, 0, n, s));
  }
  if (mode != 1) return 0;
  uint64_t h = 0;
  SYZ_HIP(hipMemcpyAsync(&h, ne, 8, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  S.live -= h;
  return h;
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzgpu_sigset_create(size_t capacity_hint, syzgpu_sigset** out) {
  SYZ_API_BODY({
    if (!out) fail(SYZGPU_EINVAL, "null pointer");
    std::unique_ptr<SigSet> S(new SigSet());
    S->alloc(pow2_at_least(2 * (uint64_t)capacity_hint));
    *out = reinterpret_cast<syzgpu_sigset*>(S.release());
  })
}

int syzgpu_sigset_destroy(syzgpu_sigset* set) {
  SYZ_API_BODY({ delete reinterpret_cast<SigSet*>(set); })
}

int syzgpu_sigset_clear(syzgpu_sigset* set, void* stream) {
  SYZ_API_BODY({
    if (!set) fail(SYZGPU_EINVAL, "null set");
    std::lock_guard<std::recursive_mutex> hl_(reinterpret_cast<SigSet*>(const_cast<syzgpu_sigset*>(set))->mu);
    if (!set) fail(SYZGPU_EINVAL, "null set");
    SigSet& S = *reinterpret_cast<SigSet*>(set);
    hipStream_t s = (hipStream_t)stream;
    SYZ_HIP(hipMemsetAsync(S.tag, 0, S.cap * 8, s));
    SYZ_HIP(hipMemsetAsync(S.claim, 0, S.cap * 4, s));
    SYZ_HIP(hipMemsetAsync(S.owner, 0xFF, S.cap * 4, s));
    SYZ_HIP(hipMemsetAsync(S.dead, 0, S.cap * 4, s));
    S.live = S.used = 0;
  })
}

int syzgpu_sigset_size(const syzgpu_sigset* set, uint64_t* n) {
  SYZ_API_BODY({
    if (!set) fail(SYZGPU_EINVAL, "null set");
    std::lock_guard<std::recursive_mutex> hl_(reinterpret_cast<SigSet*>(const_cast<syzgpu_sigset*>(set))->mu);
    if (!set || !n) fail(SYZGPU_EINVAL, "null pointer");
    *n = reinterpret_cast<const SigSet*>(set)->live;
  })
}

int syzgpu_sigset_insert_dev(syzgpu_sigset* set, const uint8_t* sigs, const uint8_t* mask, size_t n, uint64_t seq,
                             uint8_t* added, uint64_t* nadded, void* stream) {
  SYZ_API_BODY({
    if (!set) fail(SYZGPU_EINVAL, "null set");
    std::lock_guard<std::recursive_mutex> hl_(reinterpret_cast<SigSet*>(const_cast<syzgpu_sigset*>(set))->mu);
    if (!set || (n && !sigs)) fail(SYZGPU_EINVAL, "null pointer");
    sig_check_ptr(sigs);
    const uint64_t a = sigset_insert(*reinterpret_cast<SigSet*>(set), reinterpret_cast<const uint32_t*>(sigs), mask,
                                     n, seq, nullptr, added, (hipStream_t)stream);
    if (nadded) *nadded = a;
  })
}

int syzgpu_sigset_lookup_dev(syzgpu_sigset* set, const uint8_t* sigs, size_t n, uint8_t* found, uint64_t* seq,
                             void* stream) {
  SYZ_API_BODY({
    if (!set) fail(SYZGPU_EINVAL, "null set");
    std::lock_guard<std::recursive_mutex> hl_(reinterpret_cast<SigSet*>(const_cast<syzgpu_sigset*>(set))->mu);
    if (!set || (n && !sigs)) fail(SYZGPU_EINVAL, "null pointer");
    sig_check_ptr(sigs);
    sigset_find(*reinterpret_cast<SigSet*>(set), reinterpret_cast<const uint32_t*>(sigs), n, 0, found, seq,
                (hipStream_t)stream);
  })
}

int syzgpu_sigset_erase_dev(syzgpu_sigset* set, const uint8_t* sigs, size_t n, uint8_t* erased, uint64_t* nerased,
                            void* stream) {
  SYZ_API_BODY({
    if (!set) fail(SYZGPU_EINVAL, "null set");
    std::lock_guard<std::recursive_mutex> hl_(reinterpret_cast<SigSet*>(const_cast<syzgpu_sigset*>(set))->mu);
    if (!set || (n && !sigs)) fail(SYZGPU_EINVAL, "null pointer");
    sig_check_ptr(sigs);
    const uint64_t e = sigset_find(*reinterpret_cast<SigSet*>(set), reinterpret_cast<const uint32_t*>(sigs), n, 1,
                                   erased, nullptr, (hipStream_t)stream);
    if (nerased) *nerased = e;
  })
}

// host-pointer forms: copy in, run on the library stream, copy out
int syzgpu_sigset_insert(syzgpu_sigset* set, const uint8_t* sigs, const uint8_t* mask, size_t n, uint64_t seq,
                         uint8_t* added, uint64_t* nadded) {
  SYZ_API_BODY({
    if (!set) fail(SYZGPU_EINVAL, "null set");
    std::lock_guard<std::recursive_mutex> hl_(reinterpret_cast<SigSet*>(const_cast<syzgpu_sigset*>(set))->mu);
    if (!set || (n && !sigs)) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    uint32_t* d = C_.scratch.get<uint32_t>("sgh_sigs", 5 * n + 5);
    uint8_t* dm = mask ? C_.scratch.get<uint8_t>("sgh_mask", n + 1) : nullptr;
    uint8_t* da = C_.scratch.get<uint8_t>("sgh_out", n + 1);
    if (n) SYZ_HIP(hipMemcpyAsync(d, sigs, 20 * n, hipMemcpyHostToDevice, s));
    if (dm && n) SYZ_HIP(hipMemcpyAsync(dm, mask, n, hipMemcpyHostToDevice, s));
    const uint64_t a = sigset_insert(*reinterpret_cast<SigSet*>(set), d, dm, n, seq, nullptr, da, s);
    if (added && n) SYZ_HIP(hipMemcpyAsync(added, da, n, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (nadded) *nadded = a;
  })
}

int syzgpu_sigset_lookup(syzgpu_sigset* set, const uint8_t* sigs, size_t n, uint8_t* found, uint64_t* seq) {
  SYZ_API_BODY({
    if (!set) fail(SYZGPU_EINVAL, "null set");
    std::lock_guard<std::recursive_mutex> hl_(reinterpret_cast<SigSet*>(const_cast<syzgpu_sigset*>(set))->mu);
    if (!set || (n && !sigs)) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    uint32_t* d = C_.scratch.get<uint32_t>("sgh_sigs", 5 * n + 5);
    uint8_t* df = C_.scratch.get<uint8_t>("sgh_out", n + 1);
    uint64_t* dq = seq ? C_.scratch.get<uint64_t>("sgh_seq", n + 1) : nullptr;
    if (n) SYZ_HIP(hipMemcpyAsync(d, sigs, 20 * n, hipMemcpyHostToDevice, s));
    sigset_find(*reinterpret_cast<SigSet*>(set), d, n, 0, df, dq, s);
    if (found && n) SYZ_HIP(hipMemcpyAsync(found, df, n, hipMemcpyDeviceToHost, s));
    if (seq && n) SYZ_HIP(hipMemcpyAsync(seq, dq, n * 8, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

int syzgpu_sigset_erase(syzgpu_sigset* set, const uint8_t* sigs, size_t n, uint8_t* erased, uint64_t* nerased) {
  SYZ_API_BODY({
    if (!set) fail(SYZGPU_EINVAL, "null set");
    std::lock_guard<std::recursive_mutex> hl_(reinterpret_cast<SigSet*>(const_cast<syzgpu_sigset*>(set))->mu);
    if (!set || (n && !sigs)) fail(SYZGPU_EINVAL, "null pointer");
    hipStream_t s = C_.stream;
    uint32_t* d = C_.scratch.get<uint32_t>("sgh_sigs", 5 * n + 5);
    uint8_t* df = C_.scratch.get<uint8_t>("sgh_out", n + 1);
    if (n) SYZ_HIP(hipMemcpyAsync(d, sigs, 20 * n, hipMemcpyHostToDevice, s));
    const uint64_t e = sigset_find(*reinterpret_cast<SigSet*>(set), d, n, 1, df, nullptr, s);
    if (erased && n) SYZ_HIP(hipMemcpyAsync(erased, df, n, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
    if (nerased) *nerased = e;
  })
}

int syzgpu_sigset_export(syzgpu_sigset* set, uint8_t* sigs, uint64_t* seq, size_t cap, size_t* out_n) {
  SYZ_API_BODY({
    if (!set) fail(SYZGPU_EINVAL, "null set");
    std::lock_guard<std::recursive_mutex> hl_(reinterpret_cast<SigSet*>(const_cast<syzgpu_sigset*>(set))->mu);
    if (!set || !out_n) fail(SYZGPU_EINVAL, "null pointer");
    SigSet& S = *reinterpret_cast<SigSet*>(set);
    hipStream_t s = C_.stream;
    uint32_t* d = C_.scratch.get<uint32_t>("sgx_sigs", 5 * S.live + 5);
    uint64_t* dq = C_.scratch.get<uint64_t>("sgx_seq", S.live + 1);
    const uint64_t m = S.cap ? sigset_export(S, d, dq, S.live, s) : 0;
    *out_n = m;
    if (m > cap) fail(SYZGPU_ECAPACITY, "output capacity too small");
    if (m && sigs) SYZ_HIP(hipMemcpyAsync(sigs, d, 20 * m, hipMemcpyDeviceToHost, s));
    if (m && seq) SYZ_HIP(hipMemcpyAsync(seq, dq, 8 * m, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}

}  // extern "C"

// A device hash set / map of (call << 32 | PC) keys: open addressing, linear probing, a power-of-two
// table kept at most half full. A lookup is one or two 8-byte loads where a binary search over the
// sorted key array was ~25 dependent ones; inserts are 64-bit CAS claims, so a batch of new keys goes in
// with no sort and no host round trip. Used for corpusCover (corpus_cover.hip) and the corpus index's
// (call, PC) -> dense id dictionary (corpus_inc.hip).
#pragma once
#include "store.hpp"

namespace syz {

constexpr uint64_t KH_EMPTY = ~0ull;  // no key: call ids are < 4096, so a key never has its top bits set

__device__ __forceinline__ uint64_t kh_mix(uint64_t k) {  // a 64-bit finaliser (xor-shift-multiply)
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// the slot holding k, or KH_EMPTY
__device__ __forceinline__ uint64_t kh_find(const uint64_t* __restrict__ keys, uint64_t mask, uint64_t k) {
  for (uint64_t h = kh_mix(k) & mask;; h = (h + 1) & mask) {
    const uint64_t x = keys[h];
    if (x == k) return h;
    if (x == KH_EMPTY) return KH_EMPTY;
  }
}

// adds the wave's successful claims to the table's count (every lane of the wave calls it)
__device__ __forceinline__ void kh_count_claims(unsigned long long* count, bool claimed) {
  const uint64_t b = __ballot(claimed);
  if (b && __lane_id() == (unsigned)(__ffsll((unsigned long long)b) - 1))
    atomicAdd(count, (unsigned long long)__popcll(b));
}

// claims a slot for k; true iff this call inserted it (false: present already, or claimed concurrently)
__device__ __forceinline__ bool kh_insert(uint64_t* keys, uint64_t mask, uint64_t k, uint64_t* slot) {
  for (uint64_t h = kh_mix(k) & mask;; h = (h + 1) & mask) {
    uint64_t x = keys[h];
    if (x == KH_EMPTY) {
      x = atomicCAS(reinterpret_cast<unsigned long long*>(&keys[h]), (unsigned long long)KH_EMPTY,
                    (unsigned long long)k);
      if (x == KH_EMPTY) {
        *slot = h;
        return true;
      }
    }
    if (x == k) {
      *slot = h;
      return false;
    }
  }
}

struct KeyHash {
  DevArr<uint64_t> keys;
  DevArr<uint32_t> vals;  // a map's values (unused by a set)
  DevArr<unsigned long long> count;  // [0]: keys held (every insert kernel adds its claims)
  uint64_t cap = 0;       // slots, a power of two
  uint64_t bound = 0;     // an upper bound of count[0] on the host (made exact by kh_reserve's wait)
  bool with_vals = false;
  ~KeyHash() {
    keys.free();
    vals.free();
    count.free();
  }
  uint64_t mask() const { return cap - 1; }
};

// empty table for at least n keys
void kh_init(KeyHash& H, uint64_t n, bool with_vals, hipStream_t s);
// room for `more` further keys (a rehash into a larger table when the bound would pass half full)
void kh_reserve(KeyHash& H, uint64_t more, hipStream_t s);
// inserts keys[0..n) (distinct, none present; values vals[i], or none), on the stream
void kh_insert_sorted(KeyHash& H, const uint64_t* keys, const uint32_t* vals, uint64_t n, hipStream_t s);
// the held keys, sorted (device scratch "kh_out"); returns their number (one wait)
uint64_t kh_export_sorted(KeyHash& H, uint64_t** out, hipStream_t s);

}  // namespace syz

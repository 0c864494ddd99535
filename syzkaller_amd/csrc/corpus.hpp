// The resident corpus handle (syzgpu_corpus): syz-manager's mgr.corpus on the device.
#pragma once
#include <memory>
#include <mutex>
#include <vector>

#include "keyhash.hpp"
#include "panels.hpp"

namespace syz {

// mgr.corpus (manager.go:52-65) as device-resident CSR covers: the source of truth. NewInput appends
// to it in place (manager.go:609-616, O(new covers)); minimizeCorpus replaces it by its kept entries
// in Go's order (mgr.corpus = newCorpus, manager.go:523-529, one gather). Minimize runs on the
// dense-id index (Corpus, ≈0.7 ms at 1M programs), which appends and keeps update in place
// (corpus_inc.hip); without an index (never built, or dropped by a failed update or key-space parts)
// on the raw pipeline (panels.hip, no build). The index is built for what needs it: the cover
// analytics, key-space parts, or an explicit reindex.
// corpusCover (manager.go:65): a device hash set of (call << 32 | PC) keys (corpus_cover.hip)
struct CoverSet {
  KeyHash h;
  bool built = false;
};

struct CorpusHandle {
  std::recursive_mutex mu;  // one call on a corpus at a time (mgr.mu serialises them in the reference)
  size_t n = 0;
  uint32_t G = 0;
  uint64_t L = 0;  // PCs
  Grow<uint32_t> pcs, group;
  Grow<uint64_t> off;
  Grow<uint16_t> prog_len;
  Grow<uint32_t> pcs2, group2;  // the keep's gather targets (swapped in)
  Grow<uint64_t> off2;
  Grow<uint16_t> prog_len2;
  uint32_t max_prog_len = 0;
  std::unique_ptr<Corpus> index;  // null: stale (built on demand)
  MinJob job;                     // the raw path's selection between begin and end
  int path = 0;                   // of the minimize in flight: 1 index, 2 raw
  // key-space parts (syzgpu_corpus_set_parts), applied to every index built for this corpus
  bool parts_set = false, has_count_hist = false;
  std::vector<uint16_t> part, nparts;
  std::vector<uint8_t> count_hist;
  CoverSet cc;  // built on first use (cc_ensure)
};

// The index of H's current covers, built (with H's key parts) if stale.
Corpus& corpus_index(CorpusHandle& H, hipStream_t s);
// The same with its id -> PC dictionary complete (rebuilt if appends or keeps were applied to it
// incrementally): the cover analytics' form.
Corpus& corpus_index_full(CorpusHandle& H, hipStream_t s);
// corpus_inc.hip: the index brought up to H after an append (H's entries from n0 and PCs from L0 are
// new) or a keep (H = the old entries idx[0..m) of n0); they throw on failure (the caller drops it)
void corpus_index_append(Corpus& K, const CorpusHandle& H, size_t n0, uint64_t L0, hipStream_t s);
void corpus_index_note_append(Corpus& K, size_t n0, uint64_t L0);
void corpus_index_keep(Corpus& K, const CorpusHandle& H, const int64_t* idx, size_t m, size_t n0, hipStream_t s);
// a recorded keep applied (the index's users call it first: corpus_index does)
void corpus_index_sync(Corpus& K, const CorpusHandle& H, hipStream_t s);
// m covers (device CSR, offsets from 0) appended in place; cc_update: also union them into corpusCover
// (when built)
void append_covers(CorpusHandle& H, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                   const uint16_t* prog_len, size_t m, hipStream_t s, bool cc_update = true);
// room for m more entries and Lm more PCs, before anything changes (a gate that mutates corpusCover
// first reserves, so the append after it cannot fail on capacity or the entry limit)
void append_reserve(CorpusHandle& H, size_t m, uint64_t Lm, hipStream_t s);
// corpus_cover.hip: corpusCover built from H's covers if it is not yet; the union of appended covers;
// NewInput's gate over a batch (is_new: device bytes or null; returns the number appended)
void cc_ensure(CorpusHandle& H, hipStream_t s);
void cc_add(CorpusHandle& H, const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t m,
            uint64_t Lm, hipStream_t s);
uint64_t corpus_new_inputs(CorpusHandle& H, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                           const uint16_t* prog_len, size_t m, uint8_t* is_new, hipStream_t s);
// corpusCover as per-call CSR into device buffers (out capacity cap; returns the total)
uint64_t cc_export(CorpusHandle& H, uint32_t* out, uint64_t* out_off, uint64_t cap, hipStream_t s);

}  // namespace syz

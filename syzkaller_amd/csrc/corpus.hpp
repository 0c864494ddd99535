// The resident corpus handle (syzgpu_corpus): syz-manager's mgr.corpus on the device.
#pragma once
#include <memory>
#include <mutex>
#include <vector>

#include "panels.hpp"

namespace syz {

// mgr.corpus (manager.go:52-65) as device-resident CSR covers: the source of truth. NewInput appends
// to it in place (manager.go:609-616, O(new covers)); minimizeCorpus replaces it by its kept entries
// in Go's order (mgr.corpus = newCorpus, manager.go:523-529, one gather). Minimize runs on the
// dense-id index (Corpus, ≈0.7 ms at 1M programs) while that matches the covers, and on the raw
// pipeline (panels.hip, no build) once appends or a keep have made it stale; the index is rebuilt
// only for what needs it: the cover analytics, key-space parts, or an explicit reindex.
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
};

// The index of H's current covers, built (with H's key parts) if stale.
Corpus& corpus_index(CorpusHandle& H, hipStream_t s);

}  // namespace syz

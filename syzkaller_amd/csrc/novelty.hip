// syz-fuzzer/fuzzer.go:446-470 novelty batch (placeholder until the bucket pipeline grows the
// exclusion-set mode).
#include "pipeline.hpp"
using namespace syz;
extern "C" int syzgpu_novelty_batch(const uint32_t*, const uint64_t*, const uint32_t*, size_t, uint32_t,
                                    const uint32_t*, const uint64_t*, const uint32_t*, size_t, uint8_t*, uint32_t*,
                                    size_t, uint64_t*) {
  set_last_error("novelty_batch not implemented yet");
  return SYZGPU_EINTERNAL;
}

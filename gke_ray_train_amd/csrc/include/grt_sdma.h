// Device -> pinned-host copies on the SDMA engines, ordered with HIP streams (csrc/bindings/sdma_copy.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace grt {

struct SdmaStats {
  uint64_t copies = 0, bytes = 0, busy_ns = 0;  // busy_ns: worker time from copy issue to completion
  uint32_t engine = 0, engines_available = 0, engines_preferred = 0;  // hsa_amd_sdma_engine_id_t masks (0: runtime-assigned)
  std::string error;                          // first failure since the last clear ("" = none)
};

// Copy `bytes` from device memory `src` to pinned host memory `dst` after the work already on
// stream `s`; work enqueued on `s` afterwards runs after the copy has landed.
// The copies of one device run one at a time in submission order. Submit from ONE stream per device
// (the offloaded AdamW's download stream), or from streams that never wait on each other: a copy
// whose producer waits on another stream's later copy would wait forever behind it.
// `dst` must stay allocated until the stream has passed the copy: unlike a stream copy, the copy is
// not recorded with torch's caching host allocator.
// `producer` (optional): the stream whose work so far produced `src`; the copy waits for it directly
// (recorded there) rather than for an event recorded on `s` behind a cross-stream wait.
void sdma_d2h(void* dst, const void* src, size_t bytes, int device, hipStream_t s, hipStream_t producer = nullptr);
SdmaStats sdma_stats(int device);
void sdma_clear_error(int device);

}  // namespace grt

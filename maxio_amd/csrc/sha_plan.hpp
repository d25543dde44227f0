// sha_plan.hpp — host-side sizing of the SHA-256 stream form (no HIP
// dependency, so the guard is unit-tested on the CPU:
// tests/c_manifest/sha_guard_check.cpp).
#pragma once
#include <cstdint>

namespace mxec {

// Segments of the longest message: the stream form's items are (segment,
// 64-message group) pairs, seg_max per group.
inline uint64_t sha_stream_seg_max(uint64_t longest, uint32_t seg_blocks) {
    return longest / 64 / seg_blocks + 1;
}

// The stream kernel hands out items from a 32-bit counter that every wave
// bumps once more after the last item.  The form is only allowed while
// groups * seg_max plus that overshoot stays below 2^32: a wrapped counter
// would either skip the tail items (their digests and ok flags never
// written) or hand item 0 out again.
inline bool sha_stream_items_fit(uint64_t n_msgs, uint64_t seg_max, uint64_t waves) {
    const uint64_t groups = (n_msgs + 63) / 64;
    if (groups == 0 || seg_max == 0 || seg_max > UINT32_MAX || waves > UINT32_MAX) return false;
    if (groups > (uint64_t(UINT32_MAX) - waves) / seg_max) return false;
    return groups * seg_max + waves <= UINT32_MAX;
}

}  // namespace mxec

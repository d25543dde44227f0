// deal.hpp — which device of a context gets each object of a host batch
// (pipeline.cpp mxec_encode_batch_host).  No HIP dependency, so the dealing
// is unit-tested on the CPU (tests/c_manifest/deal_check.cpp).
#pragma once
#include <algorithm>
#include <cstdint>
#include <numeric>
#include <vector>

namespace mxec {

// bytes[o]: the device bytes object o occupies (its k + m shard slots).
// A uniform batch keeps object o -> device o mod D (the layout the
// bench and configs[3] assume).  A mixed batch is dealt longest-first onto
// the least-loaded device (LPT), so no device carries several times another's
// bytes (a 10 MiB-chunk object is ~160 of a 64 KiB one): every device then
// finishes close to the total / D.  Ties go to the lowest device index, so
// the dealing is deterministic.
inline std::vector<uint32_t> deal_objects(const std::vector<uint64_t>& bytes, uint32_t D) {
    const size_t n = bytes.size();
    std::vector<uint32_t> dev(n, 0);
    if (D <= 1 || n == 0) return dev;
    const bool uniform = std::all_of(bytes.begin(), bytes.end(), [&](uint64_t b) { return b == bytes[0]; });
    if (uniform) {
        for (size_t o = 0; o < n; ++o) dev[o] = uint32_t(o % D);
        return dev;
    }
    std::vector<size_t> order(n);
    std::iota(order.begin(), order.end(), size_t(0));
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return bytes[a] > bytes[b]; });
    std::vector<uint64_t> load(D, 0);
    for (size_t o : order) {
        uint32_t best = 0;
        for (uint32_t d = 1; d < D; ++d)
            if (load[d] < load[best]) best = d;
        dev[o] = best;
        load[best] += bytes[o];
    }
    return dev;
}

}  // namespace mxec

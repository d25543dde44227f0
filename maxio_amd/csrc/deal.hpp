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

// NUMA-aware dealing for a context whose devices sit on
// more than one NUMA node (a two-socket 8-GPU host): node[o] is the node of
// object o's host pages (-1: unknown), dev_node[d] the node of device d.
// Balance first, locality second: objects go longest first (stable) to the
// least-loaded device on their pages' node while that device stays within
// the batch's fair share (total / D, plus half the object, so a uniform
// batch splits evenly), otherwise -- and for objects of unknown node, or of
// a node with no device -- to the least-loaded device of all.  A batch whose
// pages are spread over the nodes as the devices are runs every DMA on its
// own socket; one whose pages all sit on one node still uses every device
// (the remote ones take exactly the excess over the local ones' fair share:
// an idle device costs more than a DMA over the socket link).  Without any
// node information the deal is deal_objects' (o mod D for a uniform batch).
inline std::vector<uint32_t> deal_objects_numa(const std::vector<uint64_t>& bytes, const std::vector<int>& node,
                                               const std::vector<int>& dev_node) {
    const uint32_t D = uint32_t(dev_node.size());
    const size_t n = bytes.size();
    bool any = false;
    for (size_t o = 0; o < n && !any; ++o)
        for (uint32_t d = 0; d < D && !any; ++d) any = node[o] >= 0 && node[o] == dev_node[d];
    if (D <= 1 || n == 0 || !any) return deal_objects(bytes, D);
    std::vector<size_t> order(n);
    std::iota(order.begin(), order.end(), size_t(0));
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return bytes[a] > bytes[b]; });
    uint64_t total = 0;
    for (uint64_t b : bytes) total += b;
    const double fair = double(total) / D;
    std::vector<uint64_t> load(D, 0);
    std::vector<uint32_t> dev(n, 0);
    for (size_t o : order) {
        uint32_t all = 0;
        int local = -1;
        for (uint32_t d = 0; d < D; ++d) {
            if (load[d] < load[all]) all = d;
            if (node[o] >= 0 && dev_node[d] == node[o] && (local < 0 || load[d] < load[uint32_t(local)])) local = int(d);
        }
        const bool fits = local >= 0 && double(load[uint32_t(local)] + bytes[o]) <= fair + 0.5 * double(bytes[o]);
        const uint32_t pick = fits ? uint32_t(local) : all;
        dev[o] = pick;
        load[pick] += bytes[o];
    }
    return dev;
}

}  // namespace mxec

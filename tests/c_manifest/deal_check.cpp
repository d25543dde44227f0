// CPU unit test of the host-batch dealing (maxio_amd/csrc/deal.hpp, used by
// pipeline.cpp mxec_encode_batch_host): a uniform batch keeps o mod D; a
// mixed 64 KiB..10 MiB batch over 8 devices lands within 10 % bytes.
#include <cstdio>
#include <random>

#include "../../maxio_amd/csrc/deal.hpp"

using namespace mxec;

static int fails = 0;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::fprintf(stderr, "FAIL line %d: %s\n", __LINE__, #c); \
            ++fails;                                                  \
        }                                                             \
    } while (0)

int main() {
    // uniform: o mod D
    std::vector<uint64_t> u(1000, 6 * (uint64_t(10) << 20));
    auto du = deal_objects(u, 8);
    for (size_t o = 0; o < u.size(); ++o) CHECK(du[o] == o % 8);
    CHECK(deal_objects(u, 1) == std::vector<uint32_t>(u.size(), 0));
    CHECK(deal_objects({}, 8).empty());
    // mixed configs[4] stream: (4+2 / 8+4 / 10+4) x (64 KiB .. 10 MiB)
    const int km[3][2] = {{4, 2}, {8, 4}, {10, 4}};
    const uint64_t sizes[5] = {64 << 10, 256 << 10, 1 << 20, 4 << 20, 10 << 20};
    for (uint32_t D : {2u, 4u, 8u}) {
        for (int seed = 0; seed < 20; ++seed) {
            std::mt19937_64 rng(seed);
            std::vector<uint64_t> b;
            for (int o = 0; o < 600; ++o) {
                const auto& c = km[rng() % 3];
                b.push_back(uint64_t(c[0] + c[1]) * sizes[rng() % 5]);
            }
            auto d = deal_objects(b, D);
            std::vector<uint64_t> load(D, 0);
            uint64_t total = 0;
            for (size_t o = 0; o < b.size(); ++o) {
                CHECK(d[o] < D);
                load[d[o]] += b[o];
                total += b[o];
            }
            const double mean = double(total) / D;
            for (uint32_t x = 0; x < D; ++x) CHECK(load[x] > 0.9 * mean && load[x] < 1.1 * mean);
            // round robin by count on the same batch is what this replaces
            CHECK(deal_objects(b, D) == d);  // deterministic
        }
    }
    // NUMA-aware deal (deal_objects_numa) on a two-node host: devices 0-3 on
    // node 0, 4-7 on node 1 (a fake node map, as an 8-GPU two-socket box).
    const std::vector<int> two = {0, 0, 0, 0, 1, 1, 1, 1};
    {
        // no page information: exactly deal_objects
        std::vector<int> none(u.size(), -1);
        CHECK(deal_objects_numa(u, none, two) == deal_objects(u, 8));
        // a node no device sits on counts as unknown
        std::vector<int> far(u.size(), 2);
        CHECK(deal_objects_numa(u, far, two) == deal_objects(u, 8));
        // uniform, pages alternating between the nodes: every object local,
        // 125 objects per device
        std::vector<int> alt(u.size());
        for (size_t o = 0; o < u.size(); ++o) alt[o] = int(o % 2);
        auto d = deal_objects_numa(u, alt, two);
        std::vector<int> count(8, 0);
        for (size_t o = 0; o < u.size(); ++o) {
            CHECK(two[d[o]] == alt[o]);
            ++count[d[o]];
        }
        for (int c : count) CHECK(c == 125);
        // uniform, every page on node 1: still every device, evenly (the
        // remote ones take the excess), node-1 devices first
        std::vector<int> one(u.size(), 1);
        d = deal_objects_numa(u, one, two);
        std::fill(count.begin(), count.end(), 0);
        for (size_t o = 0; o < u.size(); ++o) ++count[d[o]];
        for (int c : count) CHECK(c == 125);
        CHECK(d[0] >= 4);  // the first (longest, stable order) object goes local
        // one device per node
        auto d2 = deal_objects_numa(u, alt, {0, 1});
        for (size_t o = 0; o < u.size(); ++o) CHECK(d2[o] == uint32_t(o % 2));
    }
    // mixed configs[4] sizes with pages spread over the nodes at random:
    // within 10 % of the mean per device, and nearly every object local
    for (int seed = 0; seed < 20; ++seed) {
        std::mt19937_64 rng(100 + seed);
        std::vector<uint64_t> b;
        std::vector<int> nd;
        for (int o = 0; o < 600; ++o) {
            const auto& c = km[rng() % 3];
            b.push_back(uint64_t(c[0] + c[1]) * sizes[rng() % 5]);
            nd.push_back(int(rng() % 2));
        }
        auto d = deal_objects_numa(b, nd, two);
        std::vector<uint64_t> load(8, 0);
        uint64_t total = 0, local = 0;
        for (size_t o = 0; o < b.size(); ++o) {
            CHECK(d[o] < 8);
            load[d[o]] += b[o];
            total += b[o];
            local += two[d[o]] == nd[o] ? b[o] : 0;
        }
        for (uint32_t x = 0; x < 8; ++x) CHECK(load[x] > 0.9 * total / 8 && load[x] < 1.1 * total / 8);
        CHECK(local > 0.85 * total);
        CHECK(deal_objects_numa(b, nd, two) == d);  // deterministic
    }
    if (fails) return 1;
    std::printf("deal ok\n");
    return 0;
}

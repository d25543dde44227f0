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
    if (fails) return 1;
    std::printf("deal ok\n");
    return 0;
}

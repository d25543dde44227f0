// CPU unit test of the SHA-256 stream form's item-counter guard
// (maxio_amd/csrc/sha_plan.hpp, used by ops.cpp run_sha).
#include <cstdio>
#include <cstdlib>

#include "../../maxio_amd/csrc/sha_plan.hpp"

using namespace mxec;

static int fails = 0;
#define CHECK(c)                                              \
    do {                                                      \
        if (!(c)) {                                           \
            std::fprintf(stderr, "FAIL line %d: %s\n", __LINE__, #c); \
            ++fails;                                          \
        }                                                     \
    } while (0)

int main() {
    const uint32_t seg = 512;   // kShaSegBlocks
    const uint64_t waves = 1024;  // one per SIMD on 256 CUs
    // configs[2]-sized batches: 10 240 ... 131 072 x 1 MiB messages
    CHECK(sha_stream_seg_max(1 << 20, seg) == 33);
    CHECK(sha_stream_items_fit(10240, 33, waves));
    CHECK(sha_stream_items_fit(131072, 33, waves));
    // ~4M short messages plus one 2 GiB shard: 65 536 groups x
    // 65 537 segments wraps a uint32 -> the stream form must be refused.
    const uint64_t sm = sha_stream_seg_max(uint64_t(2) << 30, seg);
    CHECK(sm == 65537);
    CHECK(!sha_stream_items_fit(uint64_t(4) << 20, sm, waves));
    // the exact edge: groups * seg_max + waves == 2^32 - 1 fits, one more does not
    const uint64_t g = 65535;  // groups
    const uint64_t s_ok = (uint64_t(UINT32_MAX) - waves) / g;
    CHECK(sha_stream_items_fit(g * 64, s_ok, waves));
    CHECK(!sha_stream_items_fit(g * 64, s_ok + 1, waves));
    CHECK(!sha_stream_items_fit(0, 1, waves));
    CHECK(!sha_stream_items_fit(64, 0, waves));
    CHECK(!sha_stream_items_fit(64, uint64_t(UINT32_MAX) + 1, waves));
    if (fails) return 1;
    std::printf("sha guard ok\n");
    return 0;
}

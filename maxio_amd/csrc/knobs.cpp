// knobs.cpp — read_knobs(): the one place the shipping library reads its
// environment (called by mxec_open).
#include "knobs.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace mxec {

const char* const kKnobNames[] = {
    "MXEC_TEST_LOGICAL_DEVICES", "MXEC_TEST_RS_GRID", "MXEC_TEST_COEF_ARENA_KB", "MXEC_DEBUG_AFFINITY",
    "MXEC_HOST_NUMA",            "MXEC_SPIN_WAIT",    "MXEC_RS_TUNE",            "MXEC_RS_MULTI",
    "MXEC_SHA_FORM",             "MXEC_DESC_UPLOAD",  "MXEC_PIPE_PIECE_MB",      "MXEC_GET_WINDOW",
    "MXEC_PIPE_COPY",
    "MXEC_GATHER_US",            "MXEC_GATHER_MAX_US", "MXEC_GATHER_IDLE_US",    "MXEC_COMBINE_BELOW",
    "MXEC_COMBINE_STREAMS",      "MXEC_COMBINE_PRIORITY", "MXEC_COMBINE_LOG",    nullptr};

namespace {
const char* env(const char* name) {
    const char* e = std::getenv(name);
    return e && *e ? e : nullptr;
}
long env_long(const char* name, long dflt) {
    const char* e = env(name);
    return e ? std::strtol(e, nullptr, 10) : dflt;
}
bool env_flag(const char* name, bool dflt) {
    const char* e = env(name);
    return e ? std::strcmp(e, "0") != 0 : dflt;
}
}  // namespace

Knobs read_knobs() {
    Knobs k;
    k.test_logical_devices = int(std::max(1L, std::min(8L, env_long("MXEC_TEST_LOGICAL_DEVICES", 1))));
    if (k.test_logical_devices > 1)
        std::fprintf(stderr, "maxio_ec: MXEC_TEST_LOGICAL_DEVICES=%d: every selected GPU is opened %d times "
                             "as separate devices (test-only setting)\n",
                     k.test_logical_devices, k.test_logical_devices);
    const long grid = env_long("MXEC_TEST_RS_GRID", 0);
    if (grid > 0) {
        k.test_rs_grid = uint32_t(std::min(grid, 1L << 30));
        std::fprintf(stderr, "maxio_ec: MXEC_TEST_RS_GRID=%u: RS launches capped at %u workgroups (test-only setting)\n",
                     k.test_rs_grid, k.test_rs_grid);
    }
    const long arena_kb = env_long("MXEC_TEST_COEF_ARENA_KB", 0);
    if (arena_kb > 0) {
        k.test_coef_arena = uint64_t(std::min(arena_kb, 64L << 10)) << 10;
        std::fprintf(stderr, "maxio_ec: MXEC_TEST_COEF_ARENA_KB=%ld: coefficient arena of %ld KiB per half "
                             "(test-only setting)\n",
                     arena_kb, long(k.test_coef_arena >> 10));
    }
    k.debug_affinity = env_flag("MXEC_DEBUG_AFFINITY", false);
    k.host_numa = env_flag("MXEC_HOST_NUMA", false);
    k.spin_wait = env_flag("MXEC_SPIN_WAIT", false);
    k.rs_tune = env_flag("MXEC_RS_TUNE", true);
    k.rs_multi = env_flag("MXEC_RS_MULTI", true);
    if (const char* f = env("MXEC_SHA_FORM")) {
        if (!std::strcmp(f, "one")) k.sha_form = 1;
        else if (!std::strcmp(f, "split")) k.sha_form = 2;
        else if (!std::strcmp(f, "stream")) k.sha_form = 3;
        else if (!std::strcmp(f, "lagpair")) k.sha_form = 6;
    }
    if (const char* u = env("MXEC_DESC_UPLOAD")) k.desc_upload = !std::strcmp(u, "inline") ? 0 : !std::strcmp(u, "stream") ? 2 : 1;
    const long piece = env_long("MXEC_PIPE_PIECE_MB", 1);
    k.pipe_piece = piece <= 0 ? 0 : uint64_t(std::min(piece, 1L << 20)) << 20;
    k.pipe_piece_auto = env("MXEC_PIPE_PIECE_MB") == nullptr;
    if (const char* c = env("MXEC_PIPE_COPY"))
        k.pipe_copy = !std::strcmp(c, "sdma") ? 0 : !std::strcmp(c, "waves") ? 1 : 2;
    if (const char* w = env("MXEC_GET_WINDOW")) k.get_window = std::max<uint64_t>(1, std::strtoull(w, nullptr, 10));
    k.gather_us = env_long("MXEC_GATHER_US", k.gather_us);
    k.gather_max_us = env_long("MXEC_GATHER_MAX_US", k.gather_max_us);
    k.gather_idle_us = env_long("MXEC_GATHER_IDLE_US", k.gather_idle_us);
    if (const char* b = env("MXEC_COMBINE_BELOW")) k.combine_below = size_t(std::strtoull(b, nullptr, 10));
    k.combine_streams = int(std::max(1L, std::min(4L, env_long("MXEC_COMBINE_STREAMS", 2))));
    k.combine_priority = env_flag("MXEC_COMBINE_PRIORITY", true);
    k.combine_log = env_flag("MXEC_COMBINE_LOG", false);
    return k;
}

}  // namespace mxec

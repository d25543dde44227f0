// knobs.cpp — read_knobs(): the one place the shipping library reads its
// environment (called by mxec_open).
#include "knobs.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <strings.h>

namespace mxec {

const char* const kKnobNames[] = {
    "MXEC_DEBUG_AFFINITY",
    "MXEC_HOST_NUMA",            "MXEC_SPIN_WAIT",    "MXEC_RS_TUNE",            "MXEC_RS_MULTI",
    "MXEC_SHA_FORM",             "MXEC_DESC_UPLOAD",  "MXEC_PIPE_PIECE_MB",      "MXEC_GET_WINDOW",
    "MXEC_PIPE_COPY",            "MXEC_PIPE_SDMA_FLOOR",   "MXEC_GET_VGROUPS",   "MXEC_GET_SPECULATE",
    "MXEC_PIPE_LANES",
    "MXEC_GATHER_US",            "MXEC_GATHER_MAX_US", "MXEC_GATHER_IDLE_US",    "MXEC_COMBINE_BELOW",
    "MXEC_COMBINE_STREAMS",      "MXEC_COMBINE_PRIORITY", "MXEC_COMBINE_LOG",    nullptr};

namespace {
const char* env(const char* name) {
    const char* e = std::getenv(name);
    return e && *e ? e : nullptr;
}
// A value the library cannot read keeps the default, with a warning: a typo
// would otherwise change the context's behaviour for its whole life, silently.
void bad_value(const char* name, const char* value, const char* kept) {
    std::fprintf(stderr, "maxio_ec: %s=\"%s\" is not a recognised value; keeping the default (%s)\n", name, value,
                 kept);
}
bool parse_long(const char* name, long* out) {
    const char* e = env(name);
    if (!e) return false;
    char* end = nullptr;
    const long v = std::strtol(e, &end, 10);
    if (end == e || *end != '\0') {
        bad_value(name, e, "see INTEGRATION.md");
        return false;
    }
    *out = v;
    return true;
}
long env_long(const char* name, long dflt) {
    long v = dflt;
    return parse_long(name, &v) ? v : dflt;
}
// 0 / 1, and the usual spellings of false / true in any case (a
// deployment that sets MXEC_HOST_NUMA=true must not get the default).
bool env_flag(const char* name, bool dflt) {
    const char* e = env(name);
    if (!e) return dflt;
    static const char* const no[] = {"0", "false", "no", "off", nullptr};
    static const char* const yes[] = {"1", "true", "yes", "on", nullptr};
    for (int i = 0; no[i]; ++i)
        if (!strcasecmp(e, no[i])) return false;
    for (int i = 0; yes[i]; ++i)
        if (!strcasecmp(e, yes[i])) return true;
    bad_value(name, e, dflt ? "1" : "0");
    return dflt;
}
// One of `names` (NULL-terminated); its index, or -1 (warned) for anything else.
int env_choice(const char* name, const char* const* names, const char* kept) {
    const char* e = env(name);
    if (!e) return -1;
    for (int i = 0; names[i]; ++i)
        if (!std::strcmp(e, names[i])) return i;
    bad_value(name, e, kept);
    return -1;
}
}  // namespace

Knobs read_knobs() {
    Knobs k;
    k.debug_affinity = env_flag("MXEC_DEBUG_AFFINITY", false);
    k.host_numa = env_flag("MXEC_HOST_NUMA", false);
    k.spin_wait = env_flag("MXEC_SPIN_WAIT", false);
    k.rs_tune = env_flag("MXEC_RS_TUNE", true);
    k.rs_multi = env_flag("MXEC_RS_MULTI", true);
    {
        static const char* const forms[] = {"auto", "one", "split", "stream", "lagpair", nullptr};
        static const int form_id[] = {0, 1, 2, 3, 6};
        const int f = env_choice("MXEC_SHA_FORM", forms, "auto");
        if (f >= 0) k.sha_form = form_id[f];
    }
    {
        static const char* const modes[] = {"inline", "auto", "stream", nullptr};
        const int u = env_choice("MXEC_DESC_UPLOAD", modes, "auto");
        if (u >= 0) k.desc_upload = u;
    }
    long piece = 0;
    if (parse_long("MXEC_PIPE_PIECE_MB", &piece)) {  // unset or unreadable: chosen per wave
        k.pipe_piece = piece <= 0 ? 0 : uint64_t(std::min(piece, 1L << 20)) << 20;
        k.pipe_piece_auto = false;
    }
    {
        static const char* const modes[] = {"sdma", "waves", "auto", nullptr};
        const int c = env_choice("MXEC_PIPE_COPY", modes, "auto");
        if (c >= 0) k.pipe_copy = c;
    }
    k.pipe_sdma_floor = std::max(0L, env_long("MXEC_PIPE_SDMA_FLOOR", k.pipe_sdma_floor));
    k.get_vgroups = int(std::max(0L, std::min(8L, env_long("MXEC_GET_VGROUPS", 0))));
    k.get_speculate = env_flag("MXEC_GET_SPECULATE", true);
    k.pipe_lanes = int(std::max(1L, std::min(8L, env_long("MXEC_PIPE_LANES", k.pipe_lanes))));
    long window = 0;
    if (parse_long("MXEC_GET_WINDOW", &window)) k.get_window = uint64_t(std::max(1L, window));
    k.gather_us = env_long("MXEC_GATHER_US", k.gather_us);
    k.gather_max_us = env_long("MXEC_GATHER_MAX_US", k.gather_max_us);
    k.gather_idle_us = env_long("MXEC_GATHER_IDLE_US", k.gather_idle_us);
    long below = 0;
    if (parse_long("MXEC_COMBINE_BELOW", &below)) k.combine_below = size_t(std::max(0L, below));
    k.combine_streams = int(std::max(1L, std::min(4L, env_long("MXEC_COMBINE_STREAMS", 2))));
    k.combine_priority = env_flag("MXEC_COMBINE_PRIORITY", true);
    k.combine_log = env_flag("MXEC_COMBINE_LOG", false);
    return k;
}

}  // namespace mxec

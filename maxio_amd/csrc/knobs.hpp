// knobs.hpp — the library's documented settings, read
// from the environment ONCE, when mxec_open creates a context, and kept in
// that context.  Nothing in the shipping library reads the environment at
// launch time, and no setting selects a kernel that the default never runs:
// the lab forms and their knobs (tools/, `make lab`) exist only in builds
// compiled with -DMXEC_LAB.
#pragma once

#include <cstddef>
#include <cstdint>

namespace mxec {

struct Knobs {
    // --- test-only: set by mxec_open_test's arguments, never by the environment
    int test_logical_devices = 1;  // open each GPU N times (N <= 8)
    uint32_t test_rs_grid = 0;     // cap on workgroups per RS launch (uniform, grouped, multi-r,
                                   //   edge): every workgroup walks many tiles
    uint64_t test_coef_arena = 0;  // coefficient-table arena per half (bytes)
    // --- debugging ------------------------------------------------------------
    bool debug_affinity = false;   // MXEC_DEBUG_AFFINITY: device-affinity checks on every launch
    // --- production ----------------------------------------------------------
    bool host_numa = false;        // MXEC_HOST_NUMA: mxec_host_alloc on the GPUs' NUMA node
    bool spin_wait = false;        // MXEC_SPIN_WAIT: host waits spin instead of sleeping
    bool rs_tune = true;           // MXEC_RS_TUNE: online grid choice for large uniform RS launches
    bool rs_multi = true;          // MXEC_RS_MULTI: mixed-r batches as one multi-r launch
    int sha_form = 0;              // MXEC_SHA_FORM: 0 auto, 1 one, 2 split, 3 stream, 6 lagpair
    int desc_upload = 1;           // MXEC_DESC_UPLOAD: 0 inline, 1 auto, 2 side stream
    uint64_t pipe_piece = uint64_t(1) << 20;  // MXEC_PIPE_PIECE_MB (0: whole chunks)
    bool pipe_piece_auto = true;   // MXEC_PIPE_PIECE_MB unset: 1, 2 or 4 MiB per wave (pipeline.cpp)
    int pipe_copy = 2;             // MXEC_PIPE_COPY: 0 sdma (hipMemcpyAsync); 1 waves (copy_kernel.hip
                                   //   for every host batch); 2 auto: SDMA, its upload rate timed as
                                   //   it goes; waves after it runs below pipe_sdma_floor
    long pipe_sdma_floor = 20;     // MXEC_PIPE_SDMA_FLOOR: GB/s (auto's switch point; 0: never waves)
    uint64_t get_window = uint64_t(1) << 30;  // MXEC_GET_WINDOW: bytes of chunks per GET window
    int get_vgroups = 0;           // MXEC_GET_VGROUPS: verification groups of a verified host GET wave (1..8; 0 = per wave)
    bool get_speculate = true;     // MXEC_GET_SPECULATE: the verified host GET rebuilds each piece as it
                                   //   arrives, before the verdict (pipeline.cpp spec_piece)
    int pipe_lanes = 4;            // MXEC_PIPE_LANES: host-batch calls admitted at once per device (1..8)
    long gather_us = 100;          // MXEC_GATHER_US
    long gather_max_us = 2000;     // MXEC_GATHER_MAX_US
    long gather_idle_us = 300;     // MXEC_GATHER_IDLE_US
    size_t combine_below = 0;      // MXEC_COMBINE_BELOW (0: combine every request)
    int combine_streams = 2;       // MXEC_COMBINE_STREAMS (1..4)
    bool combine_priority = true;  // MXEC_COMBINE_PRIORITY
    bool combine_log = false;      // MXEC_COMBINE_LOG
};

// Reads every documented MXEC_* variable (unset: the defaults above).
Knobs read_knobs();

// The names read_knobs looks up, NULL-terminated (tests compare them with
// INTEGRATION.md's table and with the library's strings).
extern const char* const kKnobNames[];

}  // namespace mxec

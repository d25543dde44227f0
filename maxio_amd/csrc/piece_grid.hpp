// piece_grid.hpp -- the piece grid of the host pipeline's piece-major waves
// (pipeline.cpp wave_pieces / verify_enqueue).  Header-only and free of HIP
// so tests/c_manifest/piece_grid_check.cpp can test it on the CPU.
//
// A wave moves every chunk in pieces: a ramp of pieces doubling from `ramp`
// bytes up to P (chain-bound verified GET waves ramp from 256 KiB: a smaller
// first piece starts every chain sooner; lab MXEC_PIPE_RAMP_KB overrides),
// then pieces of P.  A wave may widen P from a piece on (widen: a second call
// started sharing the device) -- the pieces already issued keep their
// offsets, so the grid stays a contiguous tiling of [0, longest).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <vector>

namespace mxec {

struct PieceGrid {
    // A run of uniform pieces: piece pc0 starts at off0, every piece P wide
    // until the next run's pc0.
    struct Run {
        uint64_t pc0, off0, P;
    };
    std::vector<uint64_t> starts;  // the ramp's pieces
    uint64_t P, ramp_end = 0;      // P: the current (last) run's width
    std::vector<Run> runs;         // after the ramp; widen() appends
    PieceGrid(uint64_t p, uint64_t ramp) : P(p) {
        uint64_t w = ramp;
#ifdef MXEC_LAB
        if (const char* e = getenv("MXEC_PIPE_RAMP_KB")) w = uint64_t(atol(e)) << 10;  // lab override
#endif
        w = w / 64 * 64;
        for (; w && w < p; w *= 2) {
            starts.push_back(ramp_end);
            ramp_end += w;
        }
        runs.push_back(Run{starts.size(), ramp_end, p});
    }
    const Run& run_of(uint64_t pc) const {
        size_t i = runs.size() - 1;
        while (i > 0 && runs[i].pc0 > pc) --i;
        return runs[i];
    }
    uint64_t start(uint64_t pc) const {
        if (pc < starts.size()) return starts[pc];
        const Run& r = run_of(pc);
        return r.off0 + (pc - r.pc0) * r.P;
    }
    uint64_t width(uint64_t pc) const {
        if (pc < starts.size()) return (pc + 1 < starts.size() ? starts[pc + 1] : ramp_end) - starts[pc];
        return run_of(pc).P;
    }
    // Pieces that cover [0, longest); at least one (an empty message's).
    uint64_t count(uint64_t longest) const {
        for (uint64_t pc = 0; pc < starts.size(); ++pc)
            if (longest <= start(pc) + width(pc)) return pc + 1;
        for (size_t i = 0; i < runs.size(); ++i) {
            const Run& r = runs[i];
            if (i + 1 < runs.size() && longest > runs[i + 1].off0) continue;
            const uint64_t rest = longest > r.off0 ? (longest - r.off0 + r.P - 1) / r.P : 0;
            return std::max<uint64_t>(1, r.pc0 + rest);
        }
        return 1;  // not reached
    }
    // Pieces from pc on (pc past the ramp, not yet issued) are p wide; the
    // pieces before pc keep their offsets and widths.
    void widen(uint64_t pc, uint64_t p) {
        const uint64_t off = start(pc);
        while (runs.size() > 1 && runs.back().pc0 >= pc) runs.pop_back();
        if (runs.back().pc0 == pc) runs.back() = Run{pc, off, p};
        else runs.push_back(Run{pc, off, p});
        P = p;
    }
};

}  // namespace mxec

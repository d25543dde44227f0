// CPU unit test of the piece grid of the host pipeline's piece-major waves
// (maxio_amd/csrc/piece_grid.hpp): with and without a ramp, with P widened
// from any piece past the ramp, the pieces tile [0, longest) contiguously,
// the ramp doubles from its first width, count() is the number of pieces the
// waves loop over (one for an empty message), and a widened grid keeps the
// offsets of the pieces already issued.
#include <cstdio>

#include "../../maxio_amd/csrc/piece_grid.hpp"

using namespace mxec;

static int fails = 0;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::fprintf(stderr, "FAIL line %d: %s\n", __LINE__, #c); \
            ++fails;                                                  \
        }                                                             \
    } while (0)

constexpr uint64_t KiB = 1024, MiB = 1024 * KiB;

// Walks the grid as wave_pieces does (count re-read every piece), widening
// to `wide` at piece `at` (0: never); checks the tiling.
static void walk(uint64_t P, uint64_t ramp, uint64_t longest, uint64_t at, uint64_t wide) {
    PieceGrid g(P, ramp);
    std::vector<uint64_t> before;  // offsets of the pieces issued before the widening
    uint64_t off = 0, pieces = 0;
    for (uint64_t pc = 0; pc < g.count(longest); ++pc) {
        if (at && pc == at && pc >= g.starts.size()) g.widen(pc, wide);
        CHECK(g.start(pc) == off);
        const uint64_t w = g.width(pc);
        CHECK(w > 0 && w % 64 == 0);
        if (pc + 1 < g.starts.size()) CHECK(g.width(pc + 1) == 2 * w);  // the ramp doubles
        if (!at || pc < at) before.push_back(off);
        off += w;
        ++pieces;
        CHECK(pieces < 100000);
        if (pieces >= 100000) return;
    }
    CHECK(pieces >= 1);
    CHECK(off >= longest);                            // covered
    CHECK(longest == 0 || off - g.width(pieces - 1) < longest);  // no piece past the end
    for (size_t i = 0; i < before.size(); ++i) CHECK(g.start(i) == before[i]);
}

int main() {
    // no ramp: ceil(longest / P) pieces, one for an empty message
    {
        PieceGrid g(MiB, 0);
        CHECK(g.count(0) == 1);
        CHECK(g.count(1) == 1);
        CHECK(g.count(MiB) == 1);
        CHECK(g.count(MiB + 1) == 2);
        CHECK(g.count(10 * MiB) == 10);
        CHECK(g.start(3) == 3 * MiB && g.width(3) == MiB);
    }
    // the 256 KiB ramp up to 1 MiB: 256 K, 512 K, then 1 MiB pieces
    {
        PieceGrid g(MiB, 256 * KiB);
        CHECK(g.starts.size() == 2 && g.ramp_end == 768 * KiB);
        CHECK(g.width(0) == 256 * KiB && g.width(1) == 512 * KiB && g.width(2) == MiB);
        CHECK(g.start(2) == 768 * KiB && g.start(3) == 768 * KiB + MiB);
        CHECK(g.count(100 * KiB) == 1);
        CHECK(g.count(768 * KiB) == 2);
        CHECK(g.count(10 * MiB) == 2 + 10);  // 768 K + 10 x 1 MiB >= 10 MiB, 9 would not
    }
    // widening to 2 MiB from piece 4 of a 1 MiB grid with the ramp
    {
        PieceGrid g(MiB, 256 * KiB);
        const uint64_t s4 = g.start(4);
        g.widen(4, 2 * MiB);
        CHECK(g.start(4) == s4 && g.width(4) == 2 * MiB && g.start(5) == s4 + 2 * MiB);
        CHECK(g.start(3) == 768 * KiB + MiB && g.width(3) == MiB);  // pieces before 4 keep 1 MiB
        CHECK(g.count(s4) == 4 && g.count(s4 + 1) == 5 && g.count(s4 + 2 * MiB + 1) == 6);
        g.widen(6, 4 * MiB);  // twice
        CHECK(g.start(5) == s4 + 2 * MiB && g.width(5) == 2 * MiB && g.start(6) == s4 + 4 * MiB);
        CHECK(g.width(6) == 4 * MiB && g.P == 4 * MiB && g.count(s4 + 4 * MiB + 1) == 7);
    }
    for (uint64_t longest : {uint64_t(0), uint64_t(64), 1000 * KiB, 10 * MiB, 10 * MiB + 4096, 37 * MiB + 192})
        for (uint64_t ramp : {uint64_t(0), 256 * KiB})
            for (uint64_t at : {uint64_t(0), uint64_t(2), uint64_t(3), uint64_t(7), uint64_t(20)}) {
                walk(MiB, ramp, longest, at, 2 * MiB);
                walk(2 * MiB, ramp, longest, at, 4 * MiB);
            }
    if (fails) return 1;
    std::printf("piece grid ok\n");
    return 0;
}

// kernels.hpp — launch interface of the gfx950 kernels (rs_kernel.hip,
// sha256_kernel.hip).  Host code builds the descriptor tables in device
// memory and calls these launchers on a HIP stream.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mxec {

// One launch applies an r x k GF(2^8) matrix to a batch of objects that share
// (k, r, shard_size):  out[o][i][b] = XOR_j coef(o)[i][j] * in[o][j][b].
// Bytes of input j at or beyond in_len[o][j] read as zero (the crate's
// zero padding, filesystem.rs:1111 / chunk_reader.rs:192); output i is written
// for b < out_len[o][i] only.
struct RsArgs {
    const uint8_t* const* in_ptrs;  // [n_obj][k]
    uint8_t* const* out_ptrs;       // [n_obj][r_total]; this launch writes rows
                                    //   [row0, row0 + r)
    const uint64_t* in_len;         // [n_obj][k]
    const uint64_t* out_len;        // [n_obj][r_total]
    const uint32_t* coef;           // tables, [j][i][8] per matrix (gf256.hpp)
    const uint32_t* coef_off;       // [n_obj] dword offset of object's table
    const uint64_t* edge_list;      // [n_edge] object << 32 | tile: tiles a
                                    //   length boundary or the shard end cuts
    uint64_t n_edge;
    uint64_t edge_tile_bytes;       // tile size the list was built for
    uint64_t shard_size;
    uint32_t n_obj, k, r, r_total, row0;
    uint32_t aligned;               // all pointers 16-byte aligned (else every
                                    //   tile is in the edge list)
};

// Tuning knobs of the interior kernel (tools/kernel_lab.cpp sweeps them).
struct RsVariant {
    int vecs = 2;           // 16-byte column vectors per lane per tile (1, 2, 4)
    bool nt = false;        // nontemporal loads / stores
    int blocks_per_cu = 8;  // grid = n_cus * blocks_per_cu (grid-stride)
};

hipError_t launch_rs_apply(const RsArgs& a, int n_cus, hipStream_t s);
hipError_t launch_rs_apply_variant(const RsArgs& a, int n_cus, hipStream_t s, const RsVariant& v);
// Geometry the default launch uses for a given total row count, and its tile.
RsVariant rs_default_variant(uint32_t r_total);
uint64_t rs_tile_bytes(const RsVariant& v);

// SHA-256 over n messages, one lane per message.  If `expected` is set the
// kernel also writes ok[i] = (digest == expected[i]).
struct ShaArgs {
    const uint8_t* const* ptrs;  // [n]
    const uint64_t* lens;        // [n]
    uint8_t* digests;            // [n][32] (may be null when only ok is wanted)
    const uint8_t* expected;     // [*][32] or null
    const uint64_t* exp_idx;     // [n]: message i compares expected[exp_idx[i]]
                                 //   (null: expected[i])
    uint8_t* ok;                 // [n] or null
    uint32_t n;
    int force = 0;               // 0 auto, 1 one wave per 64 messages, 2 split
};

hipError_t launch_sha256(const ShaArgs& a, hipStream_t s);

}  // namespace mxec

// rs_kernel.hip — Reed-Solomon GF(2^8) encode / reconstruct for gfx950.
//
// Replaces the crate's pure-Rust code_some_slices (input-major MUL_TABLE
// lookups, one byte at a time) behind filesystem.rs:1123 (encode) and
// chunk_reader.rs:211 (reconstruct).  Both are the same operation: apply an
// r x k coefficient matrix to k input shards, column by column:
//     out[i][b] = XOR_j c[i][j] * in[j][b].
//
// Design (CDNA4):
//  * HBM-bound streaming: each lane owns 16-byte columns, loads them with
//    global_load_dwordx4 (1 KiB per wave-instruction, fully coalesced), so one
//    workgroup tile covers 256 lanes x 16 B x V columns of every shard.
//  * No LDS tables and no byte lookups: c*x for 4 packed bytes is three
//    v_perm_b32 byte-selects from 8-entry tables (bits 0-2, 3-5, 6-7 of x)
//    plus a v_bitop3 XOR3.  The tables depend only on c, are wave-uniform, and
//    arrive in SGPRs by scalar loads; one of each v_perm's two table dwords must
//    be a VGPR (gfx950 constant-bus limit 1), the copy is hoisted per column.
//  * Input shards are loaded in blocks of 4 so each lane keeps 4*V 16-byte
//    loads in flight; one launch covers every (object, tile) of a batch,
//    grid-stride over 512 workgroups per CU (a few tiles each, so the tiles
//    in flight stay together in memory; rs_default_variant).  Loads and
//    stores carry the nontemporal hint (every byte is touched once).
//  * Zero padding (the crate pads the short last chunk, filesystem.rs:1111)
//    is never materialised: in the fast kernel an input whose length ends at
//    or before a tile contributes zero and is not loaded; a tile that a
//    length boundary cuts through masks that shard's vectors at the boundary
//    in the same pass.  Launches with an unaligned pointer run the
//    byte-exact edge kernel over every tile instead (a per-launch tile list
//    built by the host, run_rs).
#include "kernels.hpp"

#include <cstdlib>
#include <cstring>

namespace mxec {
namespace {

constexpr int kThreads = 256;
constexpr uint64_t kEdgeTile = kThreads * 16;  // bytes per edge-kernel step

struct Vec4 {
    uint32_t w[4];
};

__device__ __forceinline__ Vec4 load16(const uint8_t* p) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    return Vec4{{v.x, v.y, v.z, v.w}};
}

__device__ __forceinline__ void store16(uint8_t* p, const uint32_t (&w)[4]) {
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// Edge path: byte-granular load of up to 16 bytes, zero past `valid`.
__device__ __forceinline__ Vec4 load_partial(const uint8_t* p, int64_t valid, bool aligned) {
    if (aligned && valid >= 16) return load16(p);
    Vec4 r{{0, 0, 0, 0}};
    for (int b = 0; b < 16; ++b)
        if (b < valid) r.w[b >> 2] |= uint32_t(p[b]) << (8 * (b & 3));
    return r;
}

__device__ __forceinline__ void store_partial(uint8_t* p, const uint32_t (&w)[4], int64_t valid,
                                              bool aligned) {
    if (aligned && valid >= 16) {
        store16(p, w);
        return;
    }
    for (int b = 0; b < 16; ++b)
        if (b < valid) p[b] = uint8_t(w[b >> 2] >> (8 * (b & 3)));
}

// acc[i] ^= c_i * x for R outputs, 4 packed bytes; t points at the [i][8]
// coefficient tables of one input column (see gf256.hpp coef_entry).
template <int R>
__device__ __forceinline__ void mac_dword(uint32_t (&acc)[R], uint32_t x, const uint32_t* __restrict__ t,
                                          const uint32_t (&hi)[R][2]) {
    const uint32_t s0 = x & 0x07070707u;
    const uint32_t s1 = (x >> 3) & 0x07070707u;
    const uint32_t s2 = (x >> 6) & 0x03030303u;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const uint32_t p0 = __builtin_amdgcn_perm(hi[i][0], t[8 * i + 0], s0);
        const uint32_t p1 = __builtin_amdgcn_perm(hi[i][1], t[8 * i + 2], s1);
        const uint32_t p2 = __builtin_amdgcn_perm(s2, t[8 * i + 4], s2);
        // gfx950 v_bitop3_b32: three-input XOR in one instruction.
        acc[i] = __builtin_amdgcn_bitop3_b32(acc[i], p0, p1, 0x96) ^ p2;
    }
}

template <int R, int V>
__device__ __forceinline__ void mac_column(uint32_t (&acc)[V][4][R], const Vec4 (&x)[V],
                                           const uint32_t* __restrict__ t) {
    // The high table dwords are made VGPR-resident once per input column and
    // reused for all V*4 dwords of this lane.
    uint32_t hi[R][2];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        hi[i][0] = __builtin_amdgcn_readfirstlane(t[8 * i + 1]);
        hi[i][1] = __builtin_amdgcn_readfirstlane(t[8 * i + 3]);
        asm volatile("" : "+v"(hi[i][0]), "+v"(hi[i][1]));
    }
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
        for (int w = 0; w < 4; ++w) mac_dword<R>(acc[v][w], x[v].w[w], t, hi);
}

// Two input columns at once: the six partial products of each output fold
// into the accumulator with three XOR3s (1.5 per input instead of an XOR3
// and an XOR), the VALU saving that matters at R >= 3, where the kernel's
// VALU issue sits near the HBM stream's pace.
template <int R, int V>
__device__ __forceinline__ void mac_column_pair(uint32_t (&acc)[V][4][R], const Vec4 (&xa)[V], const Vec4 (&xb)[V],
                                                const uint32_t* __restrict__ ta, const uint32_t* __restrict__ tb) {
    uint32_t ha[R][2], hb[R][2];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        ha[i][0] = __builtin_amdgcn_readfirstlane(ta[8 * i + 1]);
        ha[i][1] = __builtin_amdgcn_readfirstlane(ta[8 * i + 3]);
        hb[i][0] = __builtin_amdgcn_readfirstlane(tb[8 * i + 1]);
        hb[i][1] = __builtin_amdgcn_readfirstlane(tb[8 * i + 3]);
        asm volatile("" : "+v"(ha[i][0]), "+v"(ha[i][1]), "+v"(hb[i][0]), "+v"(hb[i][1]));
    }
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t a = xa[v].w[w], b = xb[v].w[w];
            const uint32_t a0 = a & 0x07070707u, a1 = (a >> 3) & 0x07070707u, a2 = (a >> 6) & 0x03030303u;
            const uint32_t b0 = b & 0x07070707u, b1 = (b >> 3) & 0x07070707u, b2 = (b >> 6) & 0x03030303u;
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const uint32_t pa0 = __builtin_amdgcn_perm(ha[i][0], ta[8 * i + 0], a0);
                const uint32_t pa1 = __builtin_amdgcn_perm(ha[i][1], ta[8 * i + 2], a1);
                const uint32_t pa2 = __builtin_amdgcn_perm(a2, ta[8 * i + 4], a2);
                const uint32_t pb0 = __builtin_amdgcn_perm(hb[i][0], tb[8 * i + 0], b0);
                const uint32_t pb1 = __builtin_amdgcn_perm(hb[i][1], tb[8 * i + 2], b1);
                const uint32_t pb2 = __builtin_amdgcn_perm(b2, tb[8 * i + 4], b2);
                uint32_t t = __builtin_amdgcn_bitop3_b32(acc[v][w][i], pa0, pa1, 0x96);
                t = __builtin_amdgcn_bitop3_b32(t, pa2, pb0, 0x96);
                acc[v][w][i] = __builtin_amdgcn_bitop3_b32(t, pb1, pb2, 0x96);
            }
        }
}

// Global-address-space views: pointers fetched from the descriptor tables are
// generic in HIP; casting them lets the backend emit global_load/store
// (vmcnt only) instead of flat_* (vmcnt + lgkmcnt).
typedef const uint8_t __attribute__((address_space(1)))* gcptr;
typedef uint8_t __attribute__((address_space(1)))* gptr;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// NT: nontemporal (streaming) hint on the loads and stores — every shard
// byte is touched exactly once per launch.
template <bool NT>
__device__ __forceinline__ Vec4 gload16(gcptr p) {
    const auto* q = (const u32x4 __attribute__((address_space(1)))*)(p);
    const u32x4 v = NT ? __builtin_nontemporal_load(q) : *q;
    return Vec4{{v.x, v.y, v.z, v.w}};
}
template <bool NT>
__device__ __forceinline__ void gstore16(gptr p, const uint32_t (&w)[4]) {
    u32x4 v = {w[0], w[1], w[2], w[3]};
    auto* q = (u32x4 __attribute__((address_space(1)))*)(p);
    if (NT) __builtin_nontemporal_store(v, q);
    else *q = v;
}

// Edge tiles (launches with an unaligned pointer): the list entries
// (object << 32 | tile index) are every tile of every object.  Each is walked in kEdgeTile steps with
// byte-exact bounds on every input and output.  One step:
template <int R>
__device__ __forceinline__ void edge_step(
    const uint8_t* const* __restrict__ in_ptrs, uint8_t* const* __restrict__ out_ptrs,
    const uint64_t* __restrict__ in_len, const uint64_t* __restrict__ out_len,
    const uint32_t* __restrict__ coef, const uint32_t* __restrict__ coef_off, uint64_t shard_size,
    uint32_t k, uint32_t r_total, uint32_t row0, const uint64_t* __restrict__ edge_list,
    uint32_t steps_per_tile, uint64_t tile_bytes, uint32_t aligned, uint64_t step) {
    const uint64_t e = edge_list[step / steps_per_tile];
    const uint32_t obj = uint32_t(e >> 32);
    const uint64_t col = uint64_t(uint32_t(e)) * tile_bytes + (step % steps_per_tile) * kEdgeTile +
                         threadIdx.x * 16;
    if (col >= shard_size) return;
    const uint32_t* __restrict__ tab = coef + coef_off[obj] + row0 * 8;
    uint32_t acc[1][4][R];
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int i = 0; i < R; ++i) acc[0][w][i] = 0;
    // Four inputs' loads in flight before their multiply-accumulates.
    // Whole vectors load unconditionally from a global address (a safe
    // dummy when the lane's vector is not whole) so the waits stay
    // counted; the lane whose vector a length boundary cuts, and
    // unaligned launches, take the byte path afterwards.
    const uint8_t* safe = reinterpret_cast<const uint8_t*>(coef);
    auto issue = [&](uint32_t j, Vec4& x, const uint8_t*& p, int64_t& valid) {
        const uint64_t len = in_len[uint64_t(obj) * k + j];
        valid = col < len ? int64_t(len - col) : 0;
        p = in_ptrs[uint64_t(obj) * k + j] + col;
        const bool full = aligned && valid >= 16;
        x = gload16<false>(gcptr(full ? p : safe));
    };
    // After all four loads are issued: zero what was not a whole vector
    // (selects, no branch), then the rare cut lane reads its bytes.
    auto fixup = [&](Vec4& x, const uint8_t* p, int64_t valid) {
        const bool full = aligned && valid >= 16;
#pragma unroll
        for (int w = 0; w < 4; ++w) x.w[w] = full ? x.w[w] : 0u;
        if (valid > 0 && !full) x = load_partial(p, valid, aligned != 0);
    };
    uint32_t j = 0;
    for (; j + 4 <= k; j += 4) {
        Vec4 x[4][1];
        const uint8_t* p[4];
        int64_t valid[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) issue(j + u, x[u][0], p[u], valid[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) fixup(x[u][0], p[u], valid[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) mac_column<R, 1>(acc, x[u], tab + (j + u) * r_total * 8);
    }
    for (; j < k; ++j) {
        Vec4 x[1];
        const uint8_t* p;
        int64_t valid;
        issue(j, x[0], p, valid);
        fixup(x[0], p, valid);
        mac_column<R, 1>(acc, x, tab + j * r_total * 8);
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
        uint64_t olen = out_len[uint64_t(obj) * r_total + row0 + i];
        if (olen > shard_size) olen = shard_size;
        if (col < olen) {
            uint32_t o[4] = {acc[0][0][i], acc[0][1][i], acc[0][2][i], acc[0][3][i]};
            store_partial(out_ptrs[uint64_t(obj) * r_total + row0 + i] + col, o, int64_t(olen - col),
                          aligned != 0);
        }
    }
}

// The edge steps alone (unaligned launches: every tile is an edge tile).
template <int R>
__global__ __launch_bounds__(kThreads) void rs_apply_edge(
    const uint8_t* const* __restrict__ in_ptrs, uint8_t* const* __restrict__ out_ptrs,
    const uint64_t* __restrict__ in_len, const uint64_t* __restrict__ out_len,
    const uint32_t* __restrict__ coef, const uint32_t* __restrict__ coef_off, uint64_t shard_size,
    uint32_t k, uint32_t r_total, uint32_t row0, const uint64_t* __restrict__ edge_list,
    uint32_t steps_per_tile, uint64_t tile_bytes, uint32_t aligned, uint64_t n_steps) {
    for (uint64_t step = blockIdx.x; step < n_steps; step += gridDim.x)
        edge_step<R>(in_ptrs, out_ptrs, in_len, out_len, coef, coef_off, shard_size, k, r_total, row0, edge_list,
                     steps_per_tile, tile_bytes, aligned, step);
}

// Inputs and outputs that a length boundary cuts inside a tile (the short
// last data chunk, its decoded copy, a shard end that is not a tile
// multiple).  `valid` is a lane's count of bytes below the length from the
// start of its 16-byte vector (<= 0: none, >= 16: all).  A vector with at
// least one valid byte is loaded whole -- it is 16-byte aligned, so it lies
// in the page of its first byte -- and the bytes at or past the length are
// zeroed; a vector with none reads a safe dummy address, so every load
// stays unconditional and counted.
__device__ __forceinline__ Vec4 mask_tail(Vec4 x, int32_t valid) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int32_t nb = valid - 4 * w;
        const uint32_t mk = nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * nb)));
        x.w[w] &= mk;
    }
    return x;
}

template <bool NT>
__device__ __forceinline__ Vec4 gload16_upto(gcptr p, int32_t valid, gcptr safe) {
    return mask_tail(gload16<NT>(valid > 0 ? p : safe), valid);
}

// One tile of one object, 16-byte aligned pointers.  An input whose length
// ends at or before the tile reads as zero without a load, an output whose
// length ends there is not stored; a tile that a length boundary cuts
// through takes the masked loads / stores above for the cut shard only, in
// the same pass (config 5's short last chunks put one such tile in every
// object: a quarter of all tiles at 64 KiB chunks).  ip / il: the object's
// k inputs and lengths; op / ol: its R outputs and lengths; tab: its
// coefficient table at the first output row, input j's rows `stride` x 8
// dwords apart.
template <int R, int V, bool NT, bool LNT = NT, int G = 4>
__device__ __forceinline__ void rs_tile(const uint8_t* const* __restrict__ ip, const uint64_t* __restrict__ il,
                                        uint8_t* const* __restrict__ op, const uint64_t* __restrict__ ol,
                                        const uint32_t* __restrict__ tab, uint32_t k, uint32_t stride,
                                        uint64_t base, gcptr safe) {
    constexpr uint32_t kTile = kThreads * 16 * V;
    const uint64_t end = base + kTile;
    const uint64_t lane = base + threadIdx.x * 16;
    const int32_t lane_off = int32_t(threadIdx.x * 16);

    uint32_t acc[V][4][R];
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int i = 0; i < R; ++i) acc[v][w][i] = 0;

    // Input jj of a group: whole (the common case), zero, or cut.
    auto load_in = [&](uint32_t jj, Vec4 (&x)[V]) {
        const uint64_t len = il[jj];
        gcptr p = ((gcptr)(ip[jj])) + lane;
        if (len >= end) {
#pragma unroll
            for (int v = 0; v < V; ++v) x[v] = gload16<LNT>(p + v * kThreads * 16);
        } else if (len <= base) {
#pragma unroll
            for (int v = 0; v < V; ++v) x[v] = Vec4{{0, 0, 0, 0}};
        } else {
            const int32_t d = int32_t(len - base) - lane_off;
#pragma unroll
            for (int v = 0; v < V; ++v)
                x[v] = gload16_upto<LNT>(p + v * kThreads * 16, d - v * int32_t(kThreads * 16), safe);
        }
    };

    uint32_t j = 0;
    if constexpr (G == 8) {
        // Eight inputs' loads in flight per step (the lab's G = 8 form: with
        // V = 2 the same bytes in flight per lane as V = 4 x 4 inputs, half
        // the accumulators, so more waves fit).
        for (; j + 8 <= k; j += 8) {
            Vec4 x[8][V];
            bool full = true;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) full = full && il[j + jj] >= end;
            if (full) {
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) {
                    gcptr p = ((gcptr)(ip[j + jj])) + lane;
#pragma unroll
                    for (int v = 0; v < V; ++v) x[jj][v] = gload16<LNT>(p + v * kThreads * 16);
                }
            } else {
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) load_in(j + jj, x[jj]);
            }
            if constexpr (R >= 3) {
#pragma unroll
                for (int jj = 0; jj < 8; jj += 2)
                    mac_column_pair<R, V>(acc, x[jj], x[jj + 1], tab + (j + jj) * stride * 8,
                                          tab + (j + jj + 1) * stride * 8);
            } else {
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) mac_column<R, V>(acc, x[jj], tab + (j + jj) * stride * 8);
            }
        }
    }
    for (; j + 4 <= k; j += 4) {
        Vec4 x[4][V];
        // Wave-uniform: all four inputs reach past this tile (every tile
        // but the few at or past a short last chunk).  The common case
        // loads unconditionally; the per-input select would zero 4V
        // registers and branch around every load, one VALU per input
        // dword.
        if (il[j] >= end && il[j + 1] >= end && il[j + 2] >= end && il[j + 3] >= end) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                gcptr p = ((gcptr)(ip[j + jj])) + lane;
#pragma unroll
                for (int v = 0; v < V; ++v) x[jj][v] = gload16<LNT>(p + v * kThreads * 16);
            }
        } else {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) load_in(j + jj, x[jj]);
        }
        if constexpr (R >= 3) {
            mac_column_pair<R, V>(acc, x[0], x[1], tab + (j + 0) * stride * 8, tab + (j + 1) * stride * 8);
            mac_column_pair<R, V>(acc, x[2], x[3], tab + (j + 2) * stride * 8, tab + (j + 3) * stride * 8);
        } else {  // VALU has slack at R <= 2; one column at a time needs fewer VGPRs
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) mac_column<R, V>(acc, x[jj], tab + (j + jj) * stride * 8);
        }
    }
    for (; j < k; ++j) {
        if (il[j] <= base) continue;  // zero column: contributes nothing
        Vec4 x[V];
        load_in(j, x);
        mac_column<R, V>(acc, x, tab + j * stride * 8);
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const uint64_t olen = ol[i];
        if (olen <= base) continue;  // output ends at/before base
        gptr o = ((gptr)(op[i])) + lane;
        const int32_t d = olen >= end ? int32_t(kTile) : int32_t(olen - base) - lane_off;
#pragma unroll
        for (int v = 0; v < V; ++v) {
            uint32_t ov[4] = {acc[v][0][i], acc[v][1][i], acc[v][2][i], acc[v][3][i]};
            if (olen >= end) {
                gstore16<NT>(o + v * kThreads * 16, ov);
            } else {
                const int32_t valid = d - v * int32_t(kThreads * 16);
                if (valid >= 16) {
                    gstore16<NT>(o + v * kThreads * 16, ov);
                } else if (valid > 0) {  // the one straddling lane
                    for (int b = 0; b < valid; ++b)
                        o[v * kThreads * 16 + b] = uint8_t(ov[b >> 2] >> (8 * (b & 3)));
                }
            }
        }
    }
}

// Every tile of every object of a launch (grid-stride).
//
// GRP: a grouped launch — objects of different k and shard size that share
// r (config 5's mixed classes, a server's batch of mixed requests) in one
// grid: a 16-byte record per tile (object, k, first input entry, tile within
// the object), one wave-uniform scalar load, fetched one tile ahead so it
// is in SGPRs when the tile starts (the uniform kernel computes the same
// from the tile index).
template <int R, int V, bool NT, bool GRP, int OCC = 1, bool LNT = NT, int G = 4>
__global__ __launch_bounds__(kThreads, OCC) void rs_apply_fast(
    const uint8_t* const* __restrict__ in_ptrs, uint8_t* const* __restrict__ out_ptrs,
    const uint64_t* __restrict__ in_len, const uint64_t* __restrict__ out_len,
    const uint32_t* __restrict__ coef, const uint32_t* __restrict__ coef_off, uint32_t k_uniform,
    uint32_t r_total, uint32_t row0, uint32_t tiles_per_obj, uint64_t n_tiles,
    const RsTileRec* __restrict__ tiles) {
    constexpr uint32_t kTile = kThreads * 16 * V;
    const gcptr safe = (gcptr)(reinterpret_cast<const uint8_t*>(coef));
    RsTileRec next{};
    if constexpr (GRP) next = tiles[blockIdx.x];  // the grid never exceeds n_tiles
    for (uint64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        uint32_t obj, k;
        uint64_t base, in0;
        if constexpr (GRP) {
            const RsTileRec cur = next;
            if (tile + gridDim.x < n_tiles) next = tiles[tile + gridDim.x];
            obj = cur.obj;
            k = cur.k;
            in0 = cur.in0;
            base = uint64_t(cur.local) * kTile;
        } else {
            obj = uint32_t(tile / tiles_per_obj);
            base = (tile - uint64_t(obj) * tiles_per_obj) * kTile;
            k = k_uniform;
            in0 = uint64_t(obj) * k;
        }
        // Lengths are clamped to the shard size by the host, so a tile past
        // the shard end is cut by the same tests.
        rs_tile<R, V, NT, LNT, G>(in_ptrs + in0, in_len + in0, out_ptrs + uint64_t(obj) * r_total + row0,
                          out_len + uint64_t(obj) * r_total + row0, coef + coef_off[obj] + row0 * 8, k, r_total,
                          base, safe);
    }
}

// One grouped launch for objects of every output count r <= kMultiR (a
// step's encode of mixed m, or its decode of mixed erasure counts): the
// tile record's k field carries r in bits 16-23, an object's outputs sit at
// out_ptrs / out_len + obj * kMultiR (unused entries length 0), and each
// tile runs the body compiled for its r (a wave-uniform switch).  One launch
// instead of one per r: no ramp-down and ramp-up between them.
template <int V, bool NT>
__global__ __launch_bounds__(kThreads) void rs_apply_multi(
    const uint8_t* const* __restrict__ in_ptrs, uint8_t* const* __restrict__ out_ptrs,
    const uint64_t* __restrict__ in_len, const uint64_t* __restrict__ out_len,
    const uint32_t* __restrict__ coef, const uint32_t* __restrict__ coef_off, uint64_t n_tiles,
    const RsTileRec* __restrict__ tiles) {
    constexpr uint32_t kTile = kThreads * 16 * V;
    const gcptr safe = (gcptr)(reinterpret_cast<const uint8_t*>(coef));
    RsTileRec next = tiles[blockIdx.x];  // the grid never exceeds n_tiles
    for (uint64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const RsTileRec cur = next;
        if (tile + gridDim.x < n_tiles) next = tiles[tile + gridDim.x];
        const uint32_t k = cur.k & 0xFFFFu, r = (cur.k >> 16) & 0xFFu;
        const uint64_t base = uint64_t(cur.local) * kTile;
        const uint8_t* const* ip = in_ptrs + cur.in0;
        const uint64_t* il = in_len + cur.in0;
        uint8_t* const* op = out_ptrs + uint64_t(cur.obj) * kMultiR;
        const uint64_t* ol = out_len + uint64_t(cur.obj) * kMultiR;
        const uint32_t* tab = coef + coef_off[cur.obj];
        switch (r) {
            case 1: rs_tile<1, V, NT>(ip, il, op, ol, tab, k, 1, base, safe); break;
            case 2: rs_tile<2, V, NT>(ip, il, op, ol, tab, k, 2, base, safe); break;
            case 3: rs_tile<3, V, NT>(ip, il, op, ol, tab, k, 3, base, safe); break;
            default: rs_tile<4, V, NT>(ip, il, op, ol, tab, k, 4, base, safe); break;
        }
    }
}

// Grid of a launch over n items (tiles or edge steps): n_cus * per_cu,
// at most n (a grouped launch's first fetch needs every workgroup to own a
// tile) and at most the caller's cap (tests).
uint64_t grid_of(const RsArgs& a, int n_cus, int per_cu, uint64_t n) {
    uint64_t blocks = uint64_t(n_cus) * uint64_t(per_cu);
    if (a.max_blocks && blocks > a.max_blocks) blocks = a.max_blocks;
    return blocks > n ? n : blocks;
}

template <int R, int V, bool NT, bool GRP = false, int OCC = 1, bool LNT = NT, int G = 4>
hipError_t launch_fast(const RsArgs& a, uint32_t tiles_per_obj, uint64_t n_tiles, uint64_t blocks,
                       hipStream_t s) {
    hipLaunchKernelGGL((rs_apply_fast<R, V, NT, GRP, OCC, LNT, G>), dim3(uint32_t(blocks)), dim3(kThreads), 0, s,
                       a.in_ptrs, a.out_ptrs, a.in_len, a.out_len, a.coef, a.coef_off, a.k, a.r_total,
                       a.row0, tiles_per_obj, n_tiles, a.tiles);
    return hipGetLastError();
}

// Multi-r grouped launches (a.multi): V = 4, nontemporal, rs_group_variant's grid.
hipError_t launch_multi(const RsArgs& a, int n_cus, hipStream_t s) {
    const RsVariant v = rs_group_variant(kMultiR);
    const uint64_t blocks = grid_of(a, n_cus, v.blocks_per_cu, a.n_tiles);
    hipLaunchKernelGGL((rs_apply_multi<4, true>), dim3(uint32_t(blocks)), dim3(kThreads), 0, s, a.in_ptrs,
                       a.out_ptrs, a.in_len, a.out_len, a.coef, a.coef_off, a.n_tiles, a.tiles);
    return hipGetLastError();
}

// Grouped launches: rs_group_variant's geometry (nontemporal, V = 4 or 2).
template <int R>
hipError_t launch_grouped(const RsArgs& a, int n_cus, hipStream_t s) {
    const RsVariant v = rs_group_variant(uint32_t(R));
    const uint64_t blocks = grid_of(a, n_cus, v.blocks_per_cu, a.n_tiles);
    if constexpr (R <= 4) {
        if (v.vecs == 4) return launch_fast<R, 4, true, true>(a, 0, a.n_tiles, blocks, s);
    }
    return launch_fast<R, 2, true, true>(a, 0, a.n_tiles, blocks, s);
}

template <int R>
hipError_t launch_r(const RsArgs& a, int n_cus, hipStream_t s, const RsVariant& var) {
    const uint64_t tile = rs_tile_bytes(var);
    if (a.aligned) {  // cut tiles run inside the fast kernel; no edge list
        const uint32_t tiles_per_obj = uint32_t((a.shard_size + tile - 1) / tile);
        const uint64_t n_tiles = uint64_t(tiles_per_obj) * a.n_obj;
        const uint64_t blocks = grid_of(a, n_cus, var.blocks_per_cu, n_tiles);
        hipError_t e = hipErrorInvalidValue;
        if (var.nt && var.load_nt && var.store_nt && var.group == 4 && var.min_waves == 0) {
            // The shipping geometries (rs_default_variant): V = 4 while the
            // accumulators fit (R <= 4), V = 2 beyond.
            if constexpr (R <= 4) {
                if (var.vecs == 4) return launch_fast<R, 4, true>(a, tiles_per_obj, n_tiles, blocks, s);
            }
            if (var.vecs == 2) return launch_fast<R, 2, true>(a, tiles_per_obj, n_tiles, blocks, s);
        }
#ifdef MXEC_LAB
        // Lab geometries (tools/kernel_lab, the MXEC_RS_* lab knobs).
        if (var.vecs == 1) e = var.nt ? launch_fast<R, 1, true>(a, tiles_per_obj, n_tiles, blocks, s)
                                      : launch_fast<R, 1, false>(a, tiles_per_obj, n_tiles, blocks, s);
        else if (R >= 3 && R <= 4 && var.vecs == 2 && var.nt && var.group == 8)  // 8-input steps
            e = launch_fast<R, 2, true, false, 1, true, 8>(a, tiles_per_obj, n_tiles, blocks, s);
        else if (var.vecs == 2 && !var.nt) e = launch_fast<R, 2, false>(a, tiles_per_obj, n_tiles, blocks, s);
        else if (R == 4 && var.vecs == 4 && var.nt && var.min_waves == 3)
            e = launch_fast<R, 4, true, false, R == 4 ? 3 : 1>(a, tiles_per_obj, n_tiles, blocks, s);
        else if (R <= 4 && var.vecs == 4 && var.nt && !var.load_nt)  // plain loads, nontemporal stores
            e = launch_fast<R, 4, true, false, 1, false>(a, tiles_per_obj, n_tiles, blocks, s);
        else if (R <= 4 && var.vecs == 4 && var.nt && !var.store_nt)  // nontemporal loads, plain stores
            e = launch_fast<R, 4, false, false, 1, true>(a, tiles_per_obj, n_tiles, blocks, s);
        else if (R <= 4 && var.vecs == 4 && !var.nt) e = launch_fast<R, 4, false>(a, tiles_per_obj, n_tiles, blocks, s);
#endif
        return e;
    }
    if (a.n_edge && a.edge_tile_bytes != tile) return hipErrorInvalidValue;  // list built for another tile
    if (a.n_edge) {
        const uint32_t steps = uint32_t(tile / kEdgeTile);
        const uint64_t n_steps = a.n_edge * steps;
        const uint64_t blocks = grid_of(a, n_cus, 8, n_steps);
        hipLaunchKernelGGL((rs_apply_edge<R>), dim3(uint32_t(blocks)), dim3(kThreads), 0, s,
                           a.in_ptrs, a.out_ptrs, a.in_len, a.out_len, a.coef, a.coef_off,
                           a.shard_size, a.k, a.r_total, a.row0, a.edge_list, steps, tile, a.aligned,
                           n_steps);
        return hipGetLastError();
    }
    return hipSuccess;
}

}  // namespace

uint64_t rs_tile_bytes(const RsVariant& v) { return uint64_t(kThreads) * 16 * uint64_t(v.vecs); }

// Default geometry, from tools/kernel_lab sweeps on MI355X (profiles/): four
// 16-byte vectors per lane with nontemporal loads/stores while the
// accumulators fit (R <= 4: <= 173 VGPRs, two waves per SIMD; compiled for
// three, 164 VGPRs, measured 1.2-1.6 % slower), two beyond that; 512
// workgroups per CU of grid-stride.  Round 1 swept 4-64 (16 beat 8 and 4,
// 32 level or +0.9 %); round 2 swept 32-4096 in one process per box: 256
// over 32 gains 1.5-4 % in the bench's object-major layout (north star
// +3.1 %, cfg 4 +2.3 %, cfg 2 +1.5 %, cfg 3 decode +4.1 %) and 3-5 % with
// data and parity apart, 512 another 0.4-2.1 % / 1-3 %; 1024-2048 gain more
// with data and parity apart (5-12 % over 32) but lose again in the
// object-major layout (profiles/r2_lab_rs_grid_*.jsonl).  Fewer tiles
// per workgroup keep the tiles in flight closer together: with few large
// grid-stride workgroups, resident ones run different iterations and the
// chip's active tiles spread over many windows of memory.  Chosen by the
// launch's total row count so every row group of a launch shares one tile
// size (and one edge list).
RsVariant rs_default_variant(uint32_t r_total) {
    RsVariant v;
    v.vecs = r_total <= 4 ? 4 : 2;
    v.nt = true;
    // R <= 2 (config 2, two-erasure decodes) gained another 0-2 % at 1024 in
    // every layout swept; R = 4 went either way (profiles/r2_lab_rs_grid_*).
    v.blocks_per_cu = r_total <= 2 ? 1024 : 512;
#ifdef MXEC_LAB
    // Lab knobs (read per launch; `make lab` builds only):
    // MXEC_RS_LOAD_NT=0 plain loads with the nontemporal stores (R <= 4);
    // MXEC_RS_STORE_NT=0 plain stores with the nontemporal loads (R <= 4);
    // MXEC_RS_G8=1 r = 3, 4 with V = 2 and eight inputs' loads per step;
    // MXEC_RS_BPC workgroups per CU of uniform launches.
    if (const char* e = getenv("MXEC_RS_LOAD_NT")) v.load_nt = std::strcmp(e, "0") != 0;
    if (const char* e = getenv("MXEC_RS_G8"))
        if (!std::strcmp(e, "1") && r_total >= 3 && r_total <= 4) {
            v.vecs = 2;
            v.group = 8;
        }
    if (const char* e = getenv("MXEC_RS_STORE_NT")) v.store_nt = std::strcmp(e, "0") != 0;
    if (const char* e = getenv("MXEC_RS_BPC")) {
        const int b = atoi(e);
        if (b > 0 && b <= 4096) v.blocks_per_cu = b;
    }
    // MXEC_RS_VECS = 1 | 2 | 4 (4 only for R <= 4): vectors per lane of
    // uniform launches (the tile is 4 KiB x V per shard).
    if (const char* e = getenv("MXEC_RS_VECS")) {
        const int vv = atoi(e);
        if (vv == 1 || vv == 2 || (vv == 4 && r_total <= 4)) v.vecs = vv;
    }
#endif
    return v;
}

// Grouped launches (mixed batches: many objects of a few tiles each) take the
// default geometry: config 5 measured 32 / 48 / 64 / 128 / 256 / 2048 /
// one tile per workgroup within ~1 %, V = 2 3-4 % slower
// (profiles/r2_rs_group_geometry.txt, r2_rs_grid_bench_ab.txt).
// MXEC_RS_GROUP_VECS (2 | 4) and MXEC_RS_GROUP_BPC override it in lab builds.
RsVariant rs_group_variant(uint32_t r) {
    RsVariant v = rs_default_variant(r);
    v.blocks_per_cu = 512;
#ifdef MXEC_LAB
    static const int env_v = [] {
        const char* e = getenv("MXEC_RS_GROUP_VECS");
        return e ? atoi(e) : 0;
    }();
    static const int env_b = [] {
        const char* e = getenv("MXEC_RS_GROUP_BPC");
        return e ? atoi(e) : 0;
    }();
    if (r <= 4 && (env_v == 2 || env_v == 4)) v.vecs = env_v;
    if (env_b > 0 && env_b <= 4096) v.blocks_per_cu = env_b;
#endif
    return v;
}

hipError_t launch_rs_apply_variant(const RsArgs& a, int n_cus, hipStream_t s, const RsVariant& v) {
    switch (a.r) {
        case 1: return launch_r<1>(a, n_cus, s, v);
        case 2: return launch_r<2>(a, n_cus, s, v);
        case 3: return launch_r<3>(a, n_cus, s, v);
        case 4: return launch_r<4>(a, n_cus, s, v);
        case 5: return launch_r<5>(a, n_cus, s, v);
        case 6: return launch_r<6>(a, n_cus, s, v);
        case 7: return launch_r<7>(a, n_cus, s, v);
        case 8: return launch_r<8>(a, n_cus, s, v);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_rs_apply(const RsArgs& a, int n_cus, hipStream_t s) {
    if (a.tiles && a.multi) {
        if (!a.aligned || a.row0 != 0) return hipErrorInvalidValue;
        if (a.n_tiles == 0) return hipSuccess;
        return launch_multi(a, n_cus, s);
    }
    if (a.tiles) {
        if (!a.aligned || a.row0 != 0 || a.r != a.r_total) return hipErrorInvalidValue;
        if (a.n_tiles == 0) return hipSuccess;
        switch (a.r) {
            case 1: return launch_grouped<1>(a, n_cus, s);
            case 2: return launch_grouped<2>(a, n_cus, s);
            case 3: return launch_grouped<3>(a, n_cus, s);
            case 4: return launch_grouped<4>(a, n_cus, s);
            case 5: return launch_grouped<5>(a, n_cus, s);
            case 6: return launch_grouped<6>(a, n_cus, s);
            case 7: return launch_grouped<7>(a, n_cus, s);
            case 8: return launch_grouped<8>(a, n_cus, s);
            default: return hipErrorInvalidValue;
        }
    }
    RsVariant v = rs_default_variant(a.r_total);
    if (a.blocks_per_cu) v.blocks_per_cu = int(a.blocks_per_cu);
    return launch_rs_apply_variant(a, n_cus, s, v);
}

}  // namespace mxec

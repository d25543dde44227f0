// hash_device.hpp — device helpers shared by the lane-per-message hash
// kernels (sha256_kernel.hip, digest_kernel.hip): gfx950 bit ops, SHA-256
// compression (FIPS 180-4), 64-byte block loads and padded tail words.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mxec {
namespace hashdev {

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}
// m ? a : b per bit, as one v_bitop3 (0xCA).  Written as (m & a) | (~m & b)
// the compiler proved the two halves disjoint and rewrote SHA-256's Ch into
// v_and + v_bitop3 feeding an add: 2 more VALU per round, 1541 -> 1413 per
// block in the lane-per-message loops (tools/isa_count.py).
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }
// gfx950 v_bitop3_b32: any 3-input bitwise function in one instruction.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

#define SHA_S0(a) xor3(rotr((a), 2), rotr((a), 13), rotr((a), 22))
#define SHA_S1(e) xor3(rotr((e), 6), rotr((e), 11), rotr((e), 25))
#define SHA_s0(x) xor3(rotr((x), 7), rotr((x), 18), ((x) >> 3))
#define SHA_s1(x) xor3(rotr((x), 17), rotr((x), 19), ((x) >> 10))

#define SHA_RND(a, b, c, d, e, f, g, h, kt, wt)                          \
    do {                                                                 \
        const uint32_t t1 = h + SHA_S1(e) + bsel(e, f, g) + (kt) + (wt); \
        const uint32_t t2 = SHA_S0(a) + maj(a, b, c);                    \
        d += t1;                                                         \
        h = t1 + t2;                                                     \
    } while (0)

#define SHA_W(t) \
    (w[(t) & 15] += SHA_s1(w[((t) - 2) & 15]) + w[((t) - 7) & 15] + SHA_s0(w[((t) - 15) & 15]))

#define SHA_8R(i, K0, K1, K2, K3, K4, K5, K6, K7, W0, W1, W2, W3, W4, W5, W6, W7) \
    SHA_RND(a, b, c, d, e, f, g, h, K0, W0);                                     \
    SHA_RND(h, a, b, c, d, e, f, g, K1, W1);                                     \
    SHA_RND(g, h, a, b, c, d, e, f, K2, W2);                                     \
    SHA_RND(f, g, h, a, b, c, d, e, K3, W3);                                     \
    SHA_RND(e, f, g, h, a, b, c, d, K4, W4);                                     \
    SHA_RND(d, e, f, g, h, a, b, c, K5, W5);                                     \
    SHA_RND(c, d, e, f, g, h, a, b, K6, W6);                                     \
    SHA_RND(b, c, d, e, f, g, h, a, K7, W7)

// One compression; w[] holds the 16 big-endian message words on entry.
__device__ __forceinline__ void compress(uint32_t (&st)[8], uint32_t (&w)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
    SHA_8R(0, 0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u,
           0x923f82a4u, 0xab1c5ed5u, w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]);
    SHA_8R(8, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
           0x9bdc06a7u, 0xc19bf174u, w[8], w[9], w[10], w[11], w[12], w[13], w[14], w[15]);
    SHA_8R(16, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau,
           0x5cb0a9dcu, 0x76f988dau, SHA_W(16), SHA_W(17), SHA_W(18), SHA_W(19), SHA_W(20),
           SHA_W(21), SHA_W(22), SHA_W(23));
    SHA_8R(24, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u,
           0x06ca6351u, 0x14292967u, SHA_W(24), SHA_W(25), SHA_W(26), SHA_W(27), SHA_W(28),
           SHA_W(29), SHA_W(30), SHA_W(31));
    SHA_8R(32, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu,
           0x81c2c92eu, 0x92722c85u, SHA_W(32), SHA_W(33), SHA_W(34), SHA_W(35), SHA_W(36),
           SHA_W(37), SHA_W(38), SHA_W(39));
    SHA_8R(40, 0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u,
           0xf40e3585u, 0x106aa070u, SHA_W(40), SHA_W(41), SHA_W(42), SHA_W(43), SHA_W(44),
           SHA_W(45), SHA_W(46), SHA_W(47));
    SHA_8R(48, 0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au,
           0x5b9cca4fu, 0x682e6ff3u, SHA_W(48), SHA_W(49), SHA_W(50), SHA_W(51), SHA_W(52),
           SHA_W(53), SHA_W(54), SHA_W(55));
    SHA_8R(56, 0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu,
           0xbef9a3f7u, 0xc67178f2u, SHA_W(56), SHA_W(57), SHA_W(58), SHA_W(59), SHA_W(60),
           SHA_W(61), SHA_W(62), SHA_W(63));
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(1)))* gvec;

// Global (not flat) loads: the message pointers come from a table, so HIP
// sees generic pointers; the cast keeps the loads on the vmcnt queue only.
__device__ __forceinline__ void load_block(const uint8_t* p, u32x4 (&blk)[4]) {
    gvec q = (gvec)(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) blk[i] = q[i];
}

__device__ __forceinline__ void block_words(const u32x4 (&blk)[4], uint32_t (&w)[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        w[4 * i + 0] = bswap(blk[i].x);
        w[4 * i + 1] = bswap(blk[i].y);
        w[4 * i + 2] = bswap(blk[i].z);
        w[4 * i + 3] = bswap(blk[i].w);
    }
}

// Word `wi` (0..31) of the padded tail: bytes p[0..rem) then 0x80, zeros and
// the 64-bit big-endian bit length at the end of block `nblk` (1 or 2).
__device__ __forceinline__ uint32_t tail_word(const uint8_t* p, uint32_t rem, int wi, int nblk,
                                              uint64_t bits) {
    uint32_t v = 0;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
        const uint32_t idx = uint32_t(wi) * 4 + bb;
        uint32_t byte = 0;
        if (idx < rem) byte = p[idx];
        else if (idx == rem) byte = 0x80;
        v = (v << 8) | byte;
    }
    const int last = nblk * 16 - 1;
    if (wi == last - 1) v = uint32_t(bits >> 32);
    if (wi == last) v = uint32_t(bits);
    return v;
}


}  // namespace hashdev
}  // namespace mxec

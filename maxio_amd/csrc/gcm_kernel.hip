// gcm_kernel.hip — encrypt-then-EC frames: AES-256-GCM over 64 KiB frames
// for gfx950 (src/storage/crypto.rs).
//
// Frame f = nonce(12) = prefix(4) || index (u64 LE) || ciphertext || tag(16)
// (crypto.rs:94-117, 426-432); every frame is an independent GCM message, so
// one workgroup (256 threads) owns one frame at a time (grid-stride).
//
// * AES-256 counter blocks: T-table rounds (Te0..Te3 in LDS, replicated per
//   bank, one v_perm per lookup address), round keys read uniformly (scalar
//   loads); lane l encrypts blocks l, l+256, ... so loads and stores stay
//   coalesced.
// * GHASH is linear: Y = sum_i X_i * H^(m-i) over the m blocks
//   (AAD, ciphertext, length).  Lane l folds its blocks by Horner with the
//   fixed multiplier H^256 (a 4-bit position table in LDS, 32 lookups per
//   block, no reduction step), then multiplies by its own H^(m - i_last)
//   once, and the workgroup XOR-reduces.  Tag = E(J0) ^ Y.
// GF(2^128) elements are 4 big-endian u32 words (word 0 = bytes 0..3), bit 0
// of the field element = MSB of byte 0 (SP 800-38D).
#include "kernels.hpp"

namespace mxec {
namespace {

typedef gcm_u32x4 u32x4;

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// One AES-256 block: in/out as big-endian column words; te(k, w, j) =
// Te_k[byte j of w] (byte 0 = least significant).
template <class TE>
__device__ __forceinline__ void aes_block(TE te, const uint32_t* __restrict__ rk, uint32_t& s0, uint32_t& s1,
                                          uint32_t& s2, uint32_t& s3) {
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        const uint32_t t0 = xor3(xor3(te(0, s0, 3), te(1, s1, 2), te(2, s2, 1)), te(3, s3, 0), rk[4 * r + 0]);
        const uint32_t t1 = xor3(xor3(te(0, s1, 3), te(1, s2, 2), te(2, s3, 1)), te(3, s0, 0), rk[4 * r + 1]);
        const uint32_t t2 = xor3(xor3(te(0, s2, 3), te(1, s3, 2), te(2, s0, 1)), te(3, s1, 0), rk[4 * r + 2]);
        const uint32_t t3 = xor3(xor3(te(0, s3, 3), te(1, s0, 2), te(2, s1, 1)), te(3, s2, 0), rk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    // Last round: SubBytes + ShiftRows, the S-box byte taken from the table
    // whose byte lane holds S[x] unmultiplied.
    const uint32_t* k = rk + 56;
    const uint32_t u0 = (te(2, s0, 3) & 0xFF000000u) ^ (te(3, s1, 2) & 0x00FF0000u) ^
                        (te(0, s2, 1) & 0x0000FF00u) ^ (te(1, s3, 0) & 0x000000FFu) ^ k[0];
    const uint32_t u1 = (te(2, s1, 3) & 0xFF000000u) ^ (te(3, s2, 2) & 0x00FF0000u) ^
                        (te(0, s3, 1) & 0x0000FF00u) ^ (te(1, s0, 0) & 0x000000FFu) ^ k[1];
    const uint32_t u2 = (te(2, s2, 3) & 0xFF000000u) ^ (te(3, s3, 2) & 0x00FF0000u) ^
                        (te(0, s0, 1) & 0x0000FF00u) ^ (te(1, s1, 0) & 0x000000FFu) ^ k[2];
    const uint32_t u3 = (te(2, s3, 3) & 0xFF000000u) ^ (te(3, s0, 2) & 0x00FF0000u) ^
                        (te(0, s1, 1) & 0x0000FF00u) ^ (te(1, s2, 0) & 0x000000FFu) ^ k[3];
    s0 = u0; s1 = u1; s2 = u2; s3 = u3;
}

// Rounds R0..13 and the last round of two independent blocks, round by
// round (each chain hides the other's LDS latency).
template <int R0, class TE>
__device__ __forceinline__ void aes_rounds2(TE te, const uint32_t* __restrict__ rk, uint32_t& s0, uint32_t& s1,
                                            uint32_t& s2, uint32_t& s3, uint32_t& q0, uint32_t& q1,
                                            uint32_t& q2, uint32_t& q3) {
#pragma unroll
    for (int r = R0; r < 14; ++r) {
        const uint32_t t0 = xor3(xor3(te(0, s0, 3), te(1, s1, 2), te(2, s2, 1)), te(3, s3, 0), rk[4 * r + 0]);
        const uint32_t t1 = xor3(xor3(te(0, s1, 3), te(1, s2, 2), te(2, s3, 1)), te(3, s0, 0), rk[4 * r + 1]);
        const uint32_t t2 = xor3(xor3(te(0, s2, 3), te(1, s3, 2), te(2, s0, 1)), te(3, s1, 0), rk[4 * r + 2]);
        const uint32_t t3 = xor3(xor3(te(0, s3, 3), te(1, s0, 2), te(2, s1, 1)), te(3, s2, 0), rk[4 * r + 3]);
        const uint32_t v0 = xor3(xor3(te(0, q0, 3), te(1, q1, 2), te(2, q2, 1)), te(3, q3, 0), rk[4 * r + 0]);
        const uint32_t v1 = xor3(xor3(te(0, q1, 3), te(1, q2, 2), te(2, q3, 1)), te(3, q0, 0), rk[4 * r + 1]);
        const uint32_t v2 = xor3(xor3(te(0, q2, 3), te(1, q3, 2), te(2, q0, 1)), te(3, q1, 0), rk[4 * r + 2]);
        const uint32_t v3 = xor3(xor3(te(0, q3, 3), te(1, q0, 2), te(2, q1, 1)), te(3, q2, 0), rk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
        q0 = v0; q1 = v1; q2 = v2; q3 = v3;
    }
    const uint32_t* k = rk + 56;
    auto last = [&](uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, uint32_t kw) {
        return (te(2, x0, 3) & 0xFF000000u) ^ (te(3, x1, 2) & 0x00FF0000u) ^
               (te(0, x2, 1) & 0x0000FF00u) ^ (te(1, x3, 0) & 0x000000FFu) ^ kw;
    };
    const uint32_t u0 = last(s0, s1, s2, s3, k[0]), u1 = last(s1, s2, s3, s0, k[1]);
    const uint32_t u2 = last(s2, s3, s0, s1, k[2]), u3 = last(s3, s0, s1, s2, k[3]);
    const uint32_t w0 = last(q0, q1, q2, q3, k[0]), w1 = last(q1, q2, q3, q0, k[1]);
    const uint32_t w2 = last(q2, q3, q0, q1, k[2]), w3 = last(q3, q0, q1, q2, k[3]);
    s0 = u0; s1 = u1; s2 = u2; s3 = u3;
    q0 = w0; q1 = w1; q2 = w2; q3 = w3;
}

// Two whole AES-256 blocks.
template <class TE>
__device__ __forceinline__ void aes_block2(TE te, const uint32_t* __restrict__ rk, uint32_t& s0, uint32_t& s1,
                                           uint32_t& s2, uint32_t& s3, uint32_t& q0, uint32_t& q1, uint32_t& q2,
                                           uint32_t& q3) {
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
    q0 ^= rk[0]; q1 ^= rk[1]; q2 ^= rk[2]; q3 ^= rk[3];
    aes_rounds2<1>(te, rk, s0, s1, s2, s3, q0, q1, q2, q3);
}

// Counter blocks nonce(12) || ctr with ctr < 2^16 (frames of at most 65534
// blocks): after the first AddRoundKey three state words and the high half
// of the fourth are the same for every block of the frame, so round 1 has
// two block-dependent lookups (counter bytes 0, 1) and round 2 eight; the
// rest of those rounds is per-frame constants (14 + 8 of the 224 lookups of
// a block saved).
struct CtrConst {
    uint32_t c0, c1, c2, c3;  // round-1 outputs without the counter terms
    uint32_t d0, d1, d2, d3;  // round-2 outputs' constant halves
};

template <class TE>
__device__ __forceinline__ CtrConst ctr_const(TE te, const uint32_t* __restrict__ rk, uint32_t n0, uint32_t n1,
                                              uint32_t n2) {
    const uint32_t a0 = n0 ^ rk[0], a1 = n1 ^ rk[1], a2 = n2 ^ rk[2], a3 = rk[3];  // a3: bytes 2, 3 only
    CtrConst c;
    c.c0 = xor3(xor3(te(0, a0, 3), te(1, a1, 2), te(2, a2, 1)), rk[4], 0u);
    c.c1 = xor3(xor3(te(0, a1, 3), te(1, a2, 2), te(3, a0, 0)), rk[5], 0u);
    c.c2 = xor3(xor3(te(0, a2, 3), te(1, a3, 2), te(2, a0, 1)), te(3, a1, 0), rk[6]);
    c.c3 = xor3(xor3(te(0, a3, 3), te(1, a0, 2), te(2, a1, 1)), te(3, a2, 0), rk[7]);
    c.d0 = xor3(te(2, c.c2, 1), te(3, c.c3, 0), rk[8]);
    c.d1 = xor3(te(1, c.c2, 2), te(2, c.c3, 1), rk[9]);
    c.d2 = xor3(te(0, c.c2, 3), te(1, c.c3, 2), rk[10]);
    c.d3 = xor3(te(0, c.c3, 3), te(3, c.c2, 0), rk[11]);
    return c;
}

// Keystream of counters x and y (< 2^16) into (s0..s3), (q0..q3).
template <class TE>
__device__ __forceinline__ void aes_ctr2(TE te, const uint32_t* __restrict__ rk, const CtrConst& c, uint32_t x,
                                         uint32_t y, uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3,
                                         uint32_t& q0, uint32_t& q1, uint32_t& q2, uint32_t& q3) {
    const uint32_t ax = x ^ rk[3], ay = y ^ rk[3];
    const uint32_t u0 = c.c0 ^ te(3, ax, 0), u1 = c.c1 ^ te(2, ax, 1);
    const uint32_t p0 = c.c0 ^ te(3, ay, 0), p1 = c.c1 ^ te(2, ay, 1);
    s0 = xor3(c.d0, te(0, u0, 3), te(1, u1, 2));
    s1 = xor3(c.d1, te(0, u1, 3), te(3, u0, 0));
    s2 = xor3(c.d2, te(2, u0, 1), te(3, u1, 0));
    s3 = xor3(c.d3, te(1, u0, 2), te(2, u1, 1));
    q0 = xor3(c.d0, te(0, p0, 3), te(1, p1, 2));
    q1 = xor3(c.d1, te(0, p1, 3), te(3, p0, 0));
    q2 = xor3(c.d2, te(2, p0, 1), te(3, p1, 0));
    q3 = xor3(c.d3, te(1, p0, 2), te(2, p1, 1));
    aes_rounds2<3>(te, rk, s0, s1, s2, s3, q0, q1, q2, q3);
}

// x * H^256 via the position table: sum over the 32 nibbles of x.
__device__ __forceinline__ u32x4 mul_htab(const u32x4 (*ht)[16], u32x4 x) {
    u32x4 z = {0u, 0u, 0u, 0u};
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int n = 0; n < 8; n += 2) {
            const u32x4 a = ht[8 * q + n][(w[q] >> (28 - 4 * n)) & 0xF];
            const u32x4 b = ht[8 * q + n + 1][(w[q] >> (24 - 4 * n)) & 0xF];
            z.x = xor3(z.x, a.x, b.x);
            z.y = xor3(z.y, a.y, b.y);
            z.z = xor3(z.z, a.z, b.z);
            z.w = xor3(z.w, a.w, b.w);
        }
    }
    return z;
}

// Generic x * y (SP 800-38D Algorithm 1), 128 steps, branch free.
__device__ __forceinline__ u32x4 mul_bitwise(u32x4 x, u32x4 y) {
    uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
    uint32_t v0 = y.x, v1 = y.y, v2 = y.z, v3 = y.w;
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t xw = w[q];
#pragma unroll 8
        for (int b = 0; b < 32; ++b) {
            const uint32_t m = uint32_t(int32_t(xw) >> 31);  // bit set -> all ones
            xw <<= 1;
            z0 ^= v0 & m; z1 ^= v1 & m; z2 ^= v2 & m; z3 ^= v3 & m;
            const uint32_t lsb = 0u - (v3 & 1u);
            v3 = __builtin_amdgcn_alignbit(v2, v3, 1);
            v2 = __builtin_amdgcn_alignbit(v1, v2, 1);
            v1 = __builtin_amdgcn_alignbit(v0, v1, 1);
            v0 = (v0 >> 1) ^ (0xE1000000u & lsb);
        }
    }
    return u32x4{z0, z1, z2, z3};
}

// Up to 16 bytes at p (n <= 16) as big-endian words, zero padded.
__device__ __forceinline__ u32x4 load_partial_be(const uint8_t* p, uint32_t n) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < n; ++i) w[i >> 2] |= uint32_t(p[i]) << (24 - 8 * (i & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void store_partial_be(uint8_t* p, u32x4 v, uint32_t n) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t i = 0; i < n; ++i) p[i] = uint8_t(w[i >> 2] >> (24 - 8 * (i & 3)));
}

// Word q of a big-endian block keeps its first n - 4q bytes (n < 16).
__device__ __forceinline__ uint32_t mask_be(uint32_t n, uint32_t q) {
    const int c = int(n) - 4 * int(q);
    return c >= 4 ? 0xFFFFFFFFu : c <= 0 ? 0u : ~(0xFFFFFFFFu >> (8 * c));
}

// 16 bytes at a 4-byte aligned address (frame payloads sit 12 bytes into a
// frame) as big-endian words.
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ u32x4 load16_be(const uint8_t* p) {
    const u32x4a4 v = *reinterpret_cast<const u32x4a4*>(p);
    return u32x4{bswap(v.x), bswap(v.y), bswap(v.z), bswap(v.w)};
}
__device__ __forceinline__ void store16_be(uint8_t* p, u32x4 v) {
    *reinterpret_cast<u32x4a4*>(p) = u32x4a4{bswap(v.x), bswap(v.y), bswap(v.z), bswap(v.w)};
}

// LDS: the four T-tables replicated 32 times, laid out so that a lookup's
// address is ONE v_perm_b32 of the state word and a per-lane constant:
//     byte offset = pair * 65536 + x * 256 + t * 128 + (lane % 32) * 4
// for table k = 2 * pair + t.  v_perm places byte j of the state word in
// bits 8..15 and copies bits 0..7 ((lane % 32) * 4) and 16..23 (pair) from
// the lane constant; t * 128 is the ds_read_b32 immediate.  ds_read_b32
// banks are (address / 4) mod 32 over lane groups {0-31}, {32-63}, so each
// group hits its 32 banks once whatever bytes it looks up (random T-table
// indices otherwise serialise on bank conflicts).  The extraction +
// lane-bank address was two VALU per lookup before (byte extract, shift-add).
// The tables occupy LDS bytes [0, 128 KiB) (the dynamic LDS block starts at
// address 0: the kernel has no static __shared__); then one H^256 table per
// frame group.
#ifndef GCM_GROUPS
#define GCM_GROUPS 4
#endif
constexpr uint32_t kTeCopies = 32;
constexpr uint32_t kGcmGroups = GCM_GROUPS;  // frames in flight per workgroup, 256 threads each
constexpr size_t kTeWords = 4 * 256 * kTeCopies;
// Per group: the 32 x 16 position table of H^256 (8 KiB).  Its entries
// [p][0] (nibble 0 times anything) are zero; the workgroup's cross-wave XOR
// reduction borrows [0..3][0] and puts the zeros back before the next frame,
// so four groups (1 024 threads, four waves per SIMD) fit in 160 KiB.
constexpr size_t kGcmLdsBytes = kTeWords * 4 + kGcmGroups * (32 * 16) * sizeof(u32x4);
static_assert(kGcmLdsBytes <= 160 * 1024, "GCM LDS image exceeds 160 KiB");

typedef const uint32_t __attribute__((address_space(3)))* lds_u32p;

template <bool kDecrypt>
__global__ __launch_bounds__(256 * kGcmGroups) void gcm_frames_kernel(GcmArgs a) {
    extern __shared__ uint32_t smem[];
    uint32_t* te = smem;
    // The lookup addresses assume the tables start at LDS address 0.
    if (size_t((lds_u32p)(smem)) != 0) __builtin_trap();
    u32x4* gbase = reinterpret_cast<u32x4*>(smem + kTeWords);
    const uint32_t g = threadIdx.x >> 8, lane = threadIdx.x & 255;
    u32x4 (*htab)[16] = reinterpret_cast<u32x4 (*)[16]>(gbase + g * (32 * 16));
    auto red = [htab](int q) -> u32x4& { return htab[q][0]; };  // the zero entries, borrowed
    // word t = pair << 14 | x << 6 | tsel << 5 | copy  ->  Te_{2 pair + tsel}[x]
    for (uint32_t t = threadIdx.x; t < kTeWords; t += blockDim.x)
        te[t] = a.te[((t >> 14) * 2 + ((t >> 5) & 1)) * 256 + ((t >> 6) & 255)];
    const uint32_t lb0 = (lane % kTeCopies) * 4, lb1 = lb0 | 0x10000u;
    auto lk = [lb0, lb1](int k, uint32_t w, int j) {
        // result bytes: [lb.b0, w.byte j, lb.b2, 0]; sel 4..7 = bytes of w,
        // 0..3 = bytes of lb, 12 = 0x00.
        const uint32_t addr =
            __builtin_amdgcn_perm(w, k < 2 ? lb0 : lb1, 0x0C020000u | (uint32_t(4 + j) << 8));
        return reinterpret_cast<lds_u32p>(size_t(addr))[(k & 1) * 32];
    };
    int64_t cur_key = -1;
    for (uint64_t f0 = uint64_t(blockIdx.x) * kGcmGroups; f0 < a.n_frames;
         f0 += uint64_t(gridDim.x) * kGcmGroups) {
        const uint64_t f = f0 + g;
        const bool live = f < a.n_frames;  // uniform within a frame group
        GcmFrame fr{};
        if (live) fr = a.frames[f];
        const GcmKey* key = a.keys + fr.key;
        __syncthreads();  // every group is done with its htab / red slots
        if (live && int64_t(fr.key) != cur_key) {  // a new object's H^256 table
            for (uint32_t t = lane; t < 32 * 16; t += 256) (&htab[0][0])[t] = key->htab[t / 16][t % 16];
            cur_key = fr.key;
        } else if (lane < 4) {
            htab[lane][0] = u32x4{0u, 0u, 0u, 0u};  // return the reduction slots
        }
        __syncthreads();
        const uint32_t* rk = key->rk;
        const uint32_t nb = (fr.len + 15) / 16, na = (fr.aad_len + 15) / 16;
        const uint32_t m = live ? na + nb + 1 : 0;
        // The 12-byte nonce: prefix || index (u64 LE).  Encrypt builds it and
        // writes the frame header; decrypt reads the stored one (crypto.rs:323).
        uint32_t n0 = 0, n1 = 0, n2 = 0;
        if (live) {
            if (kDecrypt) {
                const u32x4 h = load_partial_be(fr.hdr, 12);
                n0 = h.x; n1 = h.y; n2 = h.z;
            } else {
                n0 = fr.prefix_be;
                n1 = bswap(uint32_t(fr.index));
                n2 = bswap(uint32_t(fr.index >> 32));
            }
        }
        // J0 = nonce || 0^31 || 1; block j of the payload uses counter 2 + j.
        u32x4 acc = {0u, 0u, 0u, 0u};
        uint32_t last = 0;
        // One block of the GHASH sequence: AAD, payload (encrypted here) or
        // the length block.
        auto block = [&](uint32_t i) -> u32x4 {
            u32x4 x;
            if (i < na) {
                const uint32_t off = 16 * i, n = min(16u, fr.aad_len - off);
                x = load_partial_be(fr.aad + off, n);
            } else if (i < na + nb) {
                const uint32_t j = i - na, off = 16 * j, n = min(16u, fr.len - off);
                uint32_t s0 = n0, s1 = n1, s2 = n2, s3 = 2u + j;
#ifndef GCM_LAB_NO_AES
                aes_block(lk, rk, s0, s1, s2, s3);
#endif
                const u32x4 ks = {s0, s1, s2, s3};
                u32x4 in = n == 16 ? load16_be(fr.in + off) : load_partial_be(fr.in + off, n);
                u32x4 out = {in.x ^ ks.x, in.y ^ ks.y, in.z ^ ks.z, in.w ^ ks.w};
                if (n == 16) {
                    store16_be(fr.out + off, out);
                } else {
                    store_partial_be(fr.out + off, out, n);
                    // keystream bytes past n must not enter GHASH
                    out.x &= mask_be(n, 0); out.y &= mask_be(n, 1);
                    out.z &= mask_be(n, 2); out.w &= mask_be(n, 3);
                }
                x = kDecrypt ? in : out;  // GHASH runs over the ciphertext
            } else {
                const uint64_t abits = uint64_t(fr.aad_len) * 8, cbits = uint64_t(fr.len) * 8;
                x = u32x4{uint32_t(abits >> 32), uint32_t(abits), uint32_t(cbits >> 32), uint32_t(cbits)};
            }
            return x;
        };
        auto fold = [&](const u32x4& x) {
#ifndef GCM_LAB_NO_GHASH
            const u32x4 h = mul_htab(htab, acc);
#else
            const u32x4 h = acc;
#endif
            acc = u32x4{h.x ^ x.x, h.y ^ x.y, h.z ^ x.z, h.w ^ x.w};
        };
        const uint32_t full_end = na + fr.len / 16;  // blocks [na, full_end) are whole payload blocks
        uint32_t i = lane;
        if (i < na) {  // an AAD block first (lanes 0..na-1), then payload pairs
            fold(block(i));
            last = i;
            i += 256;
        }
        // Two whole payload blocks per step: their AES chains are independent,
        // so the scheduler interleaves them and each hides the other's LDS
        // latency; two loads / stores in flight.
        const bool short_ctr = nb <= 65534;  // every payload counter 2 + j < 2^16
        CtrConst cc{};
#ifndef GCM_LAB_NO_AES
        if (short_ctr) cc = ctr_const(lk, rk, n0, n1, n2);
#endif
        for (; i + 256 < full_end && i >= na; i += 512) {
            const uint32_t j0 = i - na, j1 = j0 + 256;
            const u32x4 in0 = load16_be(fr.in + 16 * j0), in1 = load16_be(fr.in + 16 * j1);
            uint32_t a0 = n0, a1 = n1, a2 = n2, a3 = 2u + j0;
            uint32_t b0 = n0, b1 = n1, b2 = n2, b3 = 2u + j1;
#ifndef GCM_LAB_NO_AES
            if (short_ctr) aes_ctr2(lk, rk, cc, 2u + j0, 2u + j1, a0, a1, a2, a3, b0, b1, b2, b3);
            else aes_block2(lk, rk, a0, a1, a2, a3, b0, b1, b2, b3);
#endif
            const u32x4 o0 = {in0.x ^ a0, in0.y ^ a1, in0.z ^ a2, in0.w ^ a3};
            const u32x4 o1 = {in1.x ^ b0, in1.y ^ b1, in1.z ^ b2, in1.w ^ b3};
            store16_be(fr.out + 16 * j0, o0);
            store16_be(fr.out + 16 * j1, o1);
            fold(kDecrypt ? in0 : o0);
            fold(kDecrypt ? in1 : o1);
            last = i + 256;
        }
        for (; i < m; i += 256) {
            fold(block(i));
            last = i;
        }
        if (lane < m) acc = mul_bitwise(acc, key->hpow[m - last - 1]);  // * H^(m - last)
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) {
            acc.x ^= __shfl_xor(acc.x, s);
            acc.y ^= __shfl_xor(acc.y, s);
            acc.z ^= __shfl_xor(acc.z, s);
            acc.w ^= __shfl_xor(acc.w, s);
        }
        // The reduction slots are H^256-table entries that slower waves of
        // this frame may still be reading in their folds: every wave of the
        // workgroup is past its folds before any slot is written.
        __syncthreads();
        if ((lane & 63) == 0) red(int(lane >> 6)) = acc;
        __syncthreads();
        if (live && lane == 0) {
            u32x4 y = red(0);
            for (int q = 1; q < 4; ++q) {
                const u32x4 rq = red(q);
                y = u32x4{y.x ^ rq.x, y.y ^ rq.y, y.z ^ rq.z, y.w ^ rq.w};
            }
            uint32_t s0 = n0, s1 = n1, s2 = n2, s3 = 1u;
            aes_block(lk, rk, s0, s1, s2, s3);
            const u32x4 tag = {s0 ^ y.x, s1 ^ y.y, s2 ^ y.z, s3 ^ y.w};
            if (kDecrypt) {
                // stored index (nonce bytes 4..11, LE) must be this frame's
                const uint64_t stored = uint64_t(bswap(n1)) | uint64_t(bswap(n2)) << 32;
                const u32x4 want = load_partial_be(fr.tag, 16);
                const bool ok = want.x == tag.x && want.y == tag.y && want.z == tag.z && want.w == tag.w;
                a.status[f] = stored != fr.index ? 2 : ok ? 0 : 1;
            } else {
                store_partial_be(fr.hdr, u32x4{n0, n1, n2, 0u}, 12);
                store_partial_be(fr.tag, tag, 16);
            }
        }
    }
}

}  // namespace

hipError_t launch_gcm_frames(const GcmArgs& a, bool decrypt, int n_cus, hipStream_t s) {
    if (a.n_frames == 0) return hipSuccess;
    // 128 KiB of T-tables + 8 KiB per frame group (160 KiB at four groups):
    // one workgroup (four frames, 16 waves) per CU.
    static const hipError_t attr = [] {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gcm_frames_kernel<true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(kGcmLdsBytes));
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gcm_frames_kernel<false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, int(kGcmLdsBytes));
        return e;
    }();
    if (attr != hipSuccess) return attr;
    const uint64_t groups = (a.n_frames + kGcmGroups - 1) / kGcmGroups;
    const uint64_t grid = std::min<uint64_t>(groups, uint64_t(n_cus));
    if (decrypt)
        hipLaunchKernelGGL(gcm_frames_kernel<true>, dim3(uint32_t(grid)), dim3(256 * kGcmGroups), kGcmLdsBytes, s, a);
    else
        hipLaunchKernelGGL(gcm_frames_kernel<false>, dim3(uint32_t(grid)), dim3(256 * kGcmGroups), kGcmLdsBytes, s, a);
    return hipGetLastError();
}

}  // namespace mxec

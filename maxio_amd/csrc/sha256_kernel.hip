// sha256_kernel.hip — batched SHA-256 (FIPS 180-4) for gfx950.
//
// Replaces Sha256::digest (sha2 0.10.9) at filesystem.rs:1070 (write_chunk),
// :1131 (parity shards) and chunk_reader.rs:108 / :184 (verify on read).
//
// SHA-256 of one message is a serial chain of 64-byte compressions, so the
// only parallelism is across messages: one lane per chunk.  A lane streams its
// own message 64 bytes at a time with four global_load_dwordx4, prefetching the
// next block while compressing the current one.  The 64 rounds are fully
// unrolled (K in literals), the schedule rolls through 16 VGPRs, rotates are
// v_alignbit_b32, Ch / Maj are v_bfi_b32.  Workgroups are one wave so the
// waves of a batch spread over all SIMDs; the kernel is VALU-latency bound per
// message (see DESIGN.md for the roofline), not HBM-bound.
#include "kernels.hpp"

namespace mxec {
namespace {

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
    return (m & a) | (~m & b);  // v_bfi_b32
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

#define SHA_S0(a) (rotr((a), 2) ^ rotr((a), 13) ^ rotr((a), 22))
#define SHA_S1(e) (rotr((e), 6) ^ rotr((e), 11) ^ rotr((e), 25))
#define SHA_s0(x) (rotr((x), 7) ^ rotr((x), 18) ^ ((x) >> 3))
#define SHA_s1(x) (rotr((x), 17) ^ rotr((x), 19) ^ ((x) >> 10))

#define SHA_RND(a, b, c, d, e, f, g, h, kt, wt)                          \
    do {                                                                 \
        const uint32_t t1 = h + SHA_S1(e) + bsel(e, f, g) + (kt) + (wt); \
        const uint32_t t2 = SHA_S0(a) + bsel((a) ^ (b), c, b);           \
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

__device__ __forceinline__ void load_block(const uint8_t* p, uint4 (&blk)[4]) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) blk[i] = q[i];
}

__device__ __forceinline__ void block_words(const uint4 (&blk)[4], uint32_t (&w)[16]) {
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

__global__ __launch_bounds__(64) void sha256_kernel(const uint8_t* const* __restrict__ ptrs,
                                                    const uint64_t* __restrict__ lens,
                                                    uint8_t* __restrict__ digests,
                                                    const uint8_t* __restrict__ expected,
                                                    const uint64_t* __restrict__ exp_idx,
                                                    uint8_t* __restrict__ ok, uint32_t n) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = ptrs[i];
    const uint64_t len = lens[i];
    const uint64_t nfull = len / 64;
    uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                      0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint32_t w[16];
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        uint4 cur[4], nxt[4];
        if (nfull) load_block(p, cur);
        for (uint64_t b = 0; b < nfull; ++b) {
            if (b + 1 < nfull) load_block(p + 64 * (b + 1), nxt);
            block_words(cur, w);
            compress(st, w);
#pragma unroll
            for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
        }
    } else {
        for (uint64_t b = 0; b < nfull; ++b) {
            const uint8_t* q = p + 64 * b;
#pragma unroll
            for (int t = 0; t < 16; ++t)
                w[t] = uint32_t(q[4 * t]) << 24 | uint32_t(q[4 * t + 1]) << 16 |
                       uint32_t(q[4 * t + 2]) << 8 | uint32_t(q[4 * t + 3]);
            compress(st, w);
        }
    }
    const uint32_t rem = uint32_t(len - nfull * 64);
    const uint8_t* tp = p + nfull * 64;
    const int nblk = (rem + 9 <= 64) ? 1 : 2;
    const uint64_t bits = len * 8;
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, t, nblk, bits);
    compress(st, w);
    if (nblk == 2) {
#pragma unroll
        for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, 16 + t, nblk, bits);
        compress(st, w);
    }
    bool match = true;
    const uint64_t ei = exp_idx ? exp_idx[i] : i;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const uint32_t be = bswap(st[t]);
        if (digests) reinterpret_cast<uint32_t*>(digests + 32 * uint64_t(i))[t] = be;
        if (expected) match &= reinterpret_cast<const uint32_t*>(expected + 32 * ei)[t] == be;
    }
    if (ok) ok[i] = match ? 1 : 0;
}

}  // namespace

hipError_t launch_sha256(const ShaArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const uint32_t blocks = (a.n + 63) / 64;
    hipLaunchKernelGGL(sha256_kernel, dim3(blocks), dim3(64), 0, s, a.ptrs, a.lens, a.digests,
                       a.expected, a.exp_idx, a.ok, a.n);
    return hipGetLastError();
}

}  // namespace mxec

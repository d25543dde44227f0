// digest_kernel.hip — PUT body digests for gfx950.
//
// filesystem.rs:700-725 feeds every body byte to an Md5 hasher (the ETag,
// :775) and, when the request names one, to a ChecksumHasher (:28-63):
// CRC32 (crc32fast), CRC32C (crc32c_append), SHA-1 or SHA-256.
//
// * MD5 / SHA-1 / SHA-256 are Merkle–Damgård chains: one lane per body, all
//   requested algorithms in ONE launch (blockIdx.y picks the algorithm) so
//   their serial chains run side by side on different SIMDs.
// * CRC32 / CRC32C are linear over GF(2), so a body splits into tiles that are
//   hashed independently and recombined with shift operators
//   (x^(8n) mod P).  crc_tiles_kernel streams 16-byte units at HBM rate with
//   LDS slicing tables; crc_finish_kernel folds the tile values of each body
//   and applies init / final xor.  See DESIGN.md §4 for the algebra.
#include "hash_device.hpp"
#include "kernels.hpp"

#include <cstdlib>

namespace mxec {
namespace {

using namespace hashdev;

__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t s) {
    return __builtin_amdgcn_alignbit(x, x, 32u - s);
}

// ---- MD5 (RFC 1321) ---------------------------------------------------------
// F = b ? c : d, G = d ? b : c, H = b ^ c ^ d, I = c ^ (b | ~d), each one
// v_bitop3 (operands b, c, d).
#define MD5_F(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA)
#define MD5_G(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0xE4)
#define MD5_H(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0x96)
#define MD5_I(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0x39)
#define MD5_STEP(FN, a, b, c, d, x, t, s) a = b + rotl(a + FN(b, c, d) + (x) + (t), s)

__device__ __forceinline__ void md5_compress(uint32_t (&st)[4], const uint32_t (&x)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    MD5_STEP(MD5_F, a, b, c, d, x[0], 0xd76aa478u, 7);
    MD5_STEP(MD5_F, d, a, b, c, x[1], 0xe8c7b756u, 12);
    MD5_STEP(MD5_F, c, d, a, b, x[2], 0x242070dbu, 17);
    MD5_STEP(MD5_F, b, c, d, a, x[3], 0xc1bdceeeu, 22);
    MD5_STEP(MD5_F, a, b, c, d, x[4], 0xf57c0fafu, 7);
    MD5_STEP(MD5_F, d, a, b, c, x[5], 0x4787c62au, 12);
    MD5_STEP(MD5_F, c, d, a, b, x[6], 0xa8304613u, 17);
    MD5_STEP(MD5_F, b, c, d, a, x[7], 0xfd469501u, 22);
    MD5_STEP(MD5_F, a, b, c, d, x[8], 0x698098d8u, 7);
    MD5_STEP(MD5_F, d, a, b, c, x[9], 0x8b44f7afu, 12);
    MD5_STEP(MD5_F, c, d, a, b, x[10], 0xffff5bb1u, 17);
    MD5_STEP(MD5_F, b, c, d, a, x[11], 0x895cd7beu, 22);
    MD5_STEP(MD5_F, a, b, c, d, x[12], 0x6b901122u, 7);
    MD5_STEP(MD5_F, d, a, b, c, x[13], 0xfd987193u, 12);
    MD5_STEP(MD5_F, c, d, a, b, x[14], 0xa679438eu, 17);
    MD5_STEP(MD5_F, b, c, d, a, x[15], 0x49b40821u, 22);
    MD5_STEP(MD5_G, a, b, c, d, x[1], 0xf61e2562u, 5);
    MD5_STEP(MD5_G, d, a, b, c, x[6], 0xc040b340u, 9);
    MD5_STEP(MD5_G, c, d, a, b, x[11], 0x265e5a51u, 14);
    MD5_STEP(MD5_G, b, c, d, a, x[0], 0xe9b6c7aau, 20);
    MD5_STEP(MD5_G, a, b, c, d, x[5], 0xd62f105du, 5);
    MD5_STEP(MD5_G, d, a, b, c, x[10], 0x02441453u, 9);
    MD5_STEP(MD5_G, c, d, a, b, x[15], 0xd8a1e681u, 14);
    MD5_STEP(MD5_G, b, c, d, a, x[4], 0xe7d3fbc8u, 20);
    MD5_STEP(MD5_G, a, b, c, d, x[9], 0x21e1cde6u, 5);
    MD5_STEP(MD5_G, d, a, b, c, x[14], 0xc33707d6u, 9);
    MD5_STEP(MD5_G, c, d, a, b, x[3], 0xf4d50d87u, 14);
    MD5_STEP(MD5_G, b, c, d, a, x[8], 0x455a14edu, 20);
    MD5_STEP(MD5_G, a, b, c, d, x[13], 0xa9e3e905u, 5);
    MD5_STEP(MD5_G, d, a, b, c, x[2], 0xfcefa3f8u, 9);
    MD5_STEP(MD5_G, c, d, a, b, x[7], 0x676f02d9u, 14);
    MD5_STEP(MD5_G, b, c, d, a, x[12], 0x8d2a4c8au, 20);
    MD5_STEP(MD5_H, a, b, c, d, x[5], 0xfffa3942u, 4);
    MD5_STEP(MD5_H, d, a, b, c, x[8], 0x8771f681u, 11);
    MD5_STEP(MD5_H, c, d, a, b, x[11], 0x6d9d6122u, 16);
    MD5_STEP(MD5_H, b, c, d, a, x[14], 0xfde5380cu, 23);
    MD5_STEP(MD5_H, a, b, c, d, x[1], 0xa4beea44u, 4);
    MD5_STEP(MD5_H, d, a, b, c, x[4], 0x4bdecfa9u, 11);
    MD5_STEP(MD5_H, c, d, a, b, x[7], 0xf6bb4b60u, 16);
    MD5_STEP(MD5_H, b, c, d, a, x[10], 0xbebfbc70u, 23);
    MD5_STEP(MD5_H, a, b, c, d, x[13], 0x289b7ec6u, 4);
    MD5_STEP(MD5_H, d, a, b, c, x[0], 0xeaa127fau, 11);
    MD5_STEP(MD5_H, c, d, a, b, x[3], 0xd4ef3085u, 16);
    MD5_STEP(MD5_H, b, c, d, a, x[6], 0x04881d05u, 23);
    MD5_STEP(MD5_H, a, b, c, d, x[9], 0xd9d4d039u, 4);
    MD5_STEP(MD5_H, d, a, b, c, x[12], 0xe6db99e5u, 11);
    MD5_STEP(MD5_H, c, d, a, b, x[15], 0x1fa27cf8u, 16);
    MD5_STEP(MD5_H, b, c, d, a, x[2], 0xc4ac5665u, 23);
    MD5_STEP(MD5_I, a, b, c, d, x[0], 0xf4292244u, 6);
    MD5_STEP(MD5_I, d, a, b, c, x[7], 0x432aff97u, 10);
    MD5_STEP(MD5_I, c, d, a, b, x[14], 0xab9423a7u, 15);
    MD5_STEP(MD5_I, b, c, d, a, x[5], 0xfc93a039u, 21);
    MD5_STEP(MD5_I, a, b, c, d, x[12], 0x655b59c3u, 6);
    MD5_STEP(MD5_I, d, a, b, c, x[3], 0x8f0ccc92u, 10);
    MD5_STEP(MD5_I, c, d, a, b, x[10], 0xffeff47du, 15);
    MD5_STEP(MD5_I, b, c, d, a, x[1], 0x85845dd1u, 21);
    MD5_STEP(MD5_I, a, b, c, d, x[8], 0x6fa87e4fu, 6);
    MD5_STEP(MD5_I, d, a, b, c, x[15], 0xfe2ce6e0u, 10);
    MD5_STEP(MD5_I, c, d, a, b, x[6], 0xa3014314u, 15);
    MD5_STEP(MD5_I, b, c, d, a, x[13], 0x4e0811a1u, 21);
    MD5_STEP(MD5_I, a, b, c, d, x[4], 0xf7537e82u, 6);
    MD5_STEP(MD5_I, d, a, b, c, x[11], 0xbd3af235u, 10);
    MD5_STEP(MD5_I, c, d, a, b, x[2], 0x2ad7d2bbu, 15);
    MD5_STEP(MD5_I, b, c, d, a, x[9], 0xeb86d391u, 21);
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

// ---- SHA-1 (FIPS 180-4 §6.1) ------------------------------------------------
#define SHA1_CH(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA)
#define SHA1_PAR(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0x96)
#define SHA1_MAJ(b, c, d) __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8)
#define SHA1_W(t)                                                                          \
    (w[(t) & 15] = rotl(__builtin_amdgcn_bitop3_b32(w[((t) - 3) & 15], w[((t) - 8) & 15],   \
                                                    w[((t) - 14) & 15], 0x96) ^             \
                            w[(t) & 15],                                                    \
                        1))
// One round with the five variables renamed instead of moved.
#define SHA1_RND(FN, K, a, b, c, d, e, wt)             \
    do {                                               \
        e += rotl(a, 5) + FN(b, c, d) + (K) + (wt);    \
        b = rotl(b, 30);                               \
    } while (0)
#define SHA1_5R(FN, K, t, W0, W1, W2, W3, W4) \
    SHA1_RND(FN, K, a, b, c, d, e, W0);      \
    SHA1_RND(FN, K, e, a, b, c, d, W1);      \
    SHA1_RND(FN, K, d, e, a, b, c, W2);      \
    SHA1_RND(FN, K, c, d, e, a, b, W3);      \
    SHA1_RND(FN, K, b, c, d, e, a, W4)

__device__ __forceinline__ void sha1_compress(uint32_t (&st)[5], uint32_t (&w)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
    SHA1_5R(SHA1_CH, 0x5a827999u, 0, w[0], w[1], w[2], w[3], w[4]);
    SHA1_5R(SHA1_CH, 0x5a827999u, 5, w[5], w[6], w[7], w[8], w[9]);
    SHA1_5R(SHA1_CH, 0x5a827999u, 10, w[10], w[11], w[12], w[13], w[14]);
    SHA1_5R(SHA1_CH, 0x5a827999u, 15, w[15], SHA1_W(16), SHA1_W(17), SHA1_W(18), SHA1_W(19));
    SHA1_5R(SHA1_PAR, 0x6ed9eba1u, 20, SHA1_W(20), SHA1_W(21), SHA1_W(22), SHA1_W(23), SHA1_W(24));
    SHA1_5R(SHA1_PAR, 0x6ed9eba1u, 25, SHA1_W(25), SHA1_W(26), SHA1_W(27), SHA1_W(28), SHA1_W(29));
    SHA1_5R(SHA1_PAR, 0x6ed9eba1u, 30, SHA1_W(30), SHA1_W(31), SHA1_W(32), SHA1_W(33), SHA1_W(34));
    SHA1_5R(SHA1_PAR, 0x6ed9eba1u, 35, SHA1_W(35), SHA1_W(36), SHA1_W(37), SHA1_W(38), SHA1_W(39));
    SHA1_5R(SHA1_MAJ, 0x8f1bbcdcu, 40, SHA1_W(40), SHA1_W(41), SHA1_W(42), SHA1_W(43), SHA1_W(44));
    SHA1_5R(SHA1_MAJ, 0x8f1bbcdcu, 45, SHA1_W(45), SHA1_W(46), SHA1_W(47), SHA1_W(48), SHA1_W(49));
    SHA1_5R(SHA1_MAJ, 0x8f1bbcdcu, 50, SHA1_W(50), SHA1_W(51), SHA1_W(52), SHA1_W(53), SHA1_W(54));
    SHA1_5R(SHA1_MAJ, 0x8f1bbcdcu, 55, SHA1_W(55), SHA1_W(56), SHA1_W(57), SHA1_W(58), SHA1_W(59));
    SHA1_5R(SHA1_PAR, 0xca62c1d6u, 60, SHA1_W(60), SHA1_W(61), SHA1_W(62), SHA1_W(63), SHA1_W(64));
    SHA1_5R(SHA1_PAR, 0xca62c1d6u, 65, SHA1_W(65), SHA1_W(66), SHA1_W(67), SHA1_W(68), SHA1_W(69));
    SHA1_5R(SHA1_PAR, 0xca62c1d6u, 70, SHA1_W(70), SHA1_W(71), SHA1_W(72), SHA1_W(73), SHA1_W(74));
    SHA1_5R(SHA1_PAR, 0xca62c1d6u, 75, SHA1_W(75), SHA1_W(76), SHA1_W(77), SHA1_W(78), SHA1_W(79));
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}

// Word `wi` (0..31) of an MD5 padded tail: little-endian words, 64-bit
// little-endian bit count in the last two words of block `nblk`.
__device__ __forceinline__ uint32_t tail_word_le(const uint8_t* p, uint32_t rem, int wi, int nblk,
                                                 uint64_t bits) {
    uint32_t v = 0;
#pragma unroll
    for (int bb = 3; bb >= 0; --bb) {
        const uint32_t idx = uint32_t(wi) * 4 + bb;
        uint32_t byte = 0;
        if (idx < rem) byte = p[idx];
        else if (idx == rem) byte = 0x80;
        v = (v << 8) | byte;
    }
    const int last = nblk * 16 - 1;
    if (wi == last - 1) v = uint32_t(bits);
    if (wi == last) v = uint32_t(bits >> 32);
    return v;
}

// Full 64-byte blocks of one message.  A lane's blocks are far from every
// other lane's (one body each), so each block is a separate HBM round trip of
// ~2 us while compressing it takes well under 1 us: keep kDepth blocks in
// flight in a register ring.  WORDS(blk, w) turns 4 x 16 B into 16 words.
constexpr int kDepth = 4;

template <class Compress, class Words>
__device__ __forceinline__ void hash_blocks(const uint8_t* p, uint64_t nfull, Compress compress, Words words) {
    uint32_t w[16];
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        if (nfull == 0) return;
        // Prefetch addresses are clamped to the last block instead of
        // branched on, so the compiler can count the loads in flight.
        const uint64_t last = nfull - 1;
        u32x4 ring[kDepth][4];
#pragma unroll
        for (int j = 0; j < kDepth; ++j) load_block(p + 64 * min(uint64_t(j), last), ring[j]);
        uint64_t b = 0;
        for (; b + kDepth <= nfull; b += kDepth) {
#pragma unroll
            for (int j = 0; j < kDepth; ++j) {
                words(ring[j], w);
                load_block(p + 64 * min(b + j + kDepth, last), ring[j]);
                compress(w);
            }
        }
#pragma unroll
        for (int j = 0; j < kDepth - 1; ++j) {
            if (b + j < nfull) {
                words(ring[j], w);
                compress(w);
            }
        }
    } else {
        for (uint64_t b = 0; b < nfull; ++b) {
            u32x4 blk[4];
            const uint8_t* q = p + 64 * b;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                uint32_t v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint8_t* r = q + 16 * t + 4 * u;
                    v[u] = uint32_t(r[0]) | uint32_t(r[1]) << 8 | uint32_t(r[2]) << 16 | uint32_t(r[3]) << 24;
                }
                blk[t] = u32x4{v[0], v[1], v[2], v[3]};
            }
            words(blk, w);
            compress(w);
        }
    }
}

__device__ __forceinline__ void words_le(const u32x4 (&blk)[4], uint32_t (&w)[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        w[4 * i + 0] = blk[i].x;
        w[4 * i + 1] = blk[i].y;
        w[4 * i + 2] = blk[i].z;
        w[4 * i + 3] = blk[i].w;
    }
}

// blockIdx.y indexes a.algs: which digest this block computes for its 64
// bodies.  Uniform per block, so there is no divergence between paths.
__global__ __launch_bounds__(64) void body_hash_kernel(BodyHashArgs a) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t alg = a.algs[blockIdx.y];
    const uint8_t* p = a.ptrs[i];
    const uint64_t len = a.lens[i];
    const uint64_t nfull = len / 64;
    const uint32_t rem = uint32_t(len - nfull * 64);
    const uint8_t* tp = p + nfull * 64;
    const int nblk = (rem + 9 <= 64) ? 1 : 2;
    const uint64_t bits = len * 8;
    uint8_t* out = a.out + uint64_t(i) * a.out_stride;
    uint32_t w[16];
    if (alg == kBodyMd5) {
        uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
        hash_blocks(p, nfull, [&](uint32_t (&x)[16]) { md5_compress(st, x); }, words_le);
        for (int blk = 0; blk < nblk; ++blk) {
#pragma unroll
            for (int t = 0; t < 16; ++t) w[t] = tail_word_le(tp, rem, 16 * blk + t, nblk, bits);
            md5_compress(st, w);
        }
        uint32_t* o = reinterpret_cast<uint32_t*>(out + a.off_md5);
#pragma unroll
        for (int t = 0; t < 4; ++t) o[t] = st[t];
    } else if (alg == kBodySha1) {
        uint32_t st[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
        hash_blocks(p, nfull, [&](uint32_t (&x)[16]) { sha1_compress(st, x); },
                    [](const u32x4(&blk)[4], uint32_t(&x)[16]) { block_words(blk, x); });
        for (int blk = 0; blk < nblk; ++blk) {
#pragma unroll
            for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, 16 * blk + t, nblk, bits);
            sha1_compress(st, w);
        }
        uint32_t* o = reinterpret_cast<uint32_t*>(out + a.off_sha1);
#pragma unroll
        for (int t = 0; t < 5; ++t) o[t] = bswap(st[t]);
    } else {
        uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                          0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
        hash_blocks(p, nfull, [&](uint32_t (&x)[16]) { compress(st, x); },
                    [](const u32x4(&blk)[4], uint32_t(&x)[16]) { block_words(blk, x); });
        for (int blk = 0; blk < nblk; ++blk) {
#pragma unroll
            for (int t = 0; t < 16; ++t) w[t] = tail_word(tp, rem, 16 * blk + t, nblk, bits);
            compress(st, w);
        }
        uint32_t* o = reinterpret_cast<uint32_t*>(out + a.off_sha256);
#pragma unroll
        for (int t = 0; t < 8; ++t) o[t] = bswap(st[t]);
    }
}

// ---- CRC32 / CRC32C ------------------------------------------------------------
//
// Raw CRC R(M) (register starts at 0, no final xor) is linear:
//   R(A || B) = shift(R(A), |B|) ^ R(B),   shift(v, n) = v * x^(8n) mod P,
// and leading zero bytes do not change it.  Standard CRC with running value v
// (crc32fast / crc32c_append): C(M) = R(M) ^ shift(~v, |M|) ^ 0xFFFFFFFF.
//
// Tiling: a body's bytes [floor16(p), floor16(p + len)) are 16-byte units
// (bytes before p masked to zero); the partial unit at the end (< 16 bytes) is
// the finisher's.  Units are right-aligned into tiles of kCrcRows rows x 256
// units (4 KiB per row, 128 KiB per tile); lane L of the workgroup owns unit L
// of every row, 4096 bytes apart, and folds
//   acc = shift(acc, 4096) ^ R(unit)
// with 20 LDS lookups (4 for the shift, 16 slicing lookups for the unit).
// At the tile end lane L's value is shifted by its distance to the tile end
// ((255 - L) * 16 bytes, a per-lane constant) and the 256 lanes are XORed.

constexpr int kCrcRows = 32;
constexpr int kCrcDepth = 4;  // rows in flight per lane

// Reflected-domain a * b mod P (zlib multmodp), fixed 32 iterations.
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b, uint32_t poly) {
    uint32_t p = 0;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) {
        p ^= b & (0u - (a >> 31));
        a <<= 1;
        b = (b >> 1) ^ (poly & (0u - (b & 1u)));
    }
    return p;
}

// LDS image of CrcTables: slice[16][256] then shift4k[4][256].
struct CrcLds {
    uint32_t slice[16][256];
    uint32_t shift4k[4][256];
};

__device__ __forceinline__ void lut4v(const uint32_t (*t)[256], uint32_t v, uint32_t* o) {
    o[0] = t[0][v & 0xFF];
    o[1] = t[1][(v >> 8) & 0xFF];
    o[2] = t[2][(v >> 16) & 0xFF];
    o[3] = t[3][v >> 24];
}

__device__ __forceinline__ uint32_t lut4(const uint32_t (*t)[256], uint32_t v) {
    return t[0][v & 0xFF] ^ t[1][(v >> 8) & 0xFF] ^ t[2][(v >> 16) & 0xFF] ^ t[3][v >> 24];
}

__global__ __launch_bounds__(256) void crc_tiles_kernel(CrcArgs a) {
    __shared__ CrcLds lds;
    __shared__ uint32_t part[4];
    const CrcTables* tb = a.tables;
    for (int t = threadIdx.x; t < 16 * 256; t += 256) (&lds.slice[0][0])[t] = (&tb->slice[0][0])[t];
    for (int t = threadIdx.x; t < 4 * 256; t += 256) (&lds.shift4k[0][0])[t] = (&tb->shift4k[0][0])[t];
    const uint32_t lane = threadIdx.x;
    const uint32_t klane = tb->lane_shift[lane];
    const uint32_t poly = tb->poly;
    __syncthreads();
    for (uint64_t tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
        const CrcBody bd = a.bodies[a.tile_body[tile]];  // host-built tile -> body map
        const uint64_t t_in = tile - bd.tile0;
        // Virtual unit index of row r, lane L: t_in * kCrcRows * 256 + r * 256 + L;
        // real unit = virtual - pad (pad = leading virtual zero units).
        const int64_t first = int64_t(t_in) * kCrcRows * 256 - int64_t(bd.pad_units);
        const int r0 = first < 0 ? int((-first) / 256) : 0;  // rows entirely in the padding
        // Row r0 is the only row that can hold padding units or the masked
        // head unit; every later row is entirely real data.
        auto load_first = [&](int r) {
            const int64_t u = first + int64_t(r) * 256 + lane;
            u32x4 v = {0u, 0u, 0u, 0u};
            if (u >= 0) {
                v = ((gvec)(bd.base))[u];
                if (u == 0 && bd.head_skip) {  // bytes before the body's start
                    const uint32_t sk = bd.head_skip;
                    uint32_t* ww = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t lo_b = 4 * q;
                        const uint32_t keep = sk >= lo_b + 4 ? 0u
                                              : sk <= lo_b   ? 0xFFFFFFFFu
                                                             : (0xFFFFFFFFu << (8 * (sk - lo_b)));
                        ww[q] &= keep;
                    }
                }
            }
            return v;
        };
        gvec row_base = (gvec)(bd.base) + (first + lane);  // unit of row 0 for this lane
        auto load_row = [&](int r) { return row_base[int64_t(r) * 256]; };
        auto fold = [&](uint32_t acc, const u32x4& v) {
            // slice[k] = T_(15-k): byte j of the unit is 15 - j bytes from its end.
            // 20 lookups folded by v_bitop3 XOR3s.
            uint32_t t[20];
            lut4v(lds.shift4k, acc, t);
            lut4v(&lds.slice[0], v.x, t + 4);
            lut4v(&lds.slice[4], v.y, t + 8);
            lut4v(&lds.slice[8], v.z, t + 12);
            lut4v(&lds.slice[12], v.w, t + 16);
            uint32_t u[7];
#pragma unroll
            for (int q = 0; q < 6; ++q) u[q] = xor3(t[3 * q], t[3 * q + 1], t[3 * q + 2]);
            u[6] = t[18] ^ t[19];
            return xor3(xor3(u[0], u[1], u[2]), xor3(u[3], u[4], u[5]), u[6]);
        };
        uint32_t acc = 0;
        if (first >= 0) {
            // Common case: every row real.  Fully unrolled so the ring slots
            // stay in fixed registers; row r + kCrcDepth is issued before row
            // r is folded, and the scheduler may not hoist row r's lookups
            // above that load (it would wait for the whole ring).
            u32x4 ring[kCrcDepth];
#pragma unroll
            for (int j = 0; j < kCrcDepth; ++j) ring[j] = load_row(j);
#pragma unroll
            for (int rr = 0; rr < kCrcRows; ++rr) {
                u32x4 v = ring[rr % kCrcDepth];
                if (rr + kCrcDepth < kCrcRows) ring[rr % kCrcDepth] = load_row(rr + kCrcDepth);
                __builtin_amdgcn_sched_barrier(0);
                if (rr == 0 && first == 0 && lane == 0 && bd.head_skip) {
                    const uint32_t sk = bd.head_skip;  // bytes before the body's start
                    uint32_t* ww = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t lo_b = 4 * q;
                        const uint32_t keep = sk >= lo_b + 4 ? 0u
                                              : sk <= lo_b   ? 0xFFFFFFFFu
                                                             : (0xFFFFFFFFu << (8 * (sk - lo_b)));
                        ww[q] &= keep;
                    }
                }
                acc = fold(acc, v);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
            // First tile of a body with leading padding rows: row by row.
            acc = fold(0u, load_first(r0));
            for (int r = r0 + 1; r < kCrcRows; ++r) acc = fold(acc, load_row(r));
        }
        acc = multmodp(klane, acc, poly);
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) acc ^= __shfl_xor(acc, s);
        if ((lane & 63) == 0) part[lane >> 6] = acc;
        __syncthreads();
        if (lane == 0) a.tile_crc[tile] = part[0] ^ part[1] ^ part[2] ^ part[3];
        __syncthreads();
    }
}

// One workgroup per body: fold its tiles, the tail bytes, init and xorout.
__global__ __launch_bounds__(256) void crc_finish_kernel(CrcArgs a) {
    __shared__ uint32_t red[4];
    const uint32_t body = blockIdx.x;
    if (body >= a.n_bodies) return;
    const CrcTables* tb = a.tables;
    const uint32_t poly = tb->poly;
    const CrcBody bd = a.bodies[body];
    const uint32_t lane = threadIdx.x;
    // Lane l folds tiles [l*q, min((l+1)*q, n)) then shifts by the tiles after.
    const uint64_t n = bd.n_tiles;
    const uint64_t q = (n + 255) / 256;
    const uint64_t t0 = uint64_t(lane) * q, t1 = t0 + q < n ? t0 + q : n;
    uint32_t acc = 0;
    for (uint64_t t = t0; t < t1; ++t) acc = lut4(tb->shift_tile, acc) ^ a.tile_crc[bd.tile0 + t];
    if (t0 < t1 && t1 < n) {
        // multiply by (x^(8*TILE))^(n - t1) via the squares in tile_pow.
        uint64_t e = n - t1;
        for (int j = 0; e; ++j, e >>= 1)
            if (e & 1) acc = multmodp(tb->tile_pow[j], acc, poly);
    }
    if (t0 >= t1) acc = 0;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) acc ^= __shfl_xor(acc, s);
    if ((lane & 63) == 0) red[lane >> 6] = acc;
    __syncthreads();
    if (lane != 0) return;
    uint32_t raw = red[0] ^ red[1] ^ red[2] ^ red[3];
    // Tail bytes [tail, tail + tail_len), byte at a time (< 16 of them).
    for (uint32_t t = 0; t < bd.tail_len; ++t) {
        const uint32_t b = bd.tail[t];
        raw = (raw >> 8) ^ tb->slice[15][(raw ^ b) & 0xFF];
    }
    // C = R ^ shift(~v, len) ^ 0xFFFFFFFF
    uint32_t init = ~bd.prev;
    for (uint64_t e = bd.len, j = 0; e; ++j, e >>= 1)
        if (e & 1) init = multmodp(tb->byte_pow[j], init, poly);
    *reinterpret_cast<uint32_t*>(a.out + uint64_t(body) * a.out_stride) = raw ^ init ^ 0xFFFFFFFFu;
}

}  // namespace

hipError_t launch_body_hash(const BodyHashArgs& a, uint32_t n_algs, hipStream_t s) {
    if (a.n == 0 || n_algs == 0) return hipSuccess;
    hipLaunchKernelGGL(body_hash_kernel, dim3((a.n + 63) / 64, n_algs), dim3(64), 0, s, a);
    return hipGetLastError();
}

uint64_t crc_tile_bytes() { return uint64_t(kCrcRows) * 256 * 16; }

hipError_t launch_crc(const CrcArgs& a, int n_cus, hipStream_t s) {
    if (a.n_bodies == 0) return hipSuccess;
    if (a.n_tiles) {
        // 128 workgroups per CU of grid-stride: 8 / 32 / 128 / 512 measured
        // 4.70 / 4.74 / 4.81 / 4.79 TB/s (profiles/r2_crc_grid_ab.txt; more,
        // shorter workgroups keep the tiles in flight together, as for RS).
#ifdef MXEC_LAB
        static const uint64_t bpc = [] {  // MXEC_CRC_BPC: lab override
            const char* e = getenv("MXEC_CRC_BPC");
            const long v = e ? atol(e) : 0;
            return v > 0 && v <= 4096 ? uint64_t(v) : uint64_t(128);
        }();
#else
        constexpr uint64_t bpc = 128;
#endif
        const uint64_t grid = std::min<uint64_t>(a.n_tiles, uint64_t(n_cus) * bpc);
        hipLaunchKernelGGL(crc_tiles_kernel, dim3(uint32_t(grid)), dim3(256), 0, s, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(crc_finish_kernel, dim3(a.n_bodies), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace mxec

/*
 * body_oracle.c — CPU restatement of the PUT body digests (TEST
 * INFRASTRUCTURE ONLY; see oracle.h).
 *
 * filesystem.rs:700-725 feeds every body byte to an Md5 hasher (the ETag,
 * :775) and, when the request names one, to a ChecksumHasher (:28-63):
 *   CRC32  = crc32fast 1.5.0 Hasher (IEEE 802.3, reflected poly 0xEDB88320,
 *            init/xorout 0xFFFFFFFF), finalize -> u32, to_be_bytes -> base64;
 *   CRC32C = crc32c 0.6.8 crc32c_append(v, data) (Castagnoli, reflected poly
 *            0x82F63B78; the running value is the finished CRC of the prefix);
 *   SHA1   = sha1 0.10.6 (FIPS 180-4);
 *   SHA256 = sha2 0.10.9 (orc_sha256 in sha256_oracle.c);
 *   MD5    = md-5 0.10.6 (RFC 1321).
 * The crates are not vendored under /root/reference; these are the published
 * algorithms.  Pinned by tests/test_oracle_body.py against Python hashlib /
 * zlib, the standard check values and the reference's own tests
 * (integration.rs:2943-2945 crc32fast::hash, :3050 crc32c::crc32c).
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

/* ---- CRC32 / CRC32C: bitwise reflected CRC ------------------------------- */

static uint32_t crc_reflected(uint32_t poly, uint32_t crc, const uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        crc ^= p[i];
        for (int b = 0; b < 8; ++b) crc = (crc >> 1) ^ (poly & (0u - (crc & 1u)));
    }
    return crc;
}

uint32_t orc_crc32(const uint8_t* p, size_t n) {
    return ~crc_reflected(0xEDB88320u, 0xFFFFFFFFu, p, n);
}

uint32_t orc_crc32c_append(uint32_t crc, const uint8_t* p, size_t n) {
    return ~crc_reflected(0x82F63B78u, ~crc, p, n);
}

/* ---- MD5 (RFC 1321) -------------------------------------------------------- */

static uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

static const uint32_t kMd5T[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
    0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
    0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
    0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
    0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
    0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
    0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
    0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};
static const int kMd5S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static void md5_block(uint32_t st[4], const uint8_t* blk) {
    uint32_t x[16];
    for (int i = 0; i < 16; ++i)
        x[i] = (uint32_t)blk[4 * i] | (uint32_t)blk[4 * i + 1] << 8 | (uint32_t)blk[4 * i + 2] << 16 |
               (uint32_t)blk[4 * i + 3] << 24;
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    for (int t = 0; t < 64; ++t) {
        uint32_t f;
        int g;
        if (t < 16) {
            f = (b & c) | (~b & d);
            g = t;
        } else if (t < 32) {
            f = (d & b) | (~d & c);
            g = (5 * t + 1) & 15;
        } else if (t < 48) {
            f = b ^ c ^ d;
            g = (3 * t + 5) & 15;
        } else {
            f = c ^ (b | ~d);
            g = (7 * t) & 15;
        }
        const uint32_t tmp = d;
        d = c;
        c = b;
        b = b + rotl32(a + f + kMd5T[t] + x[g], kMd5S[t]);
        a = tmp;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

void orc_md5(const uint8_t* p, size_t n, uint8_t out[16]) {
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    size_t full = n / 64;
    for (size_t i = 0; i < full; ++i) md5_block(st, p + 64 * i);
    uint8_t tail[128];
    const size_t rem = n - full * 64;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, p + full * 64, rem);
    tail[rem] = 0x80;
    const size_t tl = rem + 9 <= 64 ? 64 : 128;
    const uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; ++i) tail[tl - 8 + i] = (uint8_t)(bits >> (8 * i));
    md5_block(st, tail);
    if (tl == 128) md5_block(st, tail + 64);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(st[i] >> (8 * j));
}

/* ---- SHA-1 (FIPS 180-4 §6.1) ------------------------------------------------ */

static void sha1_block(uint32_t st[5], const uint8_t* blk) {
    uint32_t w[80];
    for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 | (uint32_t)blk[4 * i + 2] << 8 |
               (uint32_t)blk[4 * i + 3];
    for (int t = 16; t < 80; ++t) w[t] = rotl32(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
    for (int t = 0; t < 80; ++t) {
        uint32_t f, k;
        if (t < 20) {
            f = (b & c) | (~b & d);
            k = 0x5a827999u;
        } else if (t < 40) {
            f = b ^ c ^ d;
            k = 0x6ed9eba1u;
        } else if (t < 60) {
            f = (b & c) | (b & d) | (c & d);
            k = 0x8f1bbcdcu;
        } else {
            f = b ^ c ^ d;
            k = 0xca62c1d6u;
        }
        const uint32_t tmp = rotl32(a, 5) + f + e + k + w[t];
        e = d;
        d = c;
        c = rotl32(b, 30);
        b = a;
        a = tmp;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
}

void orc_sha1(const uint8_t* p, size_t n, uint8_t out[20]) {
    uint32_t st[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
    size_t full = n / 64;
    for (size_t i = 0; i < full; ++i) sha1_block(st, p + 64 * i);
    uint8_t tail[128];
    const size_t rem = n - full * 64;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, p + full * 64, rem);
    tail[rem] = 0x80;
    const size_t tl = rem + 9 <= 64 ? 64 : 128;
    const uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha1_block(st, tail);
    if (tl == 128) sha1_block(st, tail + 64);
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(st[i] >> (24 - 8 * j));
}

/* CRC32C with the SSE4.2 crc32 instruction (the crc32c crate's hardware path
 * on x86-64) — same value as orc_crc32c_append; used as the timed CPU
 * baseline, never as a checker of itself. */
__attribute__((target("sse4.2"))) uint32_t orc_crc32c_append_fast(uint32_t crc, const uint8_t* p, size_t n) {
    uint64_t c = ~crc;
    while (n && ((uintptr_t)p & 7)) {
        c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
        --n;
    }
    for (; n >= 8; n -= 8, p += 8) {
        uint64_t v;
        memcpy(&v, p, 8);
        c = __builtin_ia32_crc32di(c, v);
    }
    while (n--) c = __builtin_ia32_crc32qi((uint32_t)c, *p++);
    return ~(uint32_t)c;
}

/*
 * sha256_oracle.c — FIPS 180-4 SHA-256, restating sha2 0.10.9's
 * Sha256::digest (Cargo.lock:1778-1786) as used by MaxIO at
 * filesystem.rs:1070 (write_chunk), :1131 (parity) and chunk_reader.rs:108,184
 * (verify).  The reference stores hex::encode(digest) (lowercase) in the
 * manifest; hex formatting is done by callers.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  orc_sha256 is the portable
 * scalar restatement (the checker).  orc_sha256_fast uses the x86 SHA
 * extensions when present — the backend sha2 0.10 selects at run time through
 * cpufeatures — and is what bench.py's cpu_baseline times.
 */
#include "oracle.h"

#include <string.h>

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void compress(uint32_t st[8], const uint8_t* p) {
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
        w[t] = ((uint32_t)p[4 * t] << 24) | ((uint32_t)p[4 * t + 1] << 16) |
               ((uint32_t)p[4 * t + 2] << 8) | (uint32_t)p[4 * t + 3];
    for (int t = 16; t < 64; ++t) {
        uint32_t s0 = ROTR(w[t - 15], 7) ^ ROTR(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = ROTR(w[t - 2], 17) ^ ROTR(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
    for (int t = 0; t < 64; ++t) {
        uint32_t S1 = ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[t] + w[t];
        uint32_t S0 = ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22);
        uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + maj;
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

typedef void (*compress_fn)(uint32_t st[8], const uint8_t* p, size_t nblocks);

static void compress_blocks_scalar(uint32_t st[8], const uint8_t* p, size_t nblocks) {
    for (size_t i = 0; i < nblocks; ++i) compress(st, p + 64 * i);
}

/* Merkle-Damgard driver shared by both backends: full blocks, then the
 * 0x80 / zero / 64-bit big-endian bit-length padding (FIPS 180-4 5.1.1). */
static void sha256_drive(const uint8_t* data, size_t len, uint8_t out[32], compress_fn fn) {
    uint32_t st[8];
    memcpy(st, H0, sizeof st);
    size_t full = len / 64;
    if (full) fn(st, data, full);
    uint8_t tail[128];
    size_t rem = len - full * 64;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, data + full * 64, rem);
    tail[rem] = 0x80;
    size_t tail_blocks = (rem + 1 + 8 <= 64) ? 1 : 2;
    uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; ++i) tail[tail_blocks * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    fn(st, tail, tail_blocks);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

void orc_sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
    sha256_drive(data, len, out, compress_blocks_scalar);
}

#if defined(__x86_64__)
int orc_have_sha_ni(void) {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return 0;
    int sha = (b >> 29) & 1;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    int sse41 = (c >> 19) & 1, ssse3 = (c >> 9) & 1;
    return sha && sse41 && ssse3;
}

/* Standard SHA-NI block loop (Intel SHA extensions whitepaper pattern). */
__attribute__((target("sha,sse4.1,ssse3"))) static void compress_blocks_shani(
    uint32_t st[8], const uint8_t* p, size_t nblocks) {
    const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i TMP = _mm_loadu_si128((const __m128i*)&st[0]);
    __m128i STATE1 = _mm_loadu_si128((const __m128i*)&st[4]);
    TMP = _mm_shuffle_epi32(TMP, 0xB1);          /* CDAB */
    STATE1 = _mm_shuffle_epi32(STATE1, 0x1B);    /* EFGH */
    __m128i STATE0 = _mm_alignr_epi8(TMP, STATE1, 8); /* ABEF */
    STATE1 = _mm_blend_epi16(STATE1, TMP, 0xF0);      /* CDGH */
    const __m128i* Kv = (const __m128i*)K256;
    while (nblocks--) {
        __m128i ABEF_SAVE = STATE0, CDGH_SAVE = STATE1;
        __m128i MSG, MSG0, MSG1, MSG2, MSG3;
        MSG0 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 0)), MASK);
        MSG1 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16)), MASK);
        MSG2 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 32)), MASK);
        MSG3 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 48)), MASK);
        __m128i W[4] = {MSG0, MSG1, MSG2, MSG3};
        for (int r = 0; r < 16; ++r) {
            __m128i cur = W[r & 3];
            if (r >= 4) {
                /* W[r&3] currently holds words 4(r-4)..; extend schedule */
                __m128i w0 = W[r & 3], w1 = W[(r + 1) & 3], w2 = W[(r + 2) & 3], w3 = W[(r + 3) & 3];
                __m128i t = _mm_sha256msg1_epu32(w0, w1);
                t = _mm_add_epi32(t, _mm_alignr_epi8(w3, w2, 4));
                cur = _mm_sha256msg2_epu32(t, w3);
                W[r & 3] = cur;
            }
            MSG = _mm_add_epi32(cur, _mm_loadu_si128(&Kv[r]));
            STATE1 = _mm_sha256rnds2_epu32(STATE1, STATE0, MSG);
            MSG = _mm_shuffle_epi32(MSG, 0x0E);
            STATE0 = _mm_sha256rnds2_epu32(STATE0, STATE1, MSG);
        }
        STATE0 = _mm_add_epi32(STATE0, ABEF_SAVE);
        STATE1 = _mm_add_epi32(STATE1, CDGH_SAVE);
        p += 64;
    }
    TMP = _mm_shuffle_epi32(STATE0, 0x1B);          /* FEBA */
    STATE1 = _mm_shuffle_epi32(STATE1, 0xB1);       /* DCHG */
    STATE0 = _mm_blend_epi16(TMP, STATE1, 0xF0);    /* DCBA */
    STATE1 = _mm_alignr_epi8(STATE1, TMP, 8);       /* ABEF */
    _mm_storeu_si128((__m128i*)&st[0], STATE0);
    _mm_storeu_si128((__m128i*)&st[4], STATE1);
}

int orc_sha256_fast(const uint8_t* data, size_t len, uint8_t out[32]) {
    static int have = -1;
    if (have < 0) have = orc_have_sha_ni();
    sha256_drive(data, len, out, have ? compress_blocks_shani : compress_blocks_scalar);
    return have;
}
#else
int orc_have_sha_ni(void) { return 0; }
int orc_sha256_fast(const uint8_t* data, size_t len, uint8_t out[32]) {
    orc_sha256(data, len, out);
    return 0;
}
#endif

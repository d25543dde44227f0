/*
 * gcm_oracle.c — CPU restatement of MaxIO's encrypt-then-EC frames (TEST
 * INFRASTRUCTURE ONLY; see oracle.h).
 *
 * src/storage/crypto.rs:1-20, 45-47, 94-117, 426-432: plaintext is cut into
 * FRAME_CHUNK_SIZE (65536) byte frames; frame i is
 *     nonce(12) = prefix(4) || i (u64 little-endian)
 *     || AES-256-GCM ciphertext || tag(16)
 * with the frame's AAD from the caller's AadBuilder (filesystem.rs:112-163:
 * SHA-256(identity prefix || i as u64 LE), or empty for no_aad()).
 * aes-gcm 0.10.3 (Cargo.lock) = NIST SP 800-38D with a 96-bit IV:
 * J0 = IV || 0^31 || 1, data counters inc32 from J0 + 1, tag = E(J0) ^ GHASH.
 * AES-256 = FIPS-197.  Pinned by tests/test_oracle_gcm.py against OpenSSL's
 * EVP_aes_256_gcm (libcrypto via ctypes), FIPS-197 C.3 and the published GCM
 * test cases.
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

static const uint8_t kSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76, 0xca, 0x82,
    0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, 0xb7, 0xfd, 0x93, 0x26,
    0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15, 0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96,
    0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75, 0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0,
    0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84, 0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb,
    0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf, 0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f,
    0x50, 0x3c, 0x9f, 0xa8, 0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff,
    0xf3, 0xd2, 0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb, 0xe0, 0x32,
    0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79, 0xe7, 0xc8, 0x37, 0x6d,
    0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08, 0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6,
    0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a, 0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e,
    0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, 0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e,
    0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf, 0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f,
    0xb0, 0x54, 0xbb, 0x16};

static uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

/* FIPS-197 §5.2: 15 round keys of 16 bytes. */
void orc_aes256_expand(const uint8_t key[32], uint8_t rk[240]) {
    memcpy(rk, key, 32);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 8 == 0) {
            const uint8_t t0 = t[0];
            t[0] = (uint8_t)(kSbox[t[1]] ^ rcon);
            t[1] = kSbox[t[2]];
            t[2] = kSbox[t[3]];
            t[3] = kSbox[t0];
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            for (int j = 0; j < 4; ++j) t[j] = kSbox[t[j]];
        }
        for (int j = 0; j < 4; ++j) rk[4 * i + j] = (uint8_t)(rk[4 * (i - 8) + j] ^ t[j]);
    }
}

/* FIPS-197 §5.1 Cipher, byte-oriented. */
void orc_aes256_encrypt_block(const uint8_t rk[240], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= 14; ++r) {
        uint8_t t[16];
        for (int i = 0; i < 16; ++i) t[i] = kSbox[s[i]];
        /* ShiftRows: row j of column c comes from column c + j */
        for (int c = 0; c < 4; ++c)
            for (int j = 0; j < 4; ++j) s[4 * c + j] = t[4 * ((c + j) & 3) + j];
        if (r != 14) {
            for (int c = 0; c < 4; ++c) {
                uint8_t* col = s + 4 * c;
                const uint8_t a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3];
                const uint8_t all = a0 ^ a1 ^ a2 ^ a3;
                col[0] = (uint8_t)(a0 ^ all ^ xtime(a0 ^ a1));
                col[1] = (uint8_t)(a1 ^ all ^ xtime(a1 ^ a2));
                col[2] = (uint8_t)(a2 ^ all ^ xtime(a2 ^ a3));
                col[3] = (uint8_t)(a3 ^ all ^ xtime(a3 ^ a0));
            }
        }
        for (int i = 0; i < 16; ++i) s[i] ^= rk[16 * r + i];
    }
    memcpy(out, s, 16);
}

/* SP 800-38D Algorithm 1: X * Y in GF(2^128), bit 0 = MSB of byte 0. */
void orc_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16]) {
    uint8_t z[16] = {0}, v[16];
    memcpy(v, y, 16);
    for (int i = 0; i < 128; ++i) {
        if (x[i / 8] & (0x80 >> (i % 8)))
            for (int j = 0; j < 16; ++j) z[j] ^= v[j];
        const int lsb = v[15] & 1;
        for (int j = 15; j > 0; --j) v[j] = (uint8_t)((v[j] >> 1) | (v[j - 1] << 7));
        v[0] >>= 1;
        if (lsb) v[0] ^= 0xe1;
    }
    memcpy(out, z, 16);
}

static void ghash_blocks(const uint8_t h[16], uint8_t y[16], const uint8_t* p, size_t n) {
    for (size_t off = 0; off < n; off += 16) {
        uint8_t blk[16] = {0};
        memcpy(blk, p + off, n - off < 16 ? n - off : 16);
        for (int j = 0; j < 16; ++j) y[j] ^= blk[j];
        orc_gf128_mul(y, h, y);
    }
}

static void inc32(uint8_t ctr[16]) {
    for (int j = 15; j >= 12; --j)
        if (++ctr[j]) break;
}

/* GCM-AE / GCM-AD with a 96-bit IV (SP 800-38D §7.1-7.2). decrypt != 0:
 * `in` is ciphertext, GHASH runs over it, tag_io is compared. */
static int gcm(const uint8_t key[32], const uint8_t iv[12], const uint8_t* aad, size_t aad_len, const uint8_t* in,
               size_t len, uint8_t* out, uint8_t tag_io[16], int decrypt) {
    uint8_t rk[240], h[16] = {0}, j0[16], ctr[16], y[16] = {0};
    orc_aes256_expand(key, rk);
    orc_aes256_encrypt_block(rk, h, h);
    memcpy(j0, iv, 12);
    j0[12] = j0[13] = j0[14] = 0;
    j0[15] = 1;
    ghash_blocks(h, y, aad, aad_len);
    if (decrypt) ghash_blocks(h, y, in, len);
    memcpy(ctr, j0, 16);
    for (size_t off = 0; off < len; off += 16) {
        uint8_t ks[16];
        inc32(ctr);
        orc_aes256_encrypt_block(rk, ctr, ks);
        const size_t n = len - off < 16 ? len - off : 16;
        for (size_t j = 0; j < n; ++j) out[off + j] = (uint8_t)(in[off + j] ^ ks[j]);
    }
    if (!decrypt) ghash_blocks(h, y, out, len);
    uint8_t lb[16];
    const uint64_t abits = (uint64_t)aad_len * 8, cbits = (uint64_t)len * 8;
    for (int j = 0; j < 8; ++j) {
        lb[j] = (uint8_t)(abits >> (56 - 8 * j));
        lb[8 + j] = (uint8_t)(cbits >> (56 - 8 * j));
    }
    for (int j = 0; j < 16; ++j) y[j] ^= lb[j];
    orc_gf128_mul(y, h, y);
    uint8_t ekj0[16], tag[16];
    orc_aes256_encrypt_block(rk, j0, ekj0);
    for (int j = 0; j < 16; ++j) tag[j] = (uint8_t)(ekj0[j] ^ y[j]);
    if (!decrypt) {
        memcpy(tag_io, tag, 16);
        return ORC_OK;
    }
    int diff = 0;
    for (int j = 0; j < 16; ++j) diff |= tag[j] ^ tag_io[j];
    return diff ? ORC_E_AUTH : ORC_OK;
}

int orc_gcm_encrypt(const uint8_t key[32], const uint8_t iv[12], const uint8_t* aad, size_t aad_len,
                    const uint8_t* pt, size_t len, uint8_t* ct, uint8_t tag[16]) {
    return gcm(key, iv, aad, aad_len, pt, len, ct, tag, 0);
}

int orc_gcm_decrypt(const uint8_t key[32], const uint8_t iv[12], const uint8_t* aad, size_t aad_len,
                    const uint8_t* ct, size_t len, const uint8_t tag[16], uint8_t* pt) {
    uint8_t t[16];
    memcpy(t, tag, 16);
    return gcm(key, iv, aad, aad_len, ct, len, pt, t, 1);
}

/* FrameEncryptor over a whole buffer (crypto.rs:94-117, 426-432).  aad: NULL
 * or n_frames * aad_len bytes (frame f's AAD at aad + f * aad_len). */
int orc_frames_encrypt(const uint8_t key[32], const uint8_t prefix[4], uint64_t first_index, const uint8_t* aad,
                       size_t aad_len, size_t frame_size, const uint8_t* pt, size_t len, uint8_t* out) {
    size_t f = 0;
    for (size_t off = 0; off < len; off += frame_size, ++f) {
        const size_t n = len - off < frame_size ? len - off : frame_size;
        uint8_t* fr = out + f * (frame_size + 28);
        const uint64_t idx = first_index + f;
        memcpy(fr, prefix, 4);
        for (int j = 0; j < 8; ++j) fr[4 + j] = (uint8_t)(idx >> (8 * j));
        gcm(key, fr, aad ? aad + f * aad_len : NULL, aad ? aad_len : 0, pt + off, n, fr + 12, fr + 12 + n, 0);
    }
    return ORC_OK;
}

/* FrameDecryptor over a whole buffer (crypto.rs:323-375): index check, then
 * tag check; returns ORC_E_AUTH / ORC_E_FRAME_INDEX on the first bad frame. */
int orc_frames_decrypt(const uint8_t key[32], uint64_t first_index, const uint8_t* aad, size_t aad_len,
                       size_t frame_size, const uint8_t* frames, size_t plaintext_size, uint8_t* out) {
    size_t f = 0;
    for (size_t off = 0; off < plaintext_size; off += frame_size, ++f) {
        const size_t n = plaintext_size - off < frame_size ? plaintext_size - off : frame_size;
        const uint8_t* fr = frames + f * (frame_size + 28);
        uint64_t idx = 0;
        for (int j = 7; j >= 0; --j) idx = (idx << 8) | fr[4 + j];
        if (idx != first_index + f) return ORC_E_FRAME_INDEX;
        uint8_t t[16];
        memcpy(t, fr + 12 + n, 16);
        if (gcm(key, fr, aad ? aad + f * aad_len : NULL, aad ? aad_len : 0, fr + 12, n, out + off, t, 1))
            return ORC_E_AUTH;
    }
    return ORC_OK;
}

// gcm.cpp — encrypt-then-EC frames (include/maxio_ec.h mxec_frames_*):
// FrameEncryptor / FrameDecryptor of src/storage/crypto.rs over whole
// buffers, AES-256-GCM per 64 KiB frame on the GPU (gcm_kernel.hip).
//
// Host work per data key: AES-256 key expansion, H = E_K(0^128), H^1..H^256
// and the 4-bit position table of H^256 (all by table multiplies, ~30 us).
#include <array>
#include <cstring>
#include <string>

#include "../../include/maxio_ec.h"
#include "kernels.hpp"
#include "ops.hpp"

using namespace mxec;

namespace {

const uint8_t kSbox[256] = {
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

uint8_t xtime(uint8_t x) { return uint8_t((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
uint32_t rotr8(uint32_t x) { return (x >> 8) | (x << 24); }

// Te0[x] = (2S, S, S, 3S) big-endian; Te1..Te3 its byte rotations.
void build_te(uint32_t te[4][256]) {
    for (int x = 0; x < 256; ++x) {
        const uint8_t s = kSbox[x], s2 = xtime(s), s3 = uint8_t(s2 ^ s);
        te[0][x] = uint32_t(s2) << 24 | uint32_t(s) << 16 | uint32_t(s) << 8 | s3;
        for (int k = 1; k < 4; ++k) te[k][x] = rotr8(te[k - 1][x]);
    }
}

// FIPS-197 key expansion, words big-endian.
void expand_key(const uint8_t key[32], uint32_t rk[60]) {
    for (int i = 0; i < 8; ++i)
        rk[i] = uint32_t(key[4 * i]) << 24 | uint32_t(key[4 * i + 1]) << 16 | uint32_t(key[4 * i + 2]) << 8 |
                key[4 * i + 3];
    uint32_t rcon = 0x01000000u;
    for (int i = 8; i < 60; ++i) {
        uint32_t t = rk[i - 1];
        auto sub = [](uint32_t w) {
            return uint32_t(kSbox[w >> 24]) << 24 | uint32_t(kSbox[(w >> 16) & 0xFF]) << 16 |
                   uint32_t(kSbox[(w >> 8) & 0xFF]) << 8 | kSbox[w & 0xFF];
        };
        if (i % 8 == 0) {
            t = sub((t << 8) | (t >> 24)) ^ rcon;
            rcon = uint32_t(xtime(uint8_t(rcon >> 24))) << 24;
        } else if (i % 8 == 4) {
            t = sub(t);
        }
        rk[i] = rk[i - 8] ^ t;
    }
}

// Byte-oriented AES-256 block on the host (for H = E_K(0) only).
void aes_block_host(const uint32_t rk[60], uint8_t blk[16]) {
    uint8_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = uint8_t(blk[i] ^ (rk[i / 4] >> (24 - 8 * (i % 4))));
    for (int r = 1; r <= 14; ++r) {
        uint8_t t[16];
        for (int i = 0; i < 16; ++i) t[i] = kSbox[s[i]];
        for (int c = 0; c < 4; ++c)
            for (int j = 0; j < 4; ++j) s[4 * c + j] = t[4 * ((c + j) & 3) + j];
        if (r != 14)
            for (int c = 0; c < 4; ++c) {
                uint8_t* col = s + 4 * c;
                const uint8_t a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3], all = uint8_t(a0 ^ a1 ^ a2 ^ a3);
                col[0] = uint8_t(a0 ^ all ^ xtime(a0 ^ a1));
                col[1] = uint8_t(a1 ^ all ^ xtime(a1 ^ a2));
                col[2] = uint8_t(a2 ^ all ^ xtime(a2 ^ a3));
                col[3] = uint8_t(a3 ^ all ^ xtime(a3 ^ a0));
            }
        for (int i = 0; i < 16; ++i) s[i] ^= uint8_t(rk[4 * r + i / 4] >> (24 - 8 * (i % 4)));
    }
    std::memcpy(blk, s, 16);
}

using Blk = std::array<uint32_t, 4>;  // big-endian words, field bit 0 = MSB of word 0

// 4-bit position table of y: t[p][v] = (v at nibble p) * y.
void position_table(const Blk& y, Blk t[32][16]) {
    Blk basis[128];
    basis[0] = y;
    for (int k = 1; k < 128; ++k) {  // basis[k] = y * x^k: right shift with reduction
        Blk v = basis[k - 1];
        const uint32_t lsb = v[3] & 1u;
        v[3] = (v[3] >> 1) | (v[2] << 31);
        v[2] = (v[2] >> 1) | (v[1] << 31);
        v[1] = (v[1] >> 1) | (v[0] << 31);
        v[0] = (v[0] >> 1) ^ (lsb ? 0xE1000000u : 0u);
        basis[k] = v;
    }
    for (int p = 0; p < 32; ++p)
        for (int v = 0; v < 16; ++v) {
            Blk z{0, 0, 0, 0};
            for (int j = 0; j < 4; ++j)
                if (v & (8 >> j))
                    for (int q = 0; q < 4; ++q) z[q] ^= basis[4 * p + j][q];
            t[p][v] = z;
        }
}

Blk mul_table(const Blk t[32][16], const Blk& x) {
    Blk z{0, 0, 0, 0};
    for (int p = 0; p < 32; ++p) {
        const uint32_t v = (x[p / 8] >> (28 - 4 * (p % 8))) & 0xF;
        for (int q = 0; q < 4; ++q) z[q] ^= t[p][v][q];
    }
    return z;
}

void build_key(const uint8_t key[32], GcmKey& k) {
    expand_key(key, k.rk);
    uint8_t h8[16] = {0};
    aes_block_host(k.rk, h8);
    Blk h;
    for (int q = 0; q < 4; ++q)
        h[q] = uint32_t(h8[4 * q]) << 24 | uint32_t(h8[4 * q + 1]) << 16 | uint32_t(h8[4 * q + 2]) << 8 | h8[4 * q + 3];
    static thread_local Blk th[32][16];
    position_table(h, th);
    Blk p = h;
    for (int e = 0; e < 256; ++e) {
        for (int q = 0; q < 4; ++q) k.hpow[e][q] = p[q];
        if (e < 255) p = mul_table(th, p);
    }
    position_table(p, th);  // p = H^256
    for (int a = 0; a < 32; ++a)
        for (int v = 0; v < 16; ++v)
            for (int q = 0; q < 4; ++q) k.htab[a][v][q] = th[a][v][q];
}

int te_tables(Device& d, const uint32_t** out) {
    std::lock_guard<std::mutex> g(d.sums_mu);
    if (!d.aes_te.p) {
        uint32_t te[4][256];
        build_te(te);
        MXEC_TRY(d.aes_te.ensure(sizeof te));
        MXEC_HIP(hipMemcpy(d.aes_te.p, te, sizeof te, hipMemcpyHostToDevice));
    }
    *out = static_cast<const uint32_t*>(d.aes_te.p);
    return MXEC_OK;
}

uint64_t n_frames(uint64_t len, uint32_t fs) { return (len + fs - 1) / fs; }

struct Job {
    const uint8_t* key;
    uint32_t prefix_be;
    uint32_t frame_size;
    uint64_t first_index;
    const uint8_t* aad;  // device
    uint32_t aad_len;
    const uint8_t* in;   // device: plaintext (encrypt) / frames (decrypt)
    uint64_t len;        // plaintext bytes
    uint8_t* out;        // device: frames (encrypt) / plaintext (decrypt)
};

// One launch over every frame of every job; decrypt statuses per frame land
// in status_dev.
int run_frames(Device& d, Slot& slot, hipStream_t s, const std::vector<Job>& jobs, bool decrypt,
               int32_t* status_dev) {
    std::vector<GcmFrame> frames;
    std::vector<GcmKey> keys(jobs.size());
    for (size_t j = 0; j < jobs.size(); ++j) {
        const Job& jb = jobs[j];
        build_key(jb.key, keys[j]);
        const uint64_t nf = n_frames(jb.len, jb.frame_size);
        const uint64_t fl = uint64_t(jb.frame_size) + MXEC_FRAME_OVERHEAD;
        for (uint64_t f = 0; f < nf; ++f) {
            GcmFrame fr{};
            const uint64_t plen = std::min<uint64_t>(jb.frame_size, jb.len - f * jb.frame_size);
            uint8_t* frame = const_cast<uint8_t*>(decrypt ? jb.in : jb.out) + f * fl;
            fr.hdr = frame;
            fr.tag = frame + 12 + plen;
            if (decrypt) {
                fr.in = frame + 12;
                fr.out = jb.out + f * jb.frame_size;
            } else {
                fr.in = jb.in + f * jb.frame_size;
                fr.out = frame + 12;
            }
            fr.aad = jb.aad_len ? jb.aad + f * jb.aad_len : nullptr;
            fr.aad_len = jb.aad_len;
            fr.index = jb.first_index + f;
            fr.len = uint32_t(plen);
            fr.key = uint32_t(j);
            fr.prefix_be = jb.prefix_be;
            frames.push_back(fr);
        }
    }
    if (frames.empty()) return MXEC_OK;
    const uint32_t* te = nullptr;
    MXEC_TRY(te_tables(d, &te));
    DescWriter w(slot);
    const size_t o_keys = w.add(keys.size() * sizeof(GcmKey));
    const size_t o_fr = w.add(frames.size() * sizeof(GcmFrame));
    std::memcpy(w.data() + o_keys, keys.data(), keys.size() * sizeof(GcmKey));
    std::memcpy(w.data() + o_fr, frames.data(), frames.size() * sizeof(GcmFrame));
    char* dev = nullptr;
    MXEC_TRY(w.commit(s, &dev));
    MXEC_TRY(affinity_check(d, &slot, s, "gcm frames"));
    GcmArgs a{};
    a.te = te;
    a.keys = reinterpret_cast<const GcmKey*>(dev + o_keys);
    a.frames = reinterpret_cast<const GcmFrame*>(dev + o_fr);
    a.status = status_dev;
    a.n_frames = frames.size();
    MXEC_HIP(launch_gcm_frames(a, decrypt, d.n_cus, s));
    return w.finish(s);
}

uint32_t prefix_word(const uint8_t p[4]) {
    return uint32_t(p[0]) << 24 | uint32_t(p[1]) << 16 | uint32_t(p[2]) << 8 | p[3];
}

int check_frame_size(uint32_t fs) {
    if (fs == 0 || fs % 16) return set_error(MXEC_E_INVALID_ARG, "frame_size must be a positive multiple of 16");
    return MXEC_OK;
}

// First failing frame of a decrypt, with crypto.rs's messages (:330-360).
int frame_error(const int32_t* st, uint64_t nf, uint64_t first_index, const uint8_t* frames_host, uint32_t fs,
                uint64_t plain) {
    for (uint64_t f = 0; f < nf; ++f) {
        if (st[f] == 2) {
            uint64_t got = 0;
            if (frames_host) {
                const uint8_t* h = frames_host + f * (uint64_t(fs) + MXEC_FRAME_OVERHEAD) + 4;
                for (int j = 7; j >= 0; --j) got = (got << 8) | h[j];
            }
            return set_error(MXEC_E_INTEGRITY, "frame index mismatch: expected " + std::to_string(first_index + f) +
                                                   ", got " + std::to_string(got));
        }
        if (st[f]) return set_error(MXEC_E_INTEGRITY, "AES-GCM decryption failed: authentication error");
    }
    (void)plain;
    return MXEC_OK;
}

}  // namespace

extern "C" {

uint64_t mxec_frames_len(uint64_t plaintext_len, uint32_t frame_size) {
    if (frame_size == 0) return 0;
    return plaintext_len + MXEC_FRAME_OVERHEAD * n_frames(plaintext_len, frame_size);
}

int mxec_frames_encrypt(mxec_ctx* ctx, const uint8_t key[32], const uint8_t nonce_prefix[4], uint64_t first_index,
                        const uint8_t* aad, uint32_t aad_len, uint32_t frame_size, const uint8_t* pt, uint64_t len,
                        uint8_t* out, uint64_t out_cap, uint64_t* out_len) {
    return guarded([&] {
        if (!key || !nonce_prefix || !out_len || (len && (!pt || !out)) || (aad_len && !aad))
            return set_error(MXEC_E_INVALID_ARG, "null argument");
        MXEC_TRY(check_frame_size(frame_size));
        const uint64_t nf = n_frames(len, frame_size), total = mxec_frames_len(len, frame_size);
        *out_len = 0;
        if (total > out_cap) return set_error(MXEC_E_INVALID_ARG, "output buffer too small");
        if (len == 0) return MXEC_OK;  // empty plaintext: no frames (crypto.rs round_trip_empty)
        DevScope ds;
        MXEC_TRY(ds.open(ctx, -1));
        Slot& slot = *ds.slot;
        hipStream_t s = slot.stream;
        const uint64_t a_in = round_up(len, kSlotAlign), a_out = round_up(total, kSlotAlign);
        const uint64_t a_aad = round_up(uint64_t(aad_len) * nf, kSlotAlign);
        MXEC_TRY(slot.shards.ensure(a_in + a_out + a_aad));
        auto* base = static_cast<uint8_t*>(slot.shards.p);
        std::vector<UploadSeg> up{{0, pt, len}};
        if (aad_len) up.push_back({a_in + a_out, aad, uint64_t(aad_len) * nf});
        MXEC_TRY(upload_segments(slot, s, base, up));
        Job jb{key, prefix_word(nonce_prefix), frame_size, first_index, base + a_in + a_out, aad_len, base, len,
               base + a_in};
        MXEC_TRY(run_frames(*ds.d, slot, s, {jb}, false, nullptr));
        MXEC_TRY(download_segments(slot, s, base, {{a_in, out, total}}));
        *out_len = total;
        return MXEC_OK;
    });
}

int mxec_frames_decrypt(mxec_ctx* ctx, const uint8_t key[32], uint64_t first_index, const uint8_t* aad,
                        uint32_t aad_len, uint32_t frame_size, const uint8_t* frames, uint64_t frames_len,
                        uint64_t plaintext_size, uint8_t* out, uint64_t out_cap, uint64_t* out_len) {
    return guarded([&] {
        if (!key || !out_len || (plaintext_size && (!frames || !out)) || (aad_len && !aad))
            return set_error(MXEC_E_INVALID_ARG, "null argument");
        MXEC_TRY(check_frame_size(frame_size));
        *out_len = 0;
        const uint64_t nf = n_frames(plaintext_size, frame_size), need = mxec_frames_len(plaintext_size, frame_size);
        if (plaintext_size > out_cap) return set_error(MXEC_E_INVALID_ARG, "output buffer too small");
        if (frames_len < need) return set_error(MXEC_E_INTEGRITY, "truncated encrypted frame");
        if (plaintext_size == 0) return MXEC_OK;
        DevScope ds;
        MXEC_TRY(ds.open(ctx, -1));
        Slot& slot = *ds.slot;
        hipStream_t s = slot.stream;
        const uint64_t a_in = round_up(need, kSlotAlign), a_out = round_up(plaintext_size, kSlotAlign);
        const uint64_t a_aad = round_up(uint64_t(aad_len) * nf, kSlotAlign);
        MXEC_TRY(slot.shards.ensure(a_in + a_out + a_aad));
        MXEC_TRY(slot.digests.grow(nf * sizeof(int32_t)));
        auto* base = static_cast<uint8_t*>(slot.shards.p);
        std::vector<UploadSeg> up{{0, frames, need}};
        if (aad_len) up.push_back({a_in + a_out, aad, uint64_t(aad_len) * nf});
        MXEC_TRY(upload_segments(slot, s, base, up));
        Job jb{key, 0, frame_size, first_index, base + a_in + a_out, aad_len, base, plaintext_size, base + a_in};
        auto* st_dev = static_cast<int32_t*>(slot.digests.p);
        MXEC_TRY(run_frames(*ds.d, slot, s, {jb}, true, st_dev));
        MXEC_TRY(slot.hdig.grow(nf * sizeof(int32_t)));
        MXEC_HIP(hipMemcpyAsync(slot.hdig.p, st_dev, nf * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        MXEC_TRY(slot_wait(slot, s));
        MXEC_TRY(frame_error(static_cast<const int32_t*>(slot.hdig.p), nf, first_index, frames, frame_size,
                             plaintext_size));
        MXEC_TRY(download_segments(slot, s, base, {{a_in, out, plaintext_size}}));
        *out_len = plaintext_size;
        return MXEC_OK;
    });
}

int mxec_frames_encrypt_device(mxec_ctx* ctx, int dev, void* stream, const mxec_frames_job* jobs, uint64_t n_jobs) {
    return guarded([&] {
        if (n_jobs == 0) return MXEC_OK;
        if (!jobs) return set_error(MXEC_E_INVALID_ARG, "null argument");
        std::vector<Job> js;
        for (uint64_t j = 0; j < n_jobs; ++j) {
            const mxec_frames_job& q = jobs[j];
            if (!q.key || (q.len && (!q.in_dev || !q.out_dev)) || (q.aad_len && !q.aad_dev))
                return set_error(MXEC_E_INVALID_ARG, "null argument");
            MXEC_TRY(check_frame_size(q.frame_size));
            js.push_back(Job{q.key, prefix_word(q.nonce_prefix), q.frame_size, q.first_index, q.aad_dev, q.aad_len,
                             q.in_dev, q.len, q.out_dev});
        }
        DevScope ds;
        MXEC_TRY(ds.open(ctx, dev));
        return run_frames(*ds.d, *ds.slot, static_cast<hipStream_t>(stream), js, false, nullptr);
    });
}

int mxec_frames_decrypt_device(mxec_ctx* ctx, int dev, void* stream, const mxec_frames_job* jobs, uint64_t n_jobs,
                               int32_t* status_out) {
    return guarded([&] {
        if (n_jobs == 0) return MXEC_OK;
        if (!jobs || !status_out) return set_error(MXEC_E_INVALID_ARG, "null argument");
        std::vector<Job> js;
        std::vector<uint64_t> first(n_jobs + 1, 0);
        for (uint64_t j = 0; j < n_jobs; ++j) {
            const mxec_frames_job& q = jobs[j];
            if (!q.key || (q.len && (!q.in_dev || !q.out_dev)) || (q.aad_len && !q.aad_dev))
                return set_error(MXEC_E_INVALID_ARG, "null argument");
            MXEC_TRY(check_frame_size(q.frame_size));
            js.push_back(Job{q.key, 0, q.frame_size, q.first_index, q.aad_dev, q.aad_len, q.in_dev, q.len, q.out_dev});
            first[j + 1] = first[j] + n_frames(q.len, q.frame_size);
        }
        DevScope ds;
        MXEC_TRY(ds.open(ctx, dev));
        Slot& slot = *ds.slot;
        hipStream_t s = static_cast<hipStream_t>(stream);
        const uint64_t nf = first[n_jobs];
        MXEC_TRY(slot.digests.grow(std::max<uint64_t>(1, nf) * sizeof(int32_t)));
        auto* st_dev = static_cast<int32_t*>(slot.digests.p);
        MXEC_TRY(run_frames(*ds.d, slot, s, js, true, st_dev));
        MXEC_TRY(slot.hdig.grow(std::max<uint64_t>(1, nf) * sizeof(int32_t)));
        if (nf) MXEC_HIP(hipMemcpyAsync(slot.hdig.p, st_dev, nf * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        MXEC_TRY(slot_wait(slot, s));
        const auto* st = static_cast<const int32_t*>(slot.hdig.p);
        int rc = MXEC_OK;
        for (uint64_t j = 0; j < n_jobs; ++j) {
            status_out[j] = MXEC_OK;
            const int e = frame_error(st + first[j], first[j + 1] - first[j], jobs[j].first_index, nullptr,
                                      jobs[j].frame_size, jobs[j].len);
            if (e) {
                status_out[j] = e;
                if (rc == MXEC_OK) rc = e;
            }
        }
        return rc;
    });
}

int mxec_frame_aads(mxec_ctx* ctx, const uint8_t* prefix, uint32_t prefix_len, uint64_t first_index,
                    uint64_t n_frames_, uint8_t (*out)[32]) {
    return guarded([&] {
        if (n_frames_ == 0) return MXEC_OK;
        if ((prefix_len && !prefix) || !out) return set_error(MXEC_E_INVALID_ARG, "null argument");
        const size_t ml = size_t(prefix_len) + 8;
        std::vector<uint8_t> msgs(ml * n_frames_);
        std::vector<const uint8_t*> ptrs(n_frames_);
        std::vector<size_t> lens(n_frames_, ml);
        for (uint64_t f = 0; f < n_frames_; ++f) {
            uint8_t* m = &msgs[f * ml];
            if (prefix_len) std::memcpy(m, prefix, prefix_len);
            const uint64_t idx = first_index + f;
            for (int j = 0; j < 8; ++j) m[prefix_len + j] = uint8_t(idx >> (8 * j));
            ptrs[f] = m;
        }
        return mxec_sha256_batch(ctx, ptrs.data(), lens.data(), n_frames_, out);
    });
}

}  // extern "C"

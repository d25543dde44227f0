// sums.cpp — PUT body digests (include/maxio_ec.h mxec_body_sums_batch*).
//
// filesystem.rs:700-725 hashes every body byte with Md5 (the ETag, :775) and
// the optional ChecksumHasher (:28-63).  MD5 / SHA-1 / SHA-256 run one lane per
// body in a single launch; CRC32 / CRC32C run the tiled linear form
// (digest_kernel.hip) whose constants are built here.
#include <cstddef>
#include <cstring>

#include "../../include/maxio_ec.h"
#include "kernels.hpp"
#include "ops.hpp"

using namespace mxec;

namespace {

static_assert(sizeof(mxec_body_sums) == 76, "mxec_body_sums layout");
constexpr uint32_t kPolyCrc32 = 0xEDB88320u;   // crc32fast (IEEE 802.3, reflected)
constexpr uint32_t kPolyCrc32c = 0x82F63B78u;  // crc32c (Castagnoli, reflected)

// a * b mod P, reflected representation (bit 31 = x^0), as zlib's multmodp.
uint32_t multmodp(uint32_t a, uint32_t b, uint32_t poly) {
    uint32_t p = 0;
    for (int i = 0; i < 32; ++i) {
        if (a & 0x80000000u) p ^= b;
        a <<= 1;
        b = (b >> 1) ^ ((b & 1u) ? poly : 0u);
    }
    return p;
}

// x^(8n) mod P.
uint32_t x8n(uint64_t n, uint32_t poly) {
    uint32_t r = 0x80000000u;         // x^0
    uint32_t base = 0x80000000u >> 8;  // x^8
    for (; n; n >>= 1) {
        if (n & 1) r = multmodp(base, r, poly);
        base = multmodp(base, base, poly);
    }
    return r;
}

void build_tables(uint32_t poly, CrcTables& t) {
    std::memset(&t, 0, sizeof t);
    t.poly = poly;
    uint32_t t0[256];
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b;
        for (int i = 0; i < 8; ++i) c = (c >> 1) ^ ((c & 1u) ? poly : 0u);
        t0[b] = c;
    }
    for (int k = 0; k < 16; ++k) {
        const uint32_t sh = x8n(uint64_t(15 - k), poly);
        for (uint32_t b = 0; b < 256; ++b) t.slice[k][b] = multmodp(sh, t0[b], poly);
    }
    const uint32_t s4k = x8n(4096, poly), stile = x8n(crc_tile_bytes(), poly);
    for (int k = 0; k < 4; ++k)
        for (uint32_t b = 0; b < 256; ++b) {
            t.shift4k[k][b] = multmodp(s4k, b << (8 * k), poly);
            t.shift_tile[k][b] = multmodp(stile, b << (8 * k), poly);
        }
    for (int l = 0; l < 256; ++l) t.lane_shift[l] = x8n(uint64_t(16) * uint64_t(255 - l), poly);
    t.tile_pow[0] = stile;
    t.byte_pow[0] = x8n(1, poly);
    for (int j = 1; j < 64; ++j) {
        t.tile_pow[j] = multmodp(t.tile_pow[j - 1], t.tile_pow[j - 1], poly);
        t.byte_pow[j] = multmodp(t.byte_pow[j - 1], t.byte_pow[j - 1], poly);
    }
}

// Device copy of both table sets: [0] CRC32, [1] CRC32C.
int crc_tables(Device& d, const CrcTables** out) {
    std::lock_guard<std::mutex> g(d.sums_mu);
    if (!d.crc_tables.p) {
        std::vector<CrcTables> h(2);
        build_tables(kPolyCrc32, h[0]);
        build_tables(kPolyCrc32c, h[1]);
        MXEC_TRY(d.crc_tables.ensure(sizeof(CrcTables) * 2));
        MXEC_HIP(hipMemcpy(d.crc_tables.p, h.data(), sizeof(CrcTables) * 2, hipMemcpyHostToDevice));
    }
    *out = static_cast<const CrcTables*>(d.crc_tables.p);
    return MXEC_OK;
}

// Tiles of one body for the CRC kernels (see digest_kernel.hip).
CrcBody crc_body(const uint8_t* p, uint64_t len, uint64_t tile0) {
    CrcBody b{};
    const uintptr_t pa = reinterpret_cast<uintptr_t>(p);
    const uintptr_t base = pa & ~uintptr_t(15), end = pa + len, endu = end & ~uintptr_t(15);
    const uint64_t units = endu > base ? (endu - base) / 16 : 0;
    const uint64_t per_tile = crc_tile_bytes() / 16;
    b.base = reinterpret_cast<const uint8_t*>(base);
    b.len = len;
    b.tile0 = tile0;
    b.n_tiles = (units + per_tile - 1) / per_tile;
    b.pad_units = b.n_tiles * per_tile - units;
    b.head_skip = uint32_t(pa - base);
    const uintptr_t tail = units ? endu : pa;
    b.tail = reinterpret_cast<const uint8_t*>(tail);
    b.tail_len = uint32_t(end - tail);
    b.prev = 0;
    return b;
}

}  // namespace

namespace mxec {

// Body digests of n device-resident bodies into records of `stride` bytes
// (mxec_body_sums layout) at out_dev; everything is enqueued on `s`.
int run_body_sums(Device& d, Slot& slot, hipStream_t s, const std::vector<const uint8_t*>& ptrs,
                  const std::vector<uint64_t>& lens, uint32_t which, uint8_t* out_dev, uint64_t stride) {
    const size_t n = ptrs.size();
    if (n == 0 || which == 0) return MXEC_OK;
    if (n > 0xFFFFFFFFull) return set_error(MXEC_E_INVALID_ARG, "too many bodies");
    std::vector<uint32_t> algs;
    if (which & MXEC_SUM_MD5) algs.push_back(kBodyMd5);
    if (which & MXEC_SUM_SHA1) algs.push_back(kBodySha1);
    if (which & MXEC_SUM_SHA256) algs.push_back(kBodySha256);
    std::vector<int> polys;
    if (which & MXEC_SUM_CRC32) polys.push_back(0);
    if (which & MXEC_SUM_CRC32C) polys.push_back(1);

    DescWriter w(slot);
    const size_t o_ptr = w.add(n * sizeof(void*));
    const size_t o_len = w.add(n * sizeof(uint64_t));
    const size_t o_alg = w.add(std::max<size_t>(1, algs.size()) * sizeof(uint32_t));
    std::vector<CrcBody> bodies(n);
    uint64_t tiles = 0;
    for (size_t i = 0; i < n; ++i) {
        bodies[i] = crc_body(ptrs[i], lens[i], tiles);
        tiles += bodies[i].n_tiles;
    }
    size_t o_body = 0, o_tiles = 0, o_tb = 0;
    if (!polys.empty()) {
        o_body = w.add(n * sizeof(CrcBody));
        o_tiles = w.add(std::max<uint64_t>(1, tiles) * sizeof(uint32_t) * polys.size());
        o_tb = w.add(std::max<uint64_t>(1, tiles) * sizeof(uint32_t));
    }
    std::memcpy(w.data() + o_ptr, ptrs.data(), n * sizeof(void*));
    std::memcpy(w.data() + o_len, lens.data(), n * sizeof(uint64_t));
    if (!algs.empty()) std::memcpy(w.data() + o_alg, algs.data(), algs.size() * sizeof(uint32_t));
    if (!polys.empty()) {
        std::memcpy(w.data() + o_body, bodies.data(), n * sizeof(CrcBody));
        // tile -> body, so a workgroup finds its body with one load instead
        // of a search of dependent loads per tile.
        auto* tb = reinterpret_cast<uint32_t*>(w.data() + o_tb);
        for (size_t i = 0; i < n; ++i)
            for (uint64_t t = 0; t < bodies[i].n_tiles; ++t) tb[bodies[i].tile0 + t] = uint32_t(i);
    }
    MXEC_TRY(affinity_check(d, &slot, s, "run_body_sums"));
    char* dev = nullptr;
    MXEC_TRY(w.commit(s, &dev));
    if (!polys.empty()) {
        const CrcTables* tab = nullptr;
        MXEC_TRY(crc_tables(d, &tab));
        for (size_t q = 0; q < polys.size(); ++q) {
            CrcArgs a{};
            a.tables = tab + polys[q];
            a.bodies = reinterpret_cast<const CrcBody*>(dev + o_body);
            a.tile_body = reinterpret_cast<const uint32_t*>(dev + o_tb);
            a.tile_crc = reinterpret_cast<uint32_t*>(dev + o_tiles) + q * std::max<uint64_t>(1, tiles);
            a.out = out_dev + (polys[q] == 0 ? offsetof(mxec_body_sums, crc32) : offsetof(mxec_body_sums, crc32c));
            a.out_stride = stride;
            a.n_tiles = tiles;
            a.n_bodies = uint32_t(n);
            MXEC_HIP(launch_crc(a, d.n_cus, s));
        }
    }
    if (!algs.empty()) {
        BodyHashArgs h{};
        h.ptrs = reinterpret_cast<const uint8_t* const*>(dev + o_ptr);
        h.lens = reinterpret_cast<const uint64_t*>(dev + o_len);
        h.algs = reinterpret_cast<const uint32_t*>(dev + o_alg);
        h.out = out_dev;
        h.out_stride = stride;
        h.off_md5 = offsetof(mxec_body_sums, md5);
        h.off_sha1 = offsetof(mxec_body_sums, sha1);
        h.off_sha256 = offsetof(mxec_body_sums, sha256);
        h.n = uint32_t(n);
        MXEC_HIP(launch_body_hash(h, uint32_t(algs.size()), s));
    }
    return w.finish(s);
}

}  // namespace mxec

extern "C" {

int mxec_body_sums_batch_device(mxec_ctx* ctx, int dev, void* stream, const uint8_t* const* bodies_dev,
                          const uint64_t* lens, uint64_t n, uint32_t which, mxec_body_sums* out_dev) {
    return guarded([&] {
        if (n == 0 || which == 0) return MXEC_OK;
        if (!bodies_dev || !lens || !out_dev) return set_error(MXEC_E_INVALID_ARG, "null argument");
        if (which & ~uint32_t(0x1F)) return set_error(MXEC_E_INVALID_ARG, "unknown digest flag");
        for (uint64_t i = 0; i < n; ++i)
            if (!bodies_dev[i]) return set_error(MXEC_E_INVALID_ARG, "null body pointer " + std::to_string(i));
        DevScope ds;
        MXEC_TRY(ds.open(ctx, dev));
        std::vector<const uint8_t*> p(bodies_dev, bodies_dev + n);
        std::vector<uint64_t> l(lens, lens + n);
        return run_body_sums(*ds.d, *ds.slot, static_cast<hipStream_t>(stream), p, l, which,
                             reinterpret_cast<uint8_t*>(out_dev), sizeof(mxec_body_sums));
    });
}

int mxec_body_sums_batch(mxec_ctx* ctx, const uint8_t* const* bodies, const uint64_t* lens, uint64_t n,
                   uint32_t which, mxec_body_sums* out) {
    return guarded([&] {
        if (n == 0 || which == 0) return MXEC_OK;
        if (!bodies || !lens || !out) return set_error(MXEC_E_INVALID_ARG, "null argument");
        if (which & ~uint32_t(0x1F)) return set_error(MXEC_E_INVALID_ARG, "unknown digest flag");
        DevScope ds;
        MXEC_TRY(ds.open(ctx, -1));
        Slot& slot = *ds.slot;
        hipStream_t s = slot.stream;
        uint64_t total = 0;
        std::vector<uint64_t> off(n);
        for (uint64_t i = 0; i < n; ++i) {
            if (lens[i] && !bodies[i]) return set_error(MXEC_E_INVALID_ARG, "null body");
            off[i] = total;
            total += round_up(lens[i], kSlotAlign);
        }
        MXEC_TRY(slot.shards.ensure(std::max<uint64_t>(total, 1)));
        MXEC_TRY(slot.digests.grow(n * sizeof(mxec_body_sums)));
        auto* base = static_cast<uint8_t*>(slot.shards.p);
        std::vector<const uint8_t*> p(n);
        std::vector<uint64_t> l(lens, lens + n);
        std::vector<UploadSeg> up;
        for (uint64_t i = 0; i < n; ++i) {
            p[i] = base + off[i];
            if (lens[i]) up.push_back({off[i], bodies[i], lens[i]});
        }
        MXEC_TRY(upload_segments(slot, s, base, up));
        auto* rec = static_cast<uint8_t*>(slot.digests.p);
        MXEC_TRY(run_body_sums(*ds.d, slot, s, p, l, which, rec, sizeof(mxec_body_sums)));
        MXEC_TRY(slot.hdig.grow(n * sizeof(mxec_body_sums)));
        MXEC_HIP(hipMemcpyAsync(slot.hdig.p, rec, n * sizeof(mxec_body_sums), hipMemcpyDeviceToHost, s));
        MXEC_TRY(slot_wait(slot, s));
        const auto* h = static_cast<const mxec_body_sums*>(slot.hdig.p);
        for (uint64_t i = 0; i < n; ++i) {
            if (which & MXEC_SUM_MD5) std::memcpy(out[i].md5, h[i].md5, 16);
            if (which & MXEC_SUM_CRC32) out[i].crc32 = h[i].crc32;
            if (which & MXEC_SUM_CRC32C) out[i].crc32c = h[i].crc32c;
            if (which & MXEC_SUM_SHA1) std::memcpy(out[i].sha1, h[i].sha1, 20);
            if (which & MXEC_SUM_SHA256) std::memcpy(out[i].sha256, h[i].sha256, 32);
        }
        return MXEC_OK;
    });
}

}  // extern "C"

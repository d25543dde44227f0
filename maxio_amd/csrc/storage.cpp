// storage.cpp — the file-level chunked-EC functions of MaxIO's
// FilesystemStorage / VerifiedChunkReader, over the GPU encode / verify /
// reconstruct entry points:
//   write_chunk                  filesystem.rs:1062-1080
//   compute_and_write_parity     filesystem.rs:1084-1145
//   put_object_chunked (body)    filesystem.rs:686-773 (chunking + manifest)
//   VerifiedChunkReader          chunk_reader.rs:35-152 (+ ranges :52-82)
//   try_reconstruct_data_chunk   chunk_reader.rs:157-226
// On-disk contract (mod.rs:145-189): `{key}.ec/{index:06}` chunk files and
// manifest.json as serde_json::to_string_pretty writes ChunkManifest.
//
// Differences in *how*, not *what*: data digests of a whole body are computed
// in one GPU batch instead of chunk by chunk, parity is encoded from the body
// already in memory instead of re-reading the data chunk files (:1108-1113),
// and a GET verifies every chunk of the range in one batch.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <mutex>
#include <new>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/maxio_ec.h"
#include "manifest.hpp"
#include "ops.hpp"
#include "runtime.hpp"

namespace fs = std::filesystem;
using mxec::set_error;

namespace {

std::string hex32(const uint8_t* d) {
    static const char* k = "0123456789abcdef";
    std::string s(64, '0');
    for (int i = 0; i < 32; ++i) {
        s[size_t(2 * i)] = k[d[i] >> 4];
        s[size_t(2 * i + 1)] = k[d[i] & 15];
    }
    return s;
}

bool unhex32(const std::string& s, uint8_t* out) {
    if (s.size() != 64) return false;
    auto v = [](char c) -> int {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    };
    for (int i = 0; i < 32; ++i) {
        int hi = v(s[size_t(2 * i)]), lo = v(s[size_t(2 * i + 1)]);
        if (hi < 0 || lo < 0) return false;
        out[i] = uint8_t(hi << 4 | lo);
    }
    return true;
}

std::string chunk_name(uint32_t index) {
    char b[32];
    std::snprintf(b, sizeof b, "%06u", index);
    return b;
}

int write_file(const fs::path& p, const uint8_t* data, size_t len) {
    const int fd = ::open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return set_error(MXEC_E_IO, "IO error: cannot create " + p.string() + ": " + std::strerror(errno));
    size_t put = 0;
    while (put < len) {
        const ssize_t w = ::write(fd, data + put, len - put);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) break;
        put += size_t(w);
    }
    const bool ok = put == len;
    if (::close(fd) != 0 || !ok) return set_error(MXEC_E_IO, "IO error: write failed for " + p.string());
    return MXEC_OK;
}

// Byte buffers whose resize() leaves new bytes uninitialised: a chunk about
// to be overwritten by read(2) or a decode need not be zero-filled first.
//
// Large buffers come from a process-wide free list by power-of-two class: a
// GET allocates a chunk-sized buffer per shard, and fresh mmap'd memory costs
// a page fault per 4 KiB on first touch and a TLB shoot-down across every
// request thread on munmap -- with 64 request threads that took more host
// CPU than the data copies.  Pages past the requested size are never
// touched, so the rounding costs address space, not memory.
class BigPool {
public:
    static constexpr size_t kMin = size_t(256) << 10;
    static BigPool& get() {
        static BigPool* p = new BigPool;  // never destroyed: used from static destructors
        return *p;
    }
    static size_t cls(size_t n) {
        size_t c = kMin;
        while (c < n) c <<= 1;
        return c;
    }
    void* take(size_t c) {
        {
            std::lock_guard<std::mutex> g(mu_);
            auto it = free_.find(c);
            if (it != free_.end() && !it->second.empty()) {
                void* p = it->second.back();
                it->second.pop_back();
                cached_ -= c;
                return p;
            }
        }
        void* p = std::malloc(c);
        if (!p) throw std::bad_alloc();
        return p;
    }
    void give(void* p, size_t c) {
        {
            std::lock_guard<std::mutex> g(mu_);
            if (cached_ + c <= kCap) {
                free_[c].push_back(p);
                cached_ += c;
                return;
            }
        }
        std::free(p);
    }

private:
    static constexpr size_t kCap = size_t(2) << 30;  // bytes kept for reuse
    std::mutex mu_;
    std::map<size_t, std::vector<void*>> free_;
    size_t cached_ = 0;
};

template <class T>
struct NoInitAlloc : std::allocator<T> {
    using value_type = T;
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    T* allocate(size_t n) {
        const size_t b = n * sizeof(T);
        if (b < BigPool::kMin) return std::allocator<T>::allocate(n);
        return static_cast<T*>(BigPool::get().take(BigPool::cls(b)));
    }
    void deallocate(T* p, size_t n) {
        const size_t b = n * sizeof(T);
        if (b < BigPool::kMin) return std::allocator<T>::deallocate(p, n);
        BigPool::get().give(p, BigPool::cls(b));
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        if constexpr (sizeof...(A) == 0) ::new (static_cast<void*>(p)) U;
        else ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
using Bytes = std::vector<uint8_t, NoInitAlloc<uint8_t>>;

// std::fs::read: whole file or an io::Error.
template <class Vec>
int read_file(const fs::path& p, Vec& out) {
    const int fd = ::open(p.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return set_error(MXEC_E_IO, "IO error: " + p.string() + ": " + std::strerror(errno));
    struct stat st;
    if (::fstat(fd, &st) != 0) {
        const int e = errno;
        ::close(fd);
        return set_error(MXEC_E_IO, "IO error: " + p.string() + ": " + std::strerror(e));
    }
    out.resize(size_t(st.st_size));
    size_t got = 0;
    while (got < out.size()) {
        const ssize_t r = ::read(fd, out.data() + got, out.size() - got);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) break;
        got += size_t(r);
    }
    ::close(fd);
    if (got != out.size()) return set_error(MXEC_E_IO, "IO error: read failed for " + p.string());
    return MXEC_OK;
}

// read_file into a caller buffer of exactly `want` bytes; *size gets the
// file's size (when it differs, nothing is read and MXEC_OK is returned so
// the caller can report the mismatch like read_file + size check would).
int read_file_to(const fs::path& p, uint8_t* dst, uint64_t want, uint64_t* size) {
    const int fd = ::open(p.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return set_error(MXEC_E_IO, "IO error: " + p.string() + ": " + std::strerror(errno));
    struct stat st;
    if (::fstat(fd, &st) != 0) {
        const int e = errno;
        ::close(fd);
        return set_error(MXEC_E_IO, "IO error: " + p.string() + ": " + std::strerror(e));
    }
    *size = uint64_t(st.st_size);
    uint64_t got = 0;
    if (*size == want) {
        while (got < want) {
            const ssize_t r = ::read(fd, dst + got, size_t(want - got));
            if (r < 0 && errno == EINTR) continue;
            if (r <= 0) break;
            got += uint64_t(r);
        }
    }
    ::close(fd);
    if (*size == want && got != want) return set_error(MXEC_E_IO, "IO error: read failed for " + p.string());
    return MXEC_OK;
}

void fill_info(mxec_chunk_info* ci, uint32_t index, uint64_t size, const uint8_t* digest, uint8_t kind) {
    ci->index = index;
    ci->size = size;
    std::string h = hex32(digest);
    std::memcpy(ci->sha256, h.c_str(), 65);
    ci->kind = kind;
}

// ---- ChunkManifest JSON (manifest.cpp) ------------------------------------
using mxec::Manifest;
using mxec::manifest_json;

int read_manifest(const fs::path& ec_dir, Manifest& m) {
    std::vector<uint8_t> raw;
    MXEC_TRY(read_file(ec_dir / "manifest.json", raw));
    // fs::read_to_string fails with an I/O error (InvalidData) on bytes that
    // are not UTF-8; then serde_json::from_str (filesystem.rs:3164-3171).
    if (!mxec::utf8_valid(raw.data(), raw.size()))
        return set_error(MXEC_E_IO, "IO error: stream did not contain valid UTF-8");
    std::string s(raw.begin(), raw.end());
    std::string why;
    if (!mxec::parse_manifest(s, m, &why)) return set_error(MXEC_E_JSON, "JSON error: " + why);
    if (m.chunks.size() < m.chunk_count) return set_error(MXEC_E_JSON, "JSON error: manifest lists fewer chunks than chunk_count");
    return MXEC_OK;
}

// try_reconstruct_data_chunk over files: read every shard, verify against the
// manifest digest, reconstruct on the GPU, return chunks[t].size bytes for
// every requested target.  The reference runs this once per bad chunk, each
// time re-reading and re-verifying all k+m shards; one pass rebuilds every
// missing shard, so several bad chunks of a GET cost one decode.
int reconstruct_from_dir(mxec_ctx* ctx, const fs::path& dir, const Manifest& man,
                         const std::vector<uint32_t>& targets, std::vector<std::vector<uint8_t>*> outs) {
    const int k = int(man.chunk_count);
    const int m = man.has_parity ? int(man.parity_shards) : 0;
    const uint64_t shard = man.has_shard ? man.shard_size : man.chunk_size;
    int rc = mxec_rs_check(k, m);
    if (rc) return set_error(rc, std::string("RS init error: ") + mxec_strerror(rc));
    const int total = k + m;
    if (int(man.chunks.size()) < total) return set_error(MXEC_E_JSON, "JSON error: manifest lists fewer shards than k+m");
    std::vector<std::vector<uint8_t>> bufs(static_cast<size_t>(total));
    std::vector<uint8_t*> ptrs(static_cast<size_t>(total));
    std::vector<size_t> lens(static_cast<size_t>(total));
    std::vector<uint8_t> present(static_cast<size_t>(total), 0);
    std::vector<uint8_t> expected(size_t(total) * 32, 0);
    for (int i = 0; i < total; ++i) {
        const auto& ci = man.chunks[size_t(i)];
        std::vector<uint8_t> data;
        bool ok = read_file(dir / chunk_name(uint32_t(i)), data) == MXEC_OK;
        // The digest covers the whole file as written (:184); a file whose size
        // differs from the manifest's cannot match it, so it is an erasure up
        // front and is rebuilt at its full manifest length.
        const size_t want = size_t(i < k ? std::min<uint64_t>(ci.size, shard) : shard);
        ok = ok && data.size() == want;
        // A digest that does not parse can never match: the shard is an erasure.
        ok = ok && unhex32(ci.sha256, &expected[size_t(i) * 32]);
        // Vec::resize(shard_size) zero pads; the kernels read bytes past a
        // shard's length as zero, so the buffer holds only the real bytes.
        bufs[size_t(i)].assign(want, 0);
        if (ok) {
            std::memcpy(bufs[size_t(i)].data(), data.data(), data.size());
            lens[size_t(i)] = data.size();
            present[size_t(i)] = 1;
        } else {
            lens[size_t(i)] = want;
        }
        ptrs[size_t(i)] = bufs[size_t(i)].data();
    }
    // Present shards are hashed over their on-disk bytes; a shard whose file
    // is longer than shard_size fails its digest exactly as in the reference.
    int np = 0;
    rc = mxec_reconstruct(ctx, k, m, shard, ptrs.data(), lens.data(),
                          reinterpret_cast<const uint8_t(*)[32]>(expected.data()), present.data(), 0, &np);
    if (rc) return rc;
    for (size_t t = 0; t < targets.size(); ++t) {
        const uint32_t target = targets[t];
        const uint64_t real = std::min<uint64_t>(man.chunks[target].size, shard);
        outs[t]->assign(bufs[target].begin(), bufs[target].begin() + long(real));
    }
    return MXEC_OK;
}

}  // namespace

extern "C" {

int mxec_write_chunk(mxec_ctx* ctx, const char* ec_dir, uint32_t index, const uint8_t* data, size_t len,
                     mxec_chunk_info* out) {
    return mxec::guarded([&]() -> int {
        if (!ec_dir || !out || (len && !data)) return set_error(MXEC_E_INVALID_ARG, "null argument");
        uint8_t dig[1][32];
        const uint8_t* b = data ? data : reinterpret_cast<const uint8_t*>("");
        MXEC_TRY(mxec_sha256_batch(ctx, &b, &len, 1, dig));
        MXEC_TRY(write_file(fs::path(ec_dir) / chunk_name(index), data, len));
        fill_info(out, index, len, dig[0], 0);
        return MXEC_OK;
    });
}

int mxec_compute_and_write_parity(mxec_ctx* ctx, const char* ec_dir, uint64_t chunk_size,
                                  uint32_t parity_shards, const mxec_chunk_info* data_chunks, int k,
                                  mxec_chunk_info* parity_out) {
    return mxec::guarded([&]() -> int {
        if (!ec_dir || (k > 0 && !data_chunks) || !parity_out) return set_error(MXEC_E_INVALID_ARG, "null argument");
        const int m = int(parity_shards);
        MXEC_TRY([&] {
            if (k + m > 255)
                return set_error(MXEC_E_TOO_MANY_SHARDS_255,
                                 "too many shards: " + std::to_string(k) + " data + " + std::to_string(m) + " parity = " +
                                     std::to_string(k + m) + " > 255 (GF(2^8) limit). Increase --chunk-size");
            return MXEC_OK;
        }());
        const fs::path dir(ec_dir);
        std::vector<Bytes> data(static_cast<size_t>(k));
        std::vector<const uint8_t*> dp(static_cast<size_t>(k));
        std::vector<size_t> dl(static_cast<size_t>(k));
        for (int j = 0; j < k; ++j) {
            MXEC_TRY(read_file(dir / chunk_name(data_chunks[j].index), data[size_t(j)]));
            if (data[size_t(j)].size() > chunk_size) data[size_t(j)].resize(chunk_size);  // Vec::resize
            dp[size_t(j)] = data[size_t(j)].data();
            dl[size_t(j)] = data[size_t(j)].size();
        }
        // Parity buffers: the encode writes every byte (no zero-fill needed).
        std::vector<Bytes> parity(static_cast<size_t>(m > 0 ? m : 0));
        for (auto& b : parity) b.resize(chunk_size);
        std::vector<uint8_t*> pp(parity.size());
        for (size_t i = 0; i < parity.size(); ++i) pp[i] = parity[i].data();
        std::vector<uint8_t> dig(size_t(k + m) * 32);
        int rc = mxec_encode(ctx, k, m, chunk_size, dp.data(), dl.data(), pp.data(),
                             reinterpret_cast<uint8_t(*)[32]>(dig.data()));
        if (rc) return rc;
        for (int i = 0; i < m; ++i) {
            MXEC_TRY(write_file(dir / chunk_name(uint32_t(k + i)), pp[size_t(i)], chunk_size));
            fill_info(&parity_out[i], uint32_t(k + i), chunk_size, &dig[size_t(k + i) * 32], 1);
        }
        return MXEC_OK;
    });
}

}  // extern "C"

namespace {

// put_object_chunked's chunking, chunk files, parity and manifest for a
// buffered body (filesystem.rs:686-828).  plain_size >= 0 records
// manifest.plaintext_size: the encrypt-then-EC drivers chunk the frame
// stream and keep the plaintext length (:973-990, :1472-1486).
int put_chunked_buffer(mxec_ctx* ctx, const char* ec_dir, uint64_t chunk_size, uint32_t parity_shards,
                       const uint8_t* body, size_t len, int64_t plain_size) {
    if (!ec_dir || (len && !body)) return set_error(MXEC_E_INVALID_ARG, "null argument");
    if (chunk_size == 0) return set_error(MXEC_E_INVALID_ARG, "chunk_size must be > 0");
    const fs::path dir(ec_dir);
    std::error_code ec;
    fs::create_directories(dir, ec);
    if (ec) return set_error(MXEC_E_IO, "IO error: " + ec.message());
    // Chunking (:709-737): full chunk_size slices, final partial unpadded;
    // empty body -> one empty chunk (:740-743).
    std::vector<const uint8_t*> dp;
    std::vector<size_t> dl;
    for (size_t off = 0; off < len; off += chunk_size) {
        dp.push_back(body + off);
        dl.push_back(size_t(std::min<uint64_t>(chunk_size, len - off)));
    }
    static const uint8_t empty = 0;
    if (dp.empty()) {
        dp.push_back(&empty);
        dl.push_back(0);
    }
    const int k = int(dp.size());
    const bool has_parity = parity_shards > 0 && len > 0;  // :748
    const int m = has_parity ? int(parity_shards) : 0;
    Manifest man;
    man.version = has_parity ? 2 : 1;
    man.total_size = len;
    man.chunk_size = chunk_size;
    man.chunk_count = uint32_t(k);
    std::vector<uint8_t> dig(size_t(k + m) * 32);
    std::vector<Bytes> parity;
    if (has_parity) {
        // The reference writes the data chunks first (write_chunk), then
        // hits the k+m guard inside compute_and_write_parity.
        auto write_data = [&]() -> int {
            for (int j = 0; j < k; ++j) MXEC_TRY(write_file(dir / chunk_name(uint32_t(j)), dp[size_t(j)], dl[size_t(j)]));
            return MXEC_OK;
        };
        if (k + m > 255) {
            MXEC_TRY(write_data());
            return set_error(MXEC_E_TOO_MANY_SHARDS_255,
                             "too many shards: " + std::to_string(k) + " data + " + std::to_string(m) + " parity = " +
                                 std::to_string(k + m) + " > 255 (GF(2^8) limit). Increase --chunk-size");
        }
        // The data chunk files are written on a helper thread while the
        // device encodes and hashes (the ~30 ms SHA-256 chain of a 1 MiB
        // chunk hides the writes); a write error still wins over anything
        // the encode reports, as the reference writes them first.
        int wrc = MXEC_OK;
        std::string wmsg;
        std::thread writer([&] {
            try {
                wrc = write_data();
                if (wrc) wmsg = mxec::last_error();
            } catch (...) {
                wrc = MXEC_E_IO;
                wmsg = "IO error: data chunk write failed";
            }
        });
        struct Joiner {  // joined on every path, an exception included
            std::thread& t;
            ~Joiner() {
                if (t.joinable()) t.join();
            }
        } joiner{writer};
        parity.resize(size_t(m));  // the encode writes every byte
        for (auto& b : parity) b.resize(chunk_size);
        std::vector<uint8_t*> pp(static_cast<size_t>(m));
        for (int i = 0; i < m; ++i) pp[size_t(i)] = parity[size_t(i)].data();
        const int erc = mxec_encode(ctx, k, m, chunk_size, dp.data(), dl.data(), pp.data(),
                                    reinterpret_cast<uint8_t(*)[32]>(dig.data()));
        const std::string emsg = erc ? std::string(mxec::last_error()) : std::string();
        writer.join();
        if (wrc) return set_error(wrc, wmsg);
        if (erc) return set_error(erc, emsg);
        for (int i = 0; i < m; ++i)
            MXEC_TRY(write_file(dir / chunk_name(uint32_t(k + i)), pp[size_t(i)], chunk_size));
    } else {
        MXEC_TRY(mxec_sha256_batch(ctx, dp.data(), dl.data(), size_t(k), reinterpret_cast<uint8_t(*)[32]>(dig.data())));
        for (int j = 0; j < k; ++j) MXEC_TRY(write_file(dir / chunk_name(uint32_t(j)), dp[size_t(j)], dl[size_t(j)]));
    }
    for (int j = 0; j < k + m; ++j) {
        Manifest::Chunk c;
        c.index = uint32_t(j);
        c.size = j < k ? dl[size_t(j)] : chunk_size;
        c.sha256 = hex32(&dig[size_t(j) * 32]);
        c.kind = j < k ? 0 : 1;
        man.chunks.push_back(c);
    }
    if (has_parity) {
        man.has_parity = true;
        man.parity_shards = parity_shards;
        man.has_shard = true;
        man.shard_size = chunk_size;
    }
    if (plain_size >= 0) {
        man.has_plain = true;
        man.plaintext_size = uint64_t(plain_size);
    }
    const std::string js = manifest_json(man);
    return write_file(dir / "manifest.json", reinterpret_cast<const uint8_t*>(js.data()), js.size());
}

// AES-256-GCM frame stream of `pt` under `key` (crypto.rs FrameEncryptor,
// 64 KiB frames, first index 0), frame i's AAD = SHA-256(aad_prefix || i LE)
// (build_frame_aad, filesystem.rs:118-128).
int encrypt_frames(mxec_ctx* ctx, const uint8_t* key, const uint8_t* nonce_prefix, const uint8_t* aad_prefix,
                   uint32_t aad_prefix_len, const uint8_t* pt, uint64_t len, std::vector<uint8_t>& ct) {
    const uint64_t nf = (len + MXEC_FRAME_CHUNK_SIZE - 1) / MXEC_FRAME_CHUNK_SIZE;
    ct.assign(size_t(mxec_frames_len(len, MXEC_FRAME_CHUNK_SIZE)), 0);
    if (nf == 0) return MXEC_OK;
    std::vector<uint8_t> aads(size_t(nf) * 32);
    MXEC_TRY(mxec_frame_aads(ctx, aad_prefix, aad_prefix_len, 0, nf, reinterpret_cast<uint8_t(*)[32]>(aads.data())));
    uint64_t n = 0;
    MXEC_TRY(mxec_frames_encrypt(ctx, key, nonce_prefix, 0, aads.data(), 32, MXEC_FRAME_CHUNK_SIZE, pt, len,
                                 ct.data(), ct.size(), &n));
    ct.resize(size_t(n));
    return MXEC_OK;
}

// The parts of a multipart upload concatenated in order (plaintext).  An
// encrypted part is a frame stream under the upload key with AADs
// SHA-256("PART" 0 upload_id 0 part_number_le4 0 || i LE) (part_aad_builder,
// filesystem.rs:147-163), decrypted by FrameDecryptor (:1378-1388).
int read_parts(mxec_ctx* ctx, const mxec_multipart_part* parts, uint32_t n_parts, const uint8_t* upload_key,
               const char* upload_id, std::vector<uint8_t>& out) {
    out.clear();
    for (uint32_t p = 0; p < n_parts; ++p) {
        const mxec_multipart_part& part = parts[p];
        if (!part.path) return set_error(MXEC_E_INVALID_ARG, "null part path");
        std::vector<uint8_t> raw;
        MXEC_TRY(read_file(part.path, raw));
        if (!part.encrypted) {
            out.insert(out.end(), raw.begin(), raw.end());
            continue;
        }
        if (!upload_key || !upload_id) return set_error(MXEC_E_INVALID_ARG, "encrypted part without upload key");
        std::string prefix = std::string("PART") + '\0' + upload_id + '\0';
        for (int b = 0; b < 4; ++b) prefix.push_back(char((part.part_number >> (8 * b)) & 0xFF));
        prefix.push_back('\0');
        const uint64_t nf = (part.size + MXEC_FRAME_CHUNK_SIZE - 1) / MXEC_FRAME_CHUNK_SIZE;
        std::vector<uint8_t> aads(size_t(nf) * 32 + 32);
        if (nf)
            MXEC_TRY(mxec_frame_aads(ctx, reinterpret_cast<const uint8_t*>(prefix.data()), uint32_t(prefix.size()), 0,
                                     nf, reinterpret_cast<uint8_t(*)[32]>(aads.data())));
        const size_t at = out.size();
        out.resize(at + size_t(part.size));
        uint64_t n = 0;
        MXEC_TRY(mxec_frames_decrypt(ctx, upload_key, 0, aads.data(), 32, MXEC_FRAME_CHUNK_SIZE, raw.data(),
                                     raw.size(), part.size, out.data() + at, part.size, &n));
        if (n != part.size) return set_error(MXEC_E_INTEGRITY, "part plaintext size mismatch");
    }
    return MXEC_OK;
}

// The multipart ETag (:1240-1244): MD5 over the parts' raw MD5s, "-N".
int multipart_etag(mxec_ctx* ctx, const mxec_multipart_part* parts, uint32_t n_parts, char* etag_out) {
    std::vector<uint8_t> md5s(size_t(n_parts) * 16 + 1);
    for (uint32_t p = 0; p < n_parts; ++p) std::memcpy(&md5s[size_t(p) * 16], parts[p].md5, 16);
    const uint8_t* b = md5s.data();
    const uint64_t l = uint64_t(n_parts) * 16;
    mxec_body_sums sums;
    MXEC_TRY(mxec_body_sums_batch(ctx, &b, &l, 1, MXEC_SUM_MD5, &sums));
    static const char* hx = "0123456789abcdef";
    for (int i = 0; i < 16; ++i) {
        etag_out[2 * i] = hx[sums.md5[i] >> 4];
        etag_out[2 * i + 1] = hx[sums.md5[i] & 15];
    }
    std::snprintf(etag_out + 32, 16, "-%u", n_parts);
    return MXEC_OK;
}

}  // namespace

extern "C" {

int mxec_put_object_chunked(mxec_ctx* ctx, const char* ec_dir, uint64_t chunk_size, uint32_t parity_shards,
                            const uint8_t* body, size_t len) {
    return mxec::guarded([&]() -> int {
        return put_chunked_buffer(ctx, ec_dir, chunk_size, parity_shards, body, len, -1);
    });
}

int mxec_put_object_chunked_encrypted(mxec_ctx* ctx, const char* ec_dir, uint64_t chunk_size,
                                      uint32_t parity_shards, const uint8_t key[32], const uint8_t nonce_prefix[4],
                                      const uint8_t* aad_prefix, uint32_t aad_prefix_len, const uint8_t* body,
                                      size_t len, uint32_t which, mxec_body_sums* sums_out) {
    return mxec::guarded([&]() -> int {
        if (!key || !nonce_prefix || (len && !body) || (aad_prefix_len && !aad_prefix) || (which && !sums_out))
            return set_error(MXEC_E_INVALID_ARG, "null argument");
        std::vector<uint8_t> ct;
        MXEC_TRY(encrypt_frames(ctx, key, nonce_prefix, aad_prefix, aad_prefix_len, body, len, ct));
        MXEC_TRY(put_chunked_buffer(ctx, ec_dir, chunk_size, parity_shards, ct.data(), ct.size(), int64_t(len)));
        if (!which) return MXEC_OK;
        // Md5 / ChecksumHasher over the plaintext as it arrives (:878-884).
        const uint8_t* b = body ? body : reinterpret_cast<const uint8_t*>("");
        const uint64_t l = len;
        return mxec_body_sums_batch(ctx, &b, &l, 1, which, sums_out);
    });
}

int mxec_complete_multipart_chunked(mxec_ctx* ctx, const char* ec_dir, uint64_t chunk_size,
                                    uint32_t parity_shards, const mxec_multipart_part* parts, uint32_t n_parts,
                                    char etag_out[48]) {
    return mxec::guarded([&]() -> int {
        if ((n_parts && !parts) || !etag_out) return set_error(MXEC_E_INVALID_ARG, "null argument");
        std::vector<uint8_t> body;
        for (uint32_t p = 0; p < n_parts; ++p)
            if (parts[p].encrypted) return set_error(MXEC_E_INVALID_ARG, "encrypted part: use the _encrypted driver");
        MXEC_TRY(read_parts(ctx, parts, n_parts, nullptr, nullptr, body));
        MXEC_TRY(put_chunked_buffer(ctx, ec_dir, chunk_size, parity_shards, body.data(), body.size(), -1));
        return multipart_etag(ctx, parts, n_parts, etag_out);
    });
}

int mxec_complete_multipart_chunked_encrypted(mxec_ctx* ctx, const char* ec_dir, uint64_t chunk_size,
                                              uint32_t parity_shards, const mxec_multipart_part* parts,
                                              uint32_t n_parts, const uint8_t upload_key[32], const char* upload_id,
                                              const uint8_t key[32], const uint8_t nonce_prefix[4],
                                              const uint8_t* aad_prefix, uint32_t aad_prefix_len,
                                              char etag_out[48]) {
    return mxec::guarded([&]() -> int {
        if ((n_parts && !parts) || !etag_out || !key || !nonce_prefix || (aad_prefix_len && !aad_prefix))
            return set_error(MXEC_E_INVALID_ARG, "null argument");
        std::vector<uint8_t> plain, ct;
        MXEC_TRY(read_parts(ctx, parts, n_parts, upload_key, upload_id, plain));
        MXEC_TRY(encrypt_frames(ctx, key, nonce_prefix, aad_prefix, aad_prefix_len, plain.data(), plain.size(), ct));
        MXEC_TRY(put_chunked_buffer(ctx, ec_dir, chunk_size, parity_shards, ct.data(), ct.size(), int64_t(plain.size())));
        return multipart_etag(ctx, parts, n_parts, etag_out);
    });
}


int mxec_try_reconstruct_data_chunk(mxec_ctx* ctx, const char* ec_dir, uint32_t target, uint8_t* out,
                                    uint64_t out_cap, uint64_t* out_len) {
    return mxec::guarded([&]() -> int {
        if (!ec_dir || !out_len) return set_error(MXEC_E_INVALID_ARG, "null argument");
        Manifest man;
        MXEC_TRY(read_manifest(ec_dir, man));
        if (target >= man.chunk_count) return set_error(MXEC_E_INVALID_INDEX, "target is not a data chunk");
        std::vector<uint8_t> buf;
        MXEC_TRY(reconstruct_from_dir(ctx, ec_dir, man, {target}, {&buf}));
        *out_len = buf.size();
        if (buf.size() > out_cap || (buf.size() && !out)) return set_error(MXEC_E_INVALID_ARG, "output buffer too small");
        if (!buf.empty()) std::memcpy(out, buf.data(), buf.size());
        return MXEC_OK;
    });
}

int mxec_put_object_chunked_sums(mxec_ctx* ctx, const char* ec_dir, uint64_t chunk_size, uint32_t parity_shards,
                                 const uint8_t* body, size_t len, uint32_t which, mxec_body_sums* sums_out) {
    return mxec::guarded([&]() -> int {
        if (which && !sums_out) return set_error(MXEC_E_INVALID_ARG, "null argument");
        MXEC_TRY(mxec_put_object_chunked(ctx, ec_dir, chunk_size, parity_shards, body, len));
        if (!which) return MXEC_OK;
        // The reference feeds the same bytes to Md5 / ChecksumHasher as it
        // chunks them (:722-725); here one batched pass over the whole body.
        const uint8_t* b = body ? body : reinterpret_cast<const uint8_t*>("");
        const uint64_t l = len;
        return mxec_body_sums_batch(ctx, &b, &l, 1, which, sums_out);
    });
}

}  // extern "C"

// ---- VerifiedChunkReader (chunk_reader.rs:12-276) --------------------------

namespace {

struct LoadedChunk {
    Bytes data;
    // When set, the chunk's bytes go straight to this caller buffer of
    // exactly the manifest's size instead of `data` (one-shot GET: the chunk
    // lands where it is served, no intermediate copy).
    uint8_t* dst = nullptr;
    uint64_t dst_size = 0;  // the file's size as read into dst
    int err = MXEC_OK;  // non-zero: this chunk fails the read that reaches it
    std::string msg;
    const uint8_t* ptr() const { return dst ? dst : data.data(); }
    uint64_t size() const { return dst ? dst_size : data.size(); }
};

// load_chunk_sync (:87-152) for chunks [first, last]: read, size check, one
// batched digest pass; with parity every bad chunk is rebuilt in one decode
// (:130-150), without parity a bad chunk carries its original error.
//
// The reference rebuilds a bad chunk with try_reconstruct_data_chunk, which
// re-reads and re-hashes every shard (:157-226), once per bad chunk.  Here:
// when a chunk of the range is already known bad before hashing (its file is
// missing or has the wrong size), every other shard is read up front and
// hashed in the SAME pass as the range; a chunk that only fails its digest
// costs one more pass over the shards not yet hashed.  Either way each shard
// is hashed once and every bad chunk of the range comes out of one decode.
//
// `dsts` (optional, one per chunk of the range, nullptr = none) places chunks
// in caller memory (LoadedChunk::dst).
int load_chunks(mxec_ctx* ctx, const fs::path& dir, const Manifest& man, uint32_t first, uint32_t last,
                std::vector<LoadedChunk>& out, const std::vector<uint8_t*>* dsts = nullptr) {
    const uint32_t n = last - first + 1;
    out.assign(n, LoadedChunk{});
    if (dsts)
        for (uint32_t c = 0; c < n; ++c) out[c].dst = (*dsts)[c];
    const bool parity = man.has_parity && man.parity_shards > 0;
    const int k = int(man.chunk_count);
    const int m = parity ? int(man.parity_shards) : 0;
    const int total = k + m;
    const uint64_t shard = man.has_shard ? man.shard_size : man.chunk_size;
    bool known_bad = false;
    for (uint32_t c = 0; c < n; ++c) {
        const uint32_t idx = first + c;
        LoadedChunk& lc = out[c];
        const int rc = lc.dst ? read_file_to(dir / chunk_name(idx), lc.dst, man.chunks[idx].size, &lc.dst_size)
                              : read_file(dir / chunk_name(idx), lc.data);
        if (rc != MXEC_OK) {
            lc.err = MXEC_E_IO;
            lc.msg = "failed to read chunk " + std::to_string(idx) + ": " + mxec::last_error();
            known_bad = true;
            continue;
        }
        if (lc.size() != man.chunks[idx].size) {
            lc.err = MXEC_E_INTEGRITY;
            lc.msg = "chunk " + std::to_string(idx) + " size mismatch: expected " +
                     std::to_string(man.chunks[idx].size) + ", got " + std::to_string(lc.size());
            known_bad = true;
        }
    }
    if (parity && int(man.chunks.size()) < total)
        return set_error(MXEC_E_JSON, "JSON error: manifest lists fewer shards than k+m");
    // Shards outside the range, for a rebuild: bytes, loaded with the length
    // the digest covers (:184), digest verified.
    auto want_len = [&](int i) {
        return size_t(i < k ? std::min<uint64_t>(man.chunks[size_t(i)].size, shard) : shard);
    };
    std::vector<Bytes> extra(parity ? size_t(total) : 0);
    std::vector<uint8_t> extra_loaded(extra.size(), 0), verified(extra.size(), 0);
    bool extra_read = false;
    auto read_extra = [&] {
        extra_read = true;
        for (int i = 0; i < total; ++i) {
            if (i >= int(first) && i <= int(last)) continue;
            Bytes& d = extra[size_t(i)];
            extra_loaded[size_t(i)] =
                read_file(dir / chunk_name(uint32_t(i)), d) == MXEC_OK && d.size() == want_len(i);
        }
    };
    if (parity && known_bad) read_extra();
    // One digest pass over everything loaded and not yet hashed.
    auto hash_pass = [&](bool range) -> int {
        std::vector<const uint8_t*> hp;
        std::vector<size_t> hl;
        std::vector<int> who;  // >= 0: range chunk c; < 0: extra shard -(i+1)
        if (range)
            for (uint32_t c = 0; c < n; ++c)
                if (!out[c].err) {
                    hp.push_back(out[c].size() == 0 ? reinterpret_cast<const uint8_t*>("") : out[c].ptr());
                    hl.push_back(out[c].size());
                    who.push_back(int(c));
                }
        for (size_t i = 0; i < extra.size(); ++i)
            if (extra_loaded[i] && !verified[i]) {
                hp.push_back(extra[i].empty() ? reinterpret_cast<const uint8_t*>("") : extra[i].data());
                hl.push_back(extra[i].size());
                who.push_back(-int(i) - 1);
            }
        if (hp.empty()) return MXEC_OK;
        std::vector<uint8_t> dig(hp.size() * 32);
        MXEC_TRY(mxec_sha256_batch(ctx, hp.data(), hl.data(), hp.size(), reinterpret_cast<uint8_t(*)[32]>(dig.data())));
        for (size_t t = 0; t < who.size(); ++t) {
            const std::string got = hex32(&dig[t * 32]);
            if (who[t] >= 0) {
                const uint32_t c = uint32_t(who[t]);
                if (got != man.chunks[first + c].sha256) {
                    out[c].err = MXEC_E_INTEGRITY;
                    out[c].msg = "checksum mismatch on chunk " + std::to_string(first + c) + ": expected " +
                                 man.chunks[first + c].sha256 + ", got " + got;
                }
            } else {
                const size_t i = size_t(-who[t] - 1);
                verified[i] = got == man.chunks[i].sha256;
                extra_loaded[i] = verified[i];  // a failed shard is an erasure, not hashed again
            }
        }
        return MXEC_OK;
    };
    // try_reconstruct_data_chunk (:157-226) over every shard at once: the
    // buffers hold each shard's real bytes (the kernels read past a shard's
    // length as zero = Vec::resize(shard_size)).  Present shards are passed
    // in place (the decode only reads them); missing ones get uninitialised
    // buffers the decode overwrites whole.  verify = true: the shards are not
    // hashed yet, so mxec_reconstruct hashes every present one against the
    // manifest in the same upload (a mismatch is one more erasure) -- one
    // upload, one hash launch, one decode for a range with a known-bad chunk.
    // Returns MXEC_OK with every range chunk good or carrying its error;
    // with verify, 1 when too few shards verified (the caller then finds out
    // chunk by chunk).
    auto decode = [&](bool verify) -> int {
        std::vector<Bytes> bufs(static_cast<size_t>(total));
        std::vector<uint8_t*> ptrs(static_cast<size_t>(total));
        std::vector<size_t> lens(static_cast<size_t>(total));
        std::vector<uint8_t> present(static_cast<size_t>(total), 0);
        std::vector<uint8_t> expected(verify ? size_t(total) * 32 : 0);
        for (int i = 0; i < total; ++i) {
            const size_t w = want_len(i);
            Bytes* b = &bufs[size_t(i)];
            bool have = false;
            uint8_t* ext = nullptr;
            if (i >= int(first) && i <= int(last)) {
                LoadedChunk& lc = out[size_t(i) - first];
                have = !lc.err;
                if (lc.dst) ext = lc.dst;  // exactly chunks[i].size == want_len(i) bytes
                else if (have) b = &lc.data;
            } else if (verify ? extra_loaded[size_t(i)] : verified[size_t(i)]) {
                have = true;
                b = &extra[size_t(i)];
            }
            if (have && verify && !unhex32(man.chunks[size_t(i)].sha256, &expected[size_t(i) * 32]))
                have = false;  // an unparsable digest never matches
            present[size_t(i)] = have ? 1 : 0;
            lens[size_t(i)] = w;
            if (ext) {
                ptrs[size_t(i)] = w ? ext : nullptr;
                continue;
            }
            if (!have) b->resize(w);
            ptrs[size_t(i)] = b->empty() ? nullptr : b->data();
        }
        // Zero-length shards still need a non-null pointer for the C API.
        uint8_t dummy = 0;
        for (auto& p : ptrs)
            if (!p) p = &dummy;
        int np = 0;
        const int rc = mxec_reconstruct(ctx, k, m, shard, ptrs.data(), lens.data(),
                                        verify ? reinterpret_cast<const uint8_t(*)[32]>(expected.data()) : nullptr,
                                        present.data(), MXEC_F_DATA_ONLY, &np);
        if (verify && rc == MXEC_E_TOO_FEW_SHARDS_PRESENT) return 1;
        const std::string msg = rc ? std::string(mxec::last_error()) : std::string();
        for (uint32_t c = 0; c < n; ++c) {
            LoadedChunk& lc = out[c];
            if (!lc.err) continue;  // good, or (verify) rebuilt in place after a mismatch
            if (rc) {
                lc.msg = msg;
                lc.err = rc;
                continue;
            }
            const uint32_t idx = first + c;
            const size_t real = size_t(std::min<uint64_t>(man.chunks[idx].size, shard));
            if (lc.dst) {
                lc.dst_size = real;
            } else {
                bufs[idx].resize(real);
                lc.data.swap(bufs[idx]);
            }
            lc.err = MXEC_OK;
            lc.msg.clear();
        }
        return MXEC_OK;
    };
    if (parity && known_bad) {
        const int rc = decode(true);
        if (rc <= 0) return rc;
        // Too few shards verified: hash shard by shard to give each range
        // chunk its own error (or rebuild from what did verify).
    }
    MXEC_TRY(hash_pass(true));
    if (!parity) return MXEC_OK;
    std::vector<uint32_t> bad;
    for (uint32_t c = 0; c < n; ++c)
        if (out[c].err) bad.push_back(c);
    if (bad.empty()) return MXEC_OK;
    if (!extra_read) {
        read_extra();
        MXEC_TRY(hash_pass(false));
    }
    return decode(false);
}

}  // namespace

struct mxec_reader {
    mxec_ctx* ctx = nullptr;
    fs::path dir;
    Manifest man;
    uint32_t next = 0, end = 0;  // next chunk to load, last chunk of the range
    uint64_t skip = 0, remaining = 0, batch_bytes = 0;
    std::vector<LoadedChunk> batch;
    size_t bi = 0;
    uint64_t pos = 0;
};

extern "C" {

int mxec_reader_open(mxec_ctx* ctx, const char* ec_dir, uint64_t offset, uint64_t length, uint64_t batch_bytes,
                     mxec_reader** out) {
    return mxec::guarded([&]() -> int {
        if (!ec_dir || !out) return set_error(MXEC_E_INVALID_ARG, "null argument");
        *out = nullptr;
        auto r = std::make_unique<mxec_reader>();
        MXEC_TRY(read_manifest(ec_dir, r->man));
        r->ctx = ctx;
        r->dir = ec_dir;
        r->batch_bytes = batch_bytes ? batch_bytes : (uint64_t(64) << 20);
        const Manifest& man = r->man;
        if (length == UINT64_MAX) length = offset < man.total_size ? man.total_size - offset : 0;
        if (offset + length > man.total_size) length = man.total_size > offset ? man.total_size - offset : 0;
        if (length > 0 && man.total_size > 0) {  // else Done at once (:40, :53-65)
            if (man.chunk_size == 0) return set_error(MXEC_E_JSON, "JSON error: chunk_size is 0");
            r->next = uint32_t(offset / man.chunk_size);
            r->end = uint32_t((offset + length - 1) / man.chunk_size);
            r->skip = offset % man.chunk_size;
            if (r->end >= man.chunk_count || r->end >= man.chunks.size())
                return set_error(MXEC_E_JSON, "JSON error: range past chunk_count");
            r->remaining = length;
        }
        *out = r.release();
        return MXEC_OK;
    });
}

int64_t mxec_reader_read(mxec_reader* r, uint8_t* buf, uint64_t cap) {
    try {
        if (!r || (cap && !buf)) return set_error(MXEC_E_INVALID_ARG, "null argument");
        uint64_t copied = 0;
        while (copied < cap && r->remaining > 0) {
            if (r->bi >= r->batch.size()) {
                // NeedLoad: the next chunks up to batch_bytes (at least one)
                uint32_t last = r->next;
                uint64_t bytes = r->man.chunks[r->next].size;
                while (last < r->end && bytes + r->man.chunks[last + 1].size <= r->batch_bytes)
                    bytes += r->man.chunks[++last].size;
                const int rc = load_chunks(r->ctx, r->dir, r->man, r->next, last, r->batch);
                if (rc) return copied ? int64_t(copied) : int64_t(rc);
                r->next = last + 1;
                r->bi = 0;
                r->pos = r->skip;  // skip applies to the first chunk of the range only
                r->skip = 0;
            }
            LoadedChunk& c = r->batch[r->bi];
            if (c.err) {  // serve everything before it first, as the reference streams
                if (copied) return int64_t(copied);
                return set_error(c.err, c.msg);
            }
            const uint64_t avail = c.data.size() > r->pos ? c.data.size() - r->pos : 0;
            const uint64_t take = std::min(std::min(avail, cap - copied), r->remaining);
            if (take) std::memcpy(buf + copied, c.data.data() + r->pos, take);
            copied += take;
            r->pos += take;
            r->remaining -= take;
            if (r->pos >= c.data.size()) {
                c.data = Bytes();
                ++r->bi;
                r->pos = 0;
            }
        }
        return int64_t(copied);
    } catch (const std::bad_alloc&) {
        return set_error(MXEC_E_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return set_error(MXEC_E_INVALID_ARG, e.what());
    } catch (...) {
        return set_error(MXEC_E_INVALID_ARG, "unknown exception");
    }
}

void mxec_reader_close(mxec_reader* r) { delete r; }

int mxec_get_object_chunked(mxec_ctx* ctx, const char* ec_dir, uint64_t offset, uint64_t length, uint8_t* out,
                            uint64_t out_cap, uint64_t* out_len) {
    return mxec::guarded([&]() -> int {
        if (!ec_dir || !out_len) return set_error(MXEC_E_INVALID_ARG, "null argument");
        *out_len = 0;
        // The reader's semantics (mxec_reader_open / _read over the whole range
        // in one batch), with every chunk the range covers whole read straight
        // into its place in `out`: no intermediate chunk buffer, no copy out.
        mxec_reader* r = nullptr;
        MXEC_TRY(mxec_reader_open(ctx, ec_dir, offset, length, uint64_t(1) << 40, &r));
        std::unique_ptr<mxec_reader, void (*)(mxec_reader*)> guard(r, mxec_reader_close);
        if (r->remaining > out_cap || (r->remaining && !out))
            return set_error(MXEC_E_INVALID_ARG, "output buffer too small");
        if (r->remaining == 0) return MXEC_OK;
        const Manifest& man = r->man;
        const uint32_t first = r->next, last = r->end;
        // Where each chunk's bytes are served: the first from `skip`, the rest
        // whole, in order, until `remaining` runs out (mxec_reader_read).
        std::vector<uint8_t*> dsts(last - first + 1, nullptr);
        uint64_t pos = 0, left = r->remaining;
        for (uint32_t c = first; c <= last && left; ++c) {
            const uint64_t sz = man.chunks[c].size;
            const uint64_t from = c == first ? r->skip : 0;
            const uint64_t take = std::min(sz > from ? sz - from : 0, left);
            if (from == 0 && take == sz && sz > 0) dsts[c - first] = out + pos;
            pos += take;
            left -= take;
        }
        // Windows of at most kGetWindow bytes of chunks (at least one chunk): one
        // hash round trip per window, and a slot's device staging stays bounded
        // however large the object.
        // MXEC_GET_WINDOW (bytes, read at mxec_open) overrides the window (tests).
        const uint64_t kGetWindow = ctx->c.knobs.get_window;
        std::vector<LoadedChunk> batch;
        pos = 0;
        left = r->remaining;
        for (uint32_t w0 = first; w0 <= last && left;) {
            uint32_t w1 = w0;
            uint64_t bytes = man.chunks[w0].size;
            while (w1 < last && bytes + man.chunks[w1 + 1].size <= kGetWindow) bytes += man.chunks[++w1].size;
            const std::vector<uint8_t*> wd(dsts.begin() + (w0 - first), dsts.begin() + (w1 - first) + 1);
            if (const int rc = load_chunks(ctx, r->dir, man, w0, w1, batch, &wd)) {
                *out_len = pos;
                return rc;
            }
            for (uint32_t c = w0; c <= w1 && left; ++c) {
                const LoadedChunk& lc = batch[c - w0];
                if (lc.err) {  // bytes before it are served, then the error (reader semantics)
                    *out_len = pos;
                    return set_error(lc.err, lc.msg);
                }
                const uint64_t from = c == first ? r->skip : 0;
                const uint64_t sz = lc.size();
                const uint64_t take = std::min(sz > from ? sz - from : 0, left);
                if (!lc.dst && take) std::memcpy(out + pos, lc.data.data() + from, take);
                pos += take;
                left -= take;
            }
            w0 = w1 + 1;
        }
        *out_len = pos;
        return MXEC_OK;
    });
}


int mxec_get_object_chunked_encrypted(mxec_ctx* ctx, const char* ec_dir, const uint8_t key[32],
                                      const uint8_t* aad_prefix, uint32_t aad_prefix_len, uint32_t frame_size,
                                      uint64_t plaintext_size, uint64_t offset, uint64_t length, uint8_t* out,
                                      uint64_t out_cap, uint64_t* out_len) {
    return mxec::guarded([&]() -> int {
        if (!ec_dir || !key || !out_len || (aad_prefix_len && !aad_prefix))
            return set_error(MXEC_E_INVALID_ARG, "null argument");
        if (frame_size == 0 || frame_size % 16) return set_error(MXEC_E_INVALID_ARG, "frame_size must be a positive multiple of 16");
        *out_len = 0;
        Manifest man;
        MXEC_TRY(read_manifest(ec_dir, man));
        if (plaintext_size == UINT64_MAX) {
            if (!man.has_plain) return set_error(MXEC_E_JSON, "JSON error: manifest has no plaintext_size");
            plaintext_size = man.plaintext_size;
        }
        if (offset >= plaintext_size || length == 0) return MXEC_OK;
        const uint64_t end = length == UINT64_MAX || length > plaintext_size - offset ? plaintext_size : offset + length;
        // FrameDecryptor::ciphertext_offset / for_range: the frames that cover
        // [offset, end), read through the verified chunk reader (with_range).
        const uint64_t fl = uint64_t(frame_size) + MXEC_FRAME_OVERHEAD;
        const uint64_t f0 = offset / frame_size, f1 = (end - 1) / frame_size;
        const uint64_t ct_off = f0 * fl;
        const uint64_t ct_len = std::min<uint64_t>(man.total_size - std::min(man.total_size, ct_off), (f1 - f0 + 1) * fl);
        if (end - offset > out_cap || !out) return set_error(MXEC_E_INVALID_ARG, "output buffer too small");
        Bytes ct(size_t(ct_len) + 1);  // every byte written by the GET below
        uint64_t got = 0;
        MXEC_TRY(mxec_get_object_chunked(ctx, ec_dir, ct_off, ct_len, ct.data(), ct_len, &got));
        const uint64_t nf = f1 - f0 + 1;
        const uint64_t pt_lo = f0 * frame_size, pt_hi = std::min<uint64_t>(plaintext_size, (f1 + 1) * uint64_t(frame_size));
        std::vector<uint8_t> aads(size_t(nf) * 32);
        MXEC_TRY(mxec_frame_aads(ctx, aad_prefix, aad_prefix_len, f0, nf, reinterpret_cast<uint8_t(*)[32]>(aads.data())));
        uint64_t n = 0;
        if (offset == pt_lo && end == pt_hi) {
            // The range is whole frames (a full GET): decrypt straight into out.
            MXEC_TRY(mxec_frames_decrypt(ctx, key, f0, aads.data(), 32, frame_size, ct.data(), got, pt_hi - pt_lo,
                                         out, out_cap, &n));
        } else {
            Bytes pt(size_t(pt_hi - pt_lo) + 1);
            MXEC_TRY(mxec_frames_decrypt(ctx, key, f0, aads.data(), 32, frame_size, ct.data(), got, pt_hi - pt_lo,
                                         pt.data(), pt.size(), &n));
            std::memcpy(out, pt.data() + (offset - pt_lo), size_t(end - offset));
        }
        *out_len = end - offset;
        return MXEC_OK;
    });
}

}  // extern "C"

// manifest_check — CPU harness for maxio_amd/csrc/manifest.cpp (the
// ChunkManifest reader / writer of libmaxio_ec.so), built by
// tests/test_manifest_strict.py with -fsanitize=address,undefined.
//
//   manifest_check FILE...   one JSON line per file: the parsed fields, or
//                            the error the reader reports
//   manifest_check --roundtrip   writer -> reader on generated manifests
#include <cstdio>
#include <fstream>
#include <iterator>
#include <random>
#include <string>

#include "../../maxio_amd/csrc/manifest.hpp"

namespace {

std::string esc(const std::string& s) {
    std::string o;
    for (unsigned char c : s) {
        if (c == '"' || c == '\\') {
            o += '\\';
            o += char(c);
        } else if (c < 0x20) {
            char b[8];
            std::snprintf(b, sizeof b, "\\u%04x", c);
            o += b;
        } else {
            o += char(c);
        }
    }
    return o;
}

void report(const std::string& name, const std::string& text) {
    mxec::Manifest m;
    std::string err;
    if (!mxec::utf8_valid(reinterpret_cast<const uint8_t*>(text.data()), text.size())) {
        std::printf("{\"file\": \"%s\", \"ok\": false, \"io\": true, \"error\": \"invalid UTF-8\"}\n", esc(name).c_str());
        return;
    }
    if (!mxec::parse_manifest(text, m, &err)) {
        std::printf("{\"file\": \"%s\", \"ok\": false, \"error\": \"%s\"}\n", esc(name).c_str(), esc(err).c_str());
        return;
    }
    std::string kinds, shas = "[";
    for (size_t i = 0; i < m.chunks.size(); ++i) {
        kinds += m.chunks[i].kind ? 'P' : 'D';
        shas += (i ? ", \"" : "\"") + esc(m.chunks[i].sha256) + "\"";
    }
    shas += "]";
    std::string idx = "[", sizes = "[";
    for (size_t i = 0; i < m.chunks.size(); ++i) {
        idx += (i ? ", " : "") + std::to_string(m.chunks[i].index);
        sizes += (i ? ", " : "") + std::to_string(m.chunks[i].size);
    }
    idx += "]";
    sizes += "]";
    std::printf(
        "{\"file\": \"%s\", \"ok\": true, \"version\": %u, \"total_size\": %llu, \"chunk_size\": %llu, "
        "\"chunk_count\": %u, \"kinds\": \"%s\", \"index\": %s, \"size\": %s, \"sha256\": %s, "
        "\"parity_shards\": %s, \"shard_size\": %s, \"plaintext_size\": %s}\n",
        esc(name).c_str(), m.version, (unsigned long long)m.total_size, (unsigned long long)m.chunk_size,
        m.chunk_count, kinds.c_str(), idx.c_str(), sizes.c_str(), shas.c_str(),
        m.has_parity ? std::to_string(m.parity_shards).c_str() : "null",
        m.has_shard ? std::to_string(m.shard_size).c_str() : "null",
        m.has_plain ? std::to_string(m.plaintext_size).c_str() : "null");
}

int roundtrip() {
    std::mt19937_64 g(0x6D6178696F);
    int bad = 0;
    for (int t = 0; t < 500; ++t) {
        mxec::Manifest m;
        m.version = uint32_t(g() % 3);
        m.total_size = g();
        m.chunk_size = g() >> (g() % 64);
        const int k = int(g() % 40), par = int(g() % 6);
        m.chunk_count = uint32_t(k);
        for (int i = 0; i < k + par; ++i) {
            mxec::Manifest::Chunk c;
            c.index = uint32_t(i);
            c.size = g() % 100000;
            for (int h = 0; h < 64; ++h) c.sha256 += "0123456789abcdef"[g() % 16];
            c.kind = i >= k;
            m.chunks.push_back(c);
        }
        m.has_parity = g() & 1;
        m.parity_shards = uint32_t(g());
        m.has_shard = g() & 1;
        m.shard_size = g();
        m.has_plain = g() & 1;
        m.plaintext_size = g();
        const std::string js = mxec::manifest_json(m);
        mxec::Manifest r;
        std::string err;
        bool ok = mxec::parse_manifest(js, r, &err) && mxec::manifest_json(r) == js;
        if (!ok) {
            std::fprintf(stderr, "roundtrip %d failed: %s\n", t, err.c_str());
            ++bad;
        }
    }
    std::printf("{\"roundtrip\": 500, \"failed\": %d}\n", bad);
    return bad ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "--roundtrip") return roundtrip();
    for (int i = 1; i < argc; ++i) {
        std::ifstream f(argv[i], std::ios::binary);
        std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        report(argv[i], text);
    }
    return 0;
}

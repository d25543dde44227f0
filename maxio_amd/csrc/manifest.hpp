// manifest.hpp — the on-disk ChunkManifest / ChunkInfo contract
// (storage/mod.rs:145-189): the serde_json::to_string_pretty writer
// (filesystem.rs:772) and a reader that accepts exactly what
// serde_json::from_str::<ChunkManifest> accepts (filesystem.rs:3171).
//
// Host-only (no HIP): built into libmaxio_ec.so and, on its own with
// -fsanitize=address,undefined, into the CPU test harness
// tests/c_manifest/manifest_check.cpp.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mxec {

struct Manifest {
    uint32_t version = 1;
    uint64_t total_size = 0, chunk_size = 0;
    uint32_t chunk_count = 0;
    struct Chunk {
        uint32_t index = 0;
        uint64_t size = 0;
        std::string sha256;
        uint8_t kind = 0;  // 0 = Data, 1 = Parity
    };
    std::vector<Chunk> chunks;
    bool has_parity = false, has_shard = false, has_plain = false;
    uint32_t parity_shards = 0;
    uint64_t shard_size = 0, plaintext_size = 0;
};

// serde_json::to_string_pretty of the manifest (fields in declaration
// order, two-space indent, `kind` only for parity, Option fields only when
// Some, no trailing newline).
std::string manifest_json(const Manifest& m);

// serde_json::from_str::<ChunkManifest>: true on success; on failure *err
// holds a serde_json-style message ("missing field `version` at line 1
// column 2").  What it enforces, as serde does:
//  * RFC 8259 JSON: whitespace is space / tab / LF / CR only; strings with
//    every escape (\uXXXX with surrogate pairs) and no raw control
//    characters; numbers without leading zeros; nothing after the value;
//    at most 127 nested arrays / objects (serde_json's recursion limit 128);
//  * a struct as an object (any field order, unknown fields skipped,
//    duplicate known fields rejected) or as an array in field order;
//  * required fields present (version, total_size, chunk_size, chunk_count,
//    chunks; index, size, sha256), Option fields absent / null / a value;
//  * u32 / u64 fields non-negative integers in range (a float, exponent,
//    sign or overflow is an error);
//  * `kind` one of "data" / "parity" (or {"parity": null}), default data.
// The text must already be valid UTF-8 (the reference reads it with
// read_to_string, which fails with an I/O error otherwise; utf8_valid).
bool parse_manifest(const std::string& text, Manifest& m, std::string* err);

// std::str::from_utf8 validity (overlongs, surrogates and > U+10FFFF
// rejected).
bool utf8_valid(const uint8_t* p, size_t n);

}  // namespace mxec

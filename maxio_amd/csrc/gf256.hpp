// gf256.hpp — host-side GF(2^8) algebra for the device RS kernels.
//
// Field and matrix conventions follow reed-solomon-erasure 6.0.0 (galois_8),
// the crate MaxIO calls at filesystem.rs:1121-1124 and chunk_reader.rs:168,211:
// polynomial 0x11D, generator 2, encoding matrix = V * inverse(V[0..k]) with
// V[r][c] = r^c.  The host only builds small k x k matrices and the per-kernel
// coefficient tables; every byte of shard data is processed on the GPU.
#pragma once

#include <cstddef>
#include <cstdint>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace mxec {

uint8_t gf_mul(uint8_t a, uint8_t b);
uint8_t gf_div(uint8_t a, uint8_t b);
uint8_t gf_pow(uint8_t a, unsigned n);

// Row-major dense matrix over GF(2^8).
struct GfMatrix {
    int rows = 0, cols = 0;
    std::vector<uint8_t> v;
    GfMatrix() = default;
    GfMatrix(int r, int c) : rows(r), cols(c), v(size_t(r) * c, 0) {}
    uint8_t& at(int r, int c) { return v[size_t(r) * cols + c]; }
    uint8_t at(int r, int c) const { return v[size_t(r) * cols + c]; }
};

GfMatrix gf_matmul(const GfMatrix& a, const GfMatrix& b);
// Gauss-Jordan inverse; returns false when singular.
bool gf_invert(const GfMatrix& in, GfMatrix& out);

// Crate-equivalent argument check of ReedSolomon::new(k, m).
int rs_check(int k, int m);
// (k+m) x k systematic encoding matrix; cached per (k, m).
std::shared_ptr<const GfMatrix> rs_matrix(int k, int m);

// Per-coefficient v_perm_b32 lookup tables used by the RS kernel.
// For coefficient c the 8 dwords are:
//   [0] c*{0,1,2,3}          [1] c*{4,5,6,7}          (bits 0-2 of x)
//   [2] c*{0,8,16,24}        [3] c*{32,40,48,56}      (bits 3-5)
//   [4] c*{0,64,128,192}     [5..7] 0                 (bits 6-7)
// so c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6] with each lookup one v_perm.
constexpr int kCoefDwords = 8;
void coef_entry(uint8_t c, uint32_t out[kCoefDwords]);
// Table for applying `rows` (r x k) to k inputs, laid out [j][i][8] so one
// scalar load per input column j fetches the coefficients of every output.
std::vector<uint32_t> coef_tables(const GfMatrix& rows);

// Decode plan of one erasure pattern (reconstruct_internal restated):
//   valid   = first k present shard indices (the decode inputs),
//   missing = the shard indices to rebuild (data first, then parity),
//   rows    = |missing| x k matrix applied to the valid shards:
//             data row e  -> row e of inverse(M[valid]),
//             parity row  -> M[k+p] * inverse(M[valid]) (parity re-encoded
//                            from the rebuilt data in one pass; GF arithmetic
//                            is exact so the bytes equal the crate's two-pass
//                            result).
struct DecodePlan {
    int k = 0, m = 0;
    std::vector<int> valid;
    std::vector<int> missing;
    GfMatrix rows;
    std::vector<uint32_t> table;  // coef_tables(rows)
};

// LRU cache of decode plans keyed on (k, m, data_only, erasure pattern),
// like the crate's data_decode_matrix_cache (capacity 254) but process-wide.
class DecodeCache {
public:
    explicit DecodeCache(size_t capacity = 16384) : cap_(capacity) {}
    // present: k+m flags; returns nullptr if fewer than k are present.
    std::shared_ptr<const DecodePlan> get(int k, int m, const uint8_t* present, bool data_only);

private:
    using Key = std::vector<uint8_t>;
    size_t cap_;
    std::mutex mu_;
    std::list<std::pair<Key, std::shared_ptr<const DecodePlan>>> lru_;
    std::map<Key, decltype(lru_)::iterator> index_;
};

DecodeCache& decode_cache();

}  // namespace mxec

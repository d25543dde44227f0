// gf256.cpp — GF(2^8) tables, encoding/decoding matrices and the v_perm
// coefficient tables consumed by rs_kernel.hip.  See gf256.hpp.
#include "gf256.hpp"

#include "../../include/maxio_ec.h"

#include <cstring>

namespace mxec {
namespace {

struct Tables {
    uint8_t log[256];
    uint8_t exp[510];
    Tables() {
        std::memset(log, 0, sizeof log);
        unsigned b = 1;
        for (unsigned i = 0; i < 255; ++i) {
            exp[i] = exp[i + 255] = uint8_t(b);
            log[b] = uint8_t(i);
            b <<= 1;
            if (b & 0x100) b ^= 0x11D;  // x^8 = x^4 + x^3 + x^2 + 1
        }
    }
};

const Tables& T() {
    static const Tables t;
    return t;
}

}  // namespace

uint8_t gf_mul(uint8_t a, uint8_t b) {
    if (!a || !b) return 0;
    return T().exp[T().log[a] + T().log[b]];
}

uint8_t gf_div(uint8_t a, uint8_t b) {
    if (!a) return 0;
    int l = int(T().log[a]) - int(T().log[b]);
    if (l < 0) l += 255;
    return T().exp[l];
}

uint8_t gf_pow(uint8_t a, unsigned n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return T().exp[(unsigned(T().log[a]) * n) % 255];
}

GfMatrix gf_matmul(const GfMatrix& a, const GfMatrix& b) {
    GfMatrix c(a.rows, b.cols);
    for (int r = 0; r < a.rows; ++r)
        for (int i = 0; i < a.cols; ++i) {
            uint8_t x = a.at(r, i);
            if (!x) continue;
            for (int col = 0; col < b.cols; ++col) c.at(r, col) ^= gf_mul(x, b.at(i, col));
        }
    return c;
}

bool gf_invert(const GfMatrix& in, GfMatrix& out) {
    const int n = in.rows;
    if (n != in.cols || n <= 0) return false;
    GfMatrix w(n, 2 * n);
    for (int r = 0; r < n; ++r) {
        for (int c = 0; c < n; ++c) w.at(r, c) = in.at(r, c);
        w.at(r, n + r) = 1;
    }
    for (int col = 0; col < n; ++col) {
        int piv = -1;
        for (int r = col; r < n; ++r)
            if (w.at(r, col)) { piv = r; break; }
        if (piv < 0) return false;
        if (piv != col)
            for (int c = 0; c < 2 * n; ++c) std::swap(w.at(piv, c), w.at(col, c));
        uint8_t inv = gf_div(1, w.at(col, col));
        for (int c = 0; c < 2 * n; ++c) w.at(col, c) = gf_mul(inv, w.at(col, c));
        for (int r = 0; r < n; ++r) {
            if (r == col || !w.at(r, col)) continue;
            uint8_t s = w.at(r, col);
            for (int c = 0; c < 2 * n; ++c) w.at(r, c) ^= gf_mul(s, w.at(col, c));
        }
    }
    out = GfMatrix(n, n);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) out.at(r, c) = w.at(r, n + c);
    return true;
}

int rs_check(int k, int m) {
    if (k <= 0) return MXEC_E_TOO_FEW_DATA_SHARDS;
    if (m <= 0) return MXEC_E_TOO_FEW_PARITY_SHARDS;
    if (k + m > 256) return MXEC_E_TOO_MANY_SHARDS;
    return MXEC_OK;
}

std::shared_ptr<const GfMatrix> rs_matrix(int k, int m) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, std::shared_ptr<const GfMatrix>> cache;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({k, m});
    if (it != cache.end()) return it->second;
    const int total = k + m;
    GfMatrix v(total, k), top(k, k), top_inv;
    for (int r = 0; r < total; ++r)
        for (int c = 0; c < k; ++c) v.at(r, c) = gf_pow(uint8_t(r), unsigned(c));
    for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) top.at(r, c) = v.at(r, c);
    if (!gf_invert(top, top_inv)) return nullptr;  // Vandermonde rows r<256 are distinct: never
    auto mat = std::make_shared<const GfMatrix>(gf_matmul(v, top_inv));
    cache[{k, m}] = mat;
    return mat;
}

void coef_entry(uint8_t c, uint32_t out[kCoefDwords]) {
    auto pack = [c](unsigned b0, unsigned b1, unsigned b2, unsigned b3) {
        return uint32_t(gf_mul(c, uint8_t(b0))) | uint32_t(gf_mul(c, uint8_t(b1))) << 8 |
               uint32_t(gf_mul(c, uint8_t(b2))) << 16 | uint32_t(gf_mul(c, uint8_t(b3))) << 24;
    };
    out[0] = pack(0, 1, 2, 3);
    out[1] = pack(4, 5, 6, 7);
    out[2] = pack(0, 8, 16, 24);
    out[3] = pack(32, 40, 48, 56);
    out[4] = pack(0, 64, 128, 192);
    out[5] = out[6] = out[7] = 0;
}

std::vector<uint32_t> coef_tables(const GfMatrix& rows) {
    std::vector<uint32_t> t(size_t(rows.rows) * rows.cols * kCoefDwords);
    for (int j = 0; j < rows.cols; ++j)
        for (int i = 0; i < rows.rows; ++i)
            coef_entry(rows.at(i, j), &t[(size_t(j) * rows.rows + i) * kCoefDwords]);
    return t;
}

std::shared_ptr<const DecodePlan> DecodeCache::get(int k, int m, const uint8_t* present,
                                                   bool data_only) {
    const int total = k + m;
    Key key;
    key.reserve(size_t(total) + 3);
    key.push_back(uint8_t(k));
    key.push_back(uint8_t(m));
    key.push_back(data_only ? 1 : 0);
    int np = 0;
    for (int i = 0; i < total; ++i) {
        key.push_back(present[i] ? 1 : 0);
        np += present[i] ? 1 : 0;
    }
    if (np < k) return nullptr;
    {
        std::lock_guard<std::mutex> g(mu_);
        auto it = index_.find(key);
        if (it != index_.end()) {
            lru_.splice(lru_.begin(), lru_, it->second);
            return it->second->second;
        }
    }
    auto mat = rs_matrix(k, m);
    auto plan = std::make_shared<DecodePlan>();
    plan->k = k;
    plan->m = m;
    for (int i = 0; i < total && int(plan->valid.size()) < k; ++i)
        if (present[i]) plan->valid.push_back(i);
    for (int i = 0; i < total; ++i)
        if (!present[i] && (i < k || !data_only)) plan->missing.push_back(i);
    GfMatrix sub(k, k), dec;
    for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) sub.at(r, c) = mat->at(plan->valid[r], c);
    if (!gf_invert(sub, dec)) return nullptr;  // rows of a systematic RS matrix: never
    plan->rows = GfMatrix(int(plan->missing.size()), k);
    for (size_t t = 0; t < plan->missing.size(); ++t) {
        const int s = plan->missing[t];
        for (int c = 0; c < k; ++c) {
            uint8_t acc;
            if (s < k) {
                acc = dec.at(s, c);
            } else {
                acc = 0;
                for (int i = 0; i < k; ++i) acc ^= gf_mul(mat->at(s, i), dec.at(i, c));
            }
            plan->rows.at(int(t), c) = acc;
        }
    }
    plan->table = coef_tables(plan->rows);
    std::shared_ptr<const DecodePlan> cplan = plan;
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(key);
    if (it != index_.end()) return it->second->second;
    lru_.emplace_front(key, cplan);
    index_[key] = lru_.begin();
    while (lru_.size() > cap_) {
        index_.erase(lru_.back().first);
        lru_.pop_back();
    }
    return cplan;
}

DecodeCache& decode_cache() {
    static DecodeCache c;
    return c;
}

}  // namespace mxec

// manifest.cpp — ChunkManifest JSON writer and a serde_json-exact reader
// (storage/mod.rs:145-189; written filesystem.rs:772, read :3171 and by
// every GET through VerifiedChunkReader).  Host-only; see manifest.hpp for
// the rules the reader enforces.
#include "manifest.hpp"

#include <sstream>

namespace mxec {

std::string manifest_json(const Manifest& m) {
    std::ostringstream o;
    o << "{\n  \"version\": " << m.version << ",\n  \"total_size\": " << m.total_size
      << ",\n  \"chunk_size\": " << m.chunk_size << ",\n  \"chunk_count\": " << m.chunk_count
      << ",\n  \"chunks\": [";
    for (size_t i = 0; i < m.chunks.size(); ++i) {
        const auto& c = m.chunks[i];
        o << (i ? ",\n" : "\n") << "    {\n      \"index\": " << c.index << ",\n      \"size\": " << c.size
          << ",\n      \"sha256\": \"" << c.sha256 << "\"";
        if (c.kind == 1) o << ",\n      \"kind\": \"parity\"";
        o << "\n    }";
    }
    o << (m.chunks.empty() ? "]" : "\n  ]");
    if (m.has_parity) o << ",\n  \"parity_shards\": " << m.parity_shards;
    if (m.has_shard) o << ",\n  \"shard_size\": " << m.shard_size;
    if (m.has_plain) o << ",\n  \"plaintext_size\": " << m.plaintext_size;
    o << "\n}";
    return o.str();
}

bool utf8_valid(const uint8_t* p, size_t n) {
    size_t i = 0;
    while (i < n) {
        const uint8_t c = p[i];
        if (c < 0x80) {
            ++i;
            continue;
        }
        size_t len;
        uint32_t cp, min;
        if ((c & 0xE0) == 0xC0) len = 2, cp = c & 0x1F, min = 0x80;
        else if ((c & 0xF0) == 0xE0) len = 3, cp = c & 0x0F, min = 0x800;
        else if ((c & 0xF8) == 0xF0) len = 4, cp = c & 0x07, min = 0x10000;
        else return false;
        if (n - i < len) return false;
        for (size_t t = 1; t < len; ++t) {
            if ((p[i + t] & 0xC0) != 0x80) return false;
            cp = cp << 6 | (p[i + t] & 0x3F);
        }
        if (cp < min || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
        i += len;
    }
    return true;
}

namespace {

// serde_json's default recursion limit: entering the 128th nested array or
// object is an error.
constexpr int kMaxDepth = 128;

class Reader {
public:
    explicit Reader(const std::string& s) : s_(s) {}
    std::string err;

    bool document(Manifest& m) {
        ws();
        if (!manifest(m)) return false;
        ws();
        if (i_ < s_.size()) return fail("trailing characters");
        return true;
    }

private:
    const std::string& s_;
    size_t i_ = 0;
    int depth_ = 0;

    bool fail(const std::string& msg) {
        if (err.empty()) {
            size_t line = 1, col = 0;
            for (size_t t = 0; t < i_ && t < s_.size(); ++t) {
                if (s_[t] == '\n') line++, col = 0;
                else col++;
            }
            err = msg + " at line " + std::to_string(line) + " column " + std::to_string(col);
        }
        return false;
    }
    int peek() const { return i_ < s_.size() ? static_cast<unsigned char>(s_[i_]) : -1; }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) ++i_;
    }
    bool enter() {
        if (++depth_ >= kMaxDepth) return fail("recursion limit exceeded");
        ++i_;
        ws();
        return true;
    }
    // After an element of an array / object: ',' (not before the closer) or
    // the closer.  *more = another element follows.
    bool next(char close, bool* more) {
        ws();
        if (peek() == ',') {
            ++i_;
            ws();
            if (peek() == close) return fail("trailing comma");
            *more = true;
            return true;
        }
        if (peek() == close) {
            ++i_;
            --depth_;
            *more = false;
            return true;
        }
        if (peek() < 0) return fail("EOF while parsing a value");
        return fail(close == '}' ? "expected `,` or `}`" : "expected `,` or `]`");
    }
    bool literal(const char* lit) {
        for (size_t t = 0; lit[t]; ++t, ++i_)
            if (i_ >= s_.size() || s_[i_] != lit[t]) return fail(i_ >= s_.size() ? "EOF while parsing a value" : "expected ident");
        return true;
    }
    static int hexv(int c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    bool hex4(uint32_t* v) {
        *v = 0;
        for (int t = 0; t < 4; ++t, ++i_) {
            if (i_ >= s_.size()) return fail("EOF while parsing a string");
            const int h = hexv(static_cast<unsigned char>(s_[i_]));
            if (h < 0) return fail("invalid escape");
            *v = *v << 4 | uint32_t(h);
        }
        return true;
    }
    static void put_utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) {
            out.push_back(char(cp));
        } else if (cp < 0x800) {
            out.push_back(char(0xC0 | cp >> 6));
            out.push_back(char(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {
            out.push_back(char(0xE0 | cp >> 12));
            out.push_back(char(0x80 | (cp >> 6 & 0x3F)));
            out.push_back(char(0x80 | (cp & 0x3F)));
        } else {
            out.push_back(char(0xF0 | cp >> 18));
            out.push_back(char(0x80 | (cp >> 12 & 0x3F)));
            out.push_back(char(0x80 | (cp >> 6 & 0x3F)));
            out.push_back(char(0x80 | (cp & 0x3F)));
        }
    }
    // At '"': the decoded string.
    bool string(std::string& out) {
        ++i_;
        for (;;) {
            if (i_ >= s_.size()) return fail("EOF while parsing a string");
            const unsigned char c = static_cast<unsigned char>(s_[i_]);
            if (c == '"') {
                ++i_;
                return true;
            }
            if (c < 0x20) return fail("control character (\\u0000-\\u001F) found while parsing a string");
            if (c != '\\') {
                out.push_back(char(c));
                ++i_;
                continue;
            }
            ++i_;
            if (i_ >= s_.size()) return fail("EOF while parsing a string");
            const char e = s_[i_++];
            switch (e) {
                case '"': out.push_back('"'); break;
                case '\\': out.push_back('\\'); break;
                case '/': out.push_back('/'); break;
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'n': out.push_back('\n'); break;
                case 'r': out.push_back('\r'); break;
                case 't': out.push_back('\t'); break;
                case 'u': {
                    uint32_t cp;
                    if (!hex4(&cp)) return false;
                    if (cp >= 0xDC00 && cp <= 0xDFFF) return fail("lone leading surrogate in hex escape");
                    if (cp >= 0xD800 && cp <= 0xDBFF) {
                        if (i_ + 1 >= s_.size() || s_[i_] != '\\' || s_[i_ + 1] != 'u')
                            return fail("unexpected end of hex escape");
                        i_ += 2;
                        uint32_t lo;
                        if (!hex4(&lo)) return false;
                        if (lo < 0xDC00 || lo > 0xDFFF) return fail("lone leading surrogate in hex escape");
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    put_utf8(out, cp);
                    break;
                }
                default:
                    return fail("invalid escape");
            }
        }
    }
    // A JSON number token; *frac_exp: it has a fraction or an exponent.
    bool number(size_t* b, size_t* e, bool* neg, bool* frac_exp) {
        *b = i_;
        *neg = peek() == '-';
        if (*neg) ++i_;
        if (peek() == '0') {
            ++i_;
            if (peek() >= '0' && peek() <= '9') return fail("invalid number");
        } else if (peek() >= '1' && peek() <= '9') {
            while (peek() >= '0' && peek() <= '9') ++i_;
        } else {
            return fail("invalid number");
        }
        *frac_exp = false;
        if (peek() == '.') {
            ++i_;
            if (!(peek() >= '0' && peek() <= '9')) return fail("invalid number");
            while (peek() >= '0' && peek() <= '9') ++i_;
            *frac_exp = true;
        }
        if (peek() == 'e' || peek() == 'E') {
            ++i_;
            if (peek() == '+' || peek() == '-') ++i_;
            if (!(peek() >= '0' && peek() <= '9')) return fail("invalid number");
            while (peek() >= '0' && peek() <= '9') ++i_;
            *frac_exp = true;
        }
        *e = i_;
        return true;
    }
    bool skip() {
        ws();
        const int c = peek();
        if (c < 0) return fail("EOF while parsing a value");
        if (c == '"') {
            std::string t;
            return string(t);
        }
        if (c == '{' || c == '[') {
            const char close = c == '{' ? '}' : ']';
            if (!enter()) return false;
            if (peek() == close) {
                ++i_;
                --depth_;
                return true;
            }
            for (bool more = true; more;) {
                if (c == '{') {
                    if (peek() != '"') return fail(peek() < 0 ? "EOF while parsing an object" : "key must be a string");
                    std::string key;
                    if (!string(key)) return false;
                    ws();
                    if (peek() != ':') return fail("expected `:`");
                    ++i_;
                }
                if (!skip() || !next(close, &more)) return false;
            }
            return true;
        }
        if (c == 't') return literal("true");
        if (c == 'f') return literal("false");
        if (c == 'n') return literal("null");
        if (c == '-' || (c >= '0' && c <= '9')) {
            size_t b, e;
            bool neg, fe;
            return number(&b, &e, &neg, &fe);
        }
        return fail("expected value");
    }
    // What serde's "invalid type" error names for the value at the cursor.
    std::string unexpected() {
        const int c = peek();
        if (c == '"') return "string";
        if (c == 't' || c == 'f') return "boolean";
        if (c == 'n') return "null";
        if (c == '[') return "sequence";
        if (c == '{') return "map";
        return "value";
    }
    // An unsigned integer field: bits = 32 or 64.
    bool uint(uint64_t* v, int bits) {
        ws();
        const char* what = bits == 32 ? "u32" : "u64";
        const int c = peek();
        if (c < 0) return fail("EOF while parsing a value");
        if (c != '-' && !(c >= '0' && c <= '9')) {
            if (c == '"' || c == 't' || c == 'f' || c == 'n' || c == '[' || c == '{')
                return fail("invalid type: " + unexpected() + ", expected " + what);
            return fail("expected value");
        }
        size_t b, e;
        bool neg, fe;
        if (!number(&b, &e, &neg, &fe)) return false;
        const std::string tok = s_.substr(b, e - b);
        if (fe) return fail("invalid type: floating point `" + tok + "`, expected " + what);
        // Digits only from here (after an optional '-').
        const size_t d0 = neg ? 1 : 0;
        bool overflow = false;
        uint64_t x = 0;
        for (size_t t = d0; t < tok.size(); ++t) {
            const uint64_t dg = uint64_t(tok[t] - '0');
            if (x > (UINT64_MAX - dg) / 10) overflow = true;
            x = x * 10 + dg;
        }
        if (neg) {
            // serde_json: "-0" is the float -0.0; -N that fits i64 is an
            // integer (out of range for an unsigned field); anything
            // larger parses as a float.
            if (x == 0 || overflow || x > uint64_t(INT64_MAX) + 1)
                return fail("invalid type: floating point `" + tok + "`, expected " + what);
            return fail("invalid value: integer `" + tok + "`, expected " + what);
        }
        if (overflow) return fail("invalid type: floating point `" + tok + "`, expected " + what);
        if (bits == 32 && x > UINT32_MAX) return fail("invalid value: integer `" + tok + "`, expected u32");
        *v = x;
        return true;
    }
    bool u32(uint32_t* v) {
        uint64_t x = 0;
        if (!uint(&x, 32)) return false;
        *v = uint32_t(x);
        return true;
    }
    // Option<u32 / u64>: null -> None.
    bool opt(bool* has, uint64_t* v, int bits) {
        ws();
        if (peek() == 'n') {
            if (!literal("null")) return false;
            *has = false;
            return true;
        }
        if (!uint(v, bits)) return false;
        *has = true;
        return true;
    }
    bool text(std::string* out) {
        ws();
        if (peek() != '"') {
            if (peek() < 0) return fail("EOF while parsing a value");
            return fail("invalid type: " + unexpected() + ", expected a string");
        }
        out->clear();
        return string(*out);
    }
    static bool variant(const std::string& name, uint8_t* kind) {
        if (name == "data") *kind = 0;
        else if (name == "parity") *kind = 1;
        else return false;
        return true;
    }
    // ChunkKind (rename_all = "lowercase"): "data" | "parity", or the
    // externally tagged map form {"parity": null}.
    bool kind(uint8_t* k) {
        ws();
        if (peek() == '"') {
            std::string name;
            if (!string(name)) return false;
            if (!variant(name, k)) return fail("unknown variant `" + name + "`, expected `data` or `parity`");
            return true;
        }
        if (peek() == '{') {
            if (!enter()) return false;
            if (peek() != '"') return fail(peek() == '}' ? "expected value" : "key must be a string");
            std::string name;
            if (!string(name)) return false;
            if (!variant(name, k)) return fail("unknown variant `" + name + "`, expected `data` or `parity`");
            ws();
            if (peek() != ':') return fail("expected `:`");
            ++i_;
            ws();
            if (peek() != 'n') return fail("invalid type: " + unexpected() + ", expected unit");
            if (!literal("null")) return false;
            ws();
            if (peek() != '}') return fail("expected value");
            ++i_;
            --depth_;
            return true;
        }
        if (peek() < 0) return fail("EOF while parsing a value");
        return fail("invalid type: " + unexpected() + ", expected enum ChunkKind");
    }

    // ---- ChunkInfo { index: u32, size: u64, sha256: String, kind } -------
    bool chunk(Manifest::Chunk* c) {
        ws();
        const int open = peek();
        bool seen[4] = {false, false, false, false};
        static const char* const names[4] = {"index", "size", "sha256", "kind"};
        if (open == '[') {  // serde's sequence form, field order
            if (!enter()) return false;
            for (int f = 0; f < 4; ++f) {
                if (peek() == ']') {
                    if (f < 3) return fail("invalid length " + std::to_string(f) + ", expected struct ChunkInfo with 4 elements");
                    break;
                }
                bool ok = f == 0 ? u32(&c->index) : f == 1 ? uint(&c->size, 64) : f == 2 ? text(&c->sha256) : kind(&c->kind);
                if (!ok) return false;
                seen[f] = true;
                ws();
                if (peek() == ',') {
                    ++i_;
                    ws();
                    if (peek() == ']') return fail("trailing comma");
                    if (f == 3) return fail("trailing characters");
                } else if (peek() != ']') {
                    return fail(peek() < 0 ? "EOF while parsing a list" : "expected `,` or `]`");
                }
            }
            ++i_;
            --depth_;
            return true;
        }
        if (open != '{') {
            if (open < 0) return fail("EOF while parsing a value");
            return fail("invalid type: " + unexpected() + ", expected struct ChunkInfo");
        }
        if (!enter()) return false;
        bool more = peek() != '}';
        if (!more) {
            ++i_;
            --depth_;
        }
        while (more) {
            if (peek() != '"') return fail(peek() < 0 ? "EOF while parsing an object" : "key must be a string");
            std::string key;
            if (!string(key)) return false;
            ws();
            if (peek() != ':') return fail("expected `:`");
            ++i_;
            int f = -1;
            for (int t = 0; t < 4; ++t)
                if (key == names[t]) f = t;
            if (f >= 0 && seen[f]) return fail(std::string("duplicate field `") + names[f] + "`");
            bool ok = f == 0 ? u32(&c->index) : f == 1 ? uint(&c->size, 64) : f == 2 ? text(&c->sha256)
                      : f == 3 ? kind(&c->kind) : skip();
            if (!ok) return false;
            if (f >= 0) seen[f] = true;
            if (!next('}', &more)) return false;
        }
        for (int f = 0; f < 3; ++f)
            if (!seen[f]) return fail(std::string("missing field `") + names[f] + "`");
        return true;
    }
    bool chunk_list(std::vector<Manifest::Chunk>* out) {
        ws();
        if (peek() != '[') {
            if (peek() < 0) return fail("EOF while parsing a value");
            return fail("invalid type: " + unexpected() + ", expected a sequence");
        }
        if (!enter()) return false;
        out->clear();
        if (peek() == ']') {
            ++i_;
            --depth_;
            return true;
        }
        for (bool more = true; more;) {
            Manifest::Chunk c;
            if (!chunk(&c)) return false;
            out->push_back(std::move(c));
            if (!next(']', &more)) return false;
        }
        return true;
    }

    // ---- ChunkManifest ----------------------------------------------------
    bool field(int f, Manifest& m) {
        uint64_t v = 0;
        switch (f) {
            case 0: return u32(&m.version);
            case 1: return uint(&m.total_size, 64);
            case 2: return uint(&m.chunk_size, 64);
            case 3: return u32(&m.chunk_count);
            case 4: return chunk_list(&m.chunks);
            case 5:
                if (!opt(&m.has_parity, &v, 32)) return false;
                m.parity_shards = uint32_t(v);
                return true;
            case 6: return opt(&m.has_shard, &m.shard_size, 64);
            case 7: return opt(&m.has_plain, &m.plaintext_size, 64);
        }
        return false;
    }
    bool manifest(Manifest& m) {
        static const char* const order[8] = {"version", "total_size", "chunk_size", "chunk_count",
                                             "chunks", "parity_shards", "shard_size", "plaintext_size"};
        m = Manifest{};
        bool seen[8] = {};
        const int open = peek();
        if (open == '[') {
            if (!enter()) return false;
            for (int f = 0; f < 8; ++f) {
                if (peek() == ']') {
                    if (f < 5) return fail("invalid length " + std::to_string(f) + ", expected struct ChunkManifest with 8 elements");
                    break;
                }
                if (!field(f, m)) return false;
                ws();
                if (peek() == ',') {
                    ++i_;
                    ws();
                    if (peek() == ']') return fail("trailing comma");
                    if (f == 7) return fail("trailing characters");
                } else if (peek() != ']') {
                    return fail(peek() < 0 ? "EOF while parsing a list" : "expected `,` or `]`");
                }
            }
            ++i_;
            --depth_;
            return true;
        }
        if (open != '{') {
            if (open < 0) return fail("EOF while parsing a value");
            if (open == '"' || open == 't' || open == 'f' || open == 'n' || open == '-' || (open >= '0' && open <= '9'))
                return fail("invalid type: " + unexpected() + ", expected struct ChunkManifest");
            return fail("expected value");
        }
        if (!enter()) return false;
        bool more = peek() != '}';
        if (!more) {
            ++i_;
            --depth_;
        }
        while (more) {
            if (peek() != '"') return fail(peek() < 0 ? "EOF while parsing an object" : "key must be a string");
            std::string key;
            if (!string(key)) return false;
            ws();
            if (peek() != ':') return fail("expected `:`");
            ++i_;
            int f = -1;
            for (int t = 0; t < 8; ++t)
                if (key == order[t]) f = t;
            if (f >= 0 && seen[f]) return fail(std::string("duplicate field `") + order[f] + "`");
            if (!(f >= 0 ? field(f, m) : skip())) return false;
            if (f >= 0) seen[f] = true;
            if (!next('}', &more)) return false;
        }
        for (int f = 0; f < 5; ++f)
            if (!seen[f]) return fail(std::string("missing field `") + order[f] + "`");
        return true;
    }
};

}  // namespace

bool parse_manifest(const std::string& text, Manifest& m, std::string* err) {
    Reader r(text);
    if (r.document(m)) return true;
    if (err) *err = r.err;
    return false;
}

}  // namespace mxec

/*
 * rs_oracle.c — CPU restatement of reed-solomon-erasure 6.0.0 (galois_8,
 * pure-Rust path, no simd-accel) as called by MaxIO's chunked-EC path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Never linked into maxio_amd.
 *
 * The crate is not vendored under /root/reference (Cargo.toml:57 pins "6",
 * Cargo.lock:1462-1473 resolves 6.0.0).  Restated from its published source:
 *   build.rs       gen_log_table / gen_exp_table / gen_mul_table, poly 29
 *   galois_8.rs    mul, div, exp; mul_slice / mul_slice_add (table lookups)
 *   matrix.rs      vandermonde, multiply, augment, gaussian_elim, invert
 *   core.rs        ReedSolomon::new, build_matrix, encode, code_some_slices,
 *                  reconstruct_internal, get_data_decode_matrix
 * Reference call sites: filesystem.rs:1121-1124 (new+encode),
 * chunk_reader.rs:168,211 (new+reconstruct).
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

#define FIELD_SIZE 256
#define GENERATING_POLYNOMIAL 29

static uint8_t LOG_TABLE[FIELD_SIZE];
static uint8_t EXP_TABLE[(FIELD_SIZE - 1) * 2];
static uint8_t MUL_TABLE[FIELD_SIZE][FIELD_SIZE];
static int tables_ready = 0;

/* build.rs gen_log_table: walk powers of the generator 2, reducing by
 * (b - 256) ^ 29 whenever b overflows 8 bits. */
static void build_tables(void) {
    if (tables_ready) return;
    size_t b = 1;
    memset(LOG_TABLE, 0, sizeof LOG_TABLE);
    for (size_t log = 0; log < FIELD_SIZE - 1; ++log) {
        LOG_TABLE[b] = (uint8_t)log;
        b <<= 1;
        if (b >= FIELD_SIZE) b = (b - FIELD_SIZE) ^ GENERATING_POLYNOMIAL;
    }
    /* gen_exp_table: EXP[LOG[i]] = i, table doubled so LOG[a]+LOG[b] indexes it */
    for (size_t i = 1; i < FIELD_SIZE; ++i) {
        size_t log = LOG_TABLE[i];
        EXP_TABLE[log] = (uint8_t)i;
        EXP_TABLE[log + FIELD_SIZE - 1] = (uint8_t)i;
    }
    /* gen_mul_table: MUL_TABLE[a][b] = mul(a, b) */
    for (size_t a = 0; a < FIELD_SIZE; ++a)
        for (size_t c = 0; c < FIELD_SIZE; ++c)
            MUL_TABLE[a][c] = (a == 0 || c == 0)
                                  ? 0
                                  : EXP_TABLE[LOG_TABLE[a] + LOG_TABLE[c]];
    tables_ready = 1;
}

uint8_t orc_gf_mul(uint8_t a, uint8_t b) {
    build_tables();
    return MUL_TABLE[a][b];
}

/* galois_8::div: a==0 -> 0; log_result = LOG[a] - LOG[b] (+255 if negative) */
uint8_t orc_gf_div(uint8_t a, uint8_t b) {
    build_tables();
    if (a == 0) return 0;
    int log_result = (int)LOG_TABLE[a] - (int)LOG_TABLE[b];
    if (log_result < 0) log_result += 255;
    return EXP_TABLE[log_result];
}

/* galois_8::exp: n==0 -> 1; a==0 -> 0; LOG[a]*n reduced mod 255 by subtraction */
uint8_t orc_gf_exp(uint8_t a, size_t n) {
    build_tables();
    if (n == 0) return 1;
    if (a == 0) return 0;
    size_t log_result = (size_t)LOG_TABLE[a] * n;
    while (log_result >= 255) log_result -= 255;
    return EXP_TABLE[log_result];
}

void orc_gf_tables(uint8_t* exp_out, uint8_t* log_out) {
    build_tables();
    if (exp_out) memcpy(exp_out, EXP_TABLE, sizeof EXP_TABLE);
    if (log_out) memcpy(log_out, LOG_TABLE, sizeof LOG_TABLE);
}

/* ---- matrix.rs ---------------------------------------------------------- */

/* gaussian_elim on a rows x cols row-major matrix (crate order: forward
 * elimination with row swap on a zero pivot, scale pivot row to 1, clear
 * below; then clear above the diagonal). */
static int gaussian_elim(uint8_t* w, int rows, int cols) {
    for (int r = 0; r < rows; ++r) {
        if (w[r * cols + r] == 0) {
            for (int rb = r + 1; rb < rows; ++rb) {
                if (w[rb * cols + r] != 0) {
                    for (int c = 0; c < cols; ++c) {
                        uint8_t t = w[r * cols + c];
                        w[r * cols + c] = w[rb * cols + c];
                        w[rb * cols + c] = t;
                    }
                    break;
                }
            }
        }
        if (w[r * cols + r] == 0) return ORC_E_SINGULAR_MATRIX;
        if (w[r * cols + r] != 1) {
            uint8_t scale = orc_gf_div(1, w[r * cols + r]);
            for (int c = 0; c < cols; ++c)
                w[r * cols + c] = orc_gf_mul(scale, w[r * cols + c]);
        }
        for (int rb = r + 1; rb < rows; ++rb) {
            if (w[rb * cols + r] != 0) {
                uint8_t scale = w[rb * cols + r];
                for (int c = 0; c < cols; ++c)
                    w[rb * cols + c] ^= orc_gf_mul(scale, w[r * cols + c]);
            }
        }
    }
    for (int d = 0; d < rows; ++d) {
        for (int ra = 0; ra < d; ++ra) {
            if (w[ra * cols + d] != 0) {
                uint8_t scale = w[ra * cols + d];
                for (int c = 0; c < cols; ++c)
                    w[ra * cols + c] ^= orc_gf_mul(scale, w[d * cols + c]);
            }
        }
    }
    return ORC_OK;
}

/* Matrix::invert: augment with identity, eliminate, take the right half. */
int orc_matrix_invert(int n, const uint8_t* in, uint8_t* out) {
    if (n <= 0) return ORC_E_INVALID_ARG;
    int cols = 2 * n;
    uint8_t* w = (uint8_t*)calloc((size_t)n * cols, 1);
    if (!w) return ORC_E_INVALID_ARG;
    for (int r = 0; r < n; ++r) {
        memcpy(w + r * cols, in + r * n, (size_t)n);
        w[r * cols + n + r] = 1;
    }
    int rc = gaussian_elim(w, n, cols);
    if (rc == ORC_OK)
        for (int r = 0; r < n; ++r) memcpy(out + r * n, w + r * cols + n, (size_t)n);
    free(w);
    return rc;
}

/* ReedSolomon::new argument checks (core.rs), field order 256. */
int orc_rs_check(int k, int m) {
    if (k <= 0) return ORC_E_TOO_FEW_DATA_SHARDS;
    if (m <= 0) return ORC_E_TOO_FEW_PARITY_SHARDS;
    if (k + m > FIELD_SIZE) return ORC_E_TOO_MANY_SHARDS;
    return ORC_OK;
}

/* build_matrix(k, k+m): vandermonde(k+m, k)[r][c] = exp(r, c), times the
 * inverse of its top k x k square, so the top rows become the identity. */
int orc_rs_matrix(int k, int m, uint8_t* matrix_out) {
    int rc = orc_rs_check(k, m);
    if (rc) return rc;
    int total = k + m;
    uint8_t* v = (uint8_t*)malloc((size_t)total * k);
    uint8_t* top_inv = (uint8_t*)malloc((size_t)k * k);
    for (int r = 0; r < total; ++r)
        for (int c = 0; c < k; ++c) v[r * k + c] = orc_gf_exp((uint8_t)r, (size_t)c);
    rc = orc_matrix_invert(k, v, top_inv); /* top is v's first k rows */
    if (rc == ORC_OK) {
        for (int r = 0; r < total; ++r)
            for (int c = 0; c < k; ++c) {
                uint8_t acc = 0;
                for (int i = 0; i < k; ++i)
                    acc ^= orc_gf_mul(v[r * k + i], top_inv[i * k + c]);
                matrix_out[r * k + c] = acc;
            }
    }
    free(v);
    free(top_inv);
    return rc;
}

/* galois_8 pure-Rust mul_slice / mul_slice_add: one MUL_TABLE row, one
 * lookup per byte. */
static void mul_slice(uint8_t c, const uint8_t* in, uint8_t* out, size_t n) {
    const uint8_t* mt = MUL_TABLE[c];
    for (size_t i = 0; i < n; ++i) out[i] = mt[in[i]];
}
static void mul_slice_add(uint8_t c, const uint8_t* in, uint8_t* out, size_t n) {
    const uint8_t* mt = MUL_TABLE[c];
    for (size_t i = 0; i < n; ++i) out[i] ^= mt[in[i]];
}

/* code_some_slices: for each input (outer), for each output row (inner). */
static void code_some_slices(int n_inputs, int n_outputs, const uint8_t* const* rows,
                             const uint8_t* const* inputs, uint8_t* const* outputs,
                             size_t size) {
    for (int j = 0; j < n_inputs; ++j)
        for (int i = 0; i < n_outputs; ++i) {
            if (j == 0)
                mul_slice(rows[i][j], inputs[j], outputs[i], size);
            else
                mul_slice_add(rows[i][j], inputs[j], outputs[i], size);
        }
}

int orc_rs_encode(int k, int m, size_t size, uint8_t* const* shards) {
    build_tables();
    int rc = orc_rs_check(k, m);
    if (rc) return rc;
    if (!shards) return ORC_E_TOO_FEW_SHARDS;
    if (size == 0) return ORC_E_EMPTY_SHARD;
    uint8_t* mat = (uint8_t*)malloc((size_t)(k + m) * k);
    rc = orc_rs_matrix(k, m, mat);
    if (rc == ORC_OK) {
        const uint8_t** rows = (const uint8_t**)malloc(sizeof(uint8_t*) * m);
        for (int i = 0; i < m; ++i) rows[i] = mat + (size_t)(k + i) * k;
        code_some_slices(k, m, rows, (const uint8_t* const*)shards, shards + k, size);
        free(rows);
    }
    free(mat);
    return rc;
}

/* reconstruct_internal restated.  valid_indices = the first k present
 * shards in index order; the decode matrix is the inverse of those rows of
 * the encoding matrix; missing data rows come from it, missing parity is
 * re-encoded from all (old + rebuilt) data shards. */
int orc_rs_reconstruct(int k, int m, size_t size, uint8_t* const* shards,
                       uint8_t* present, int data_only) {
    build_tables();
    int rc = orc_rs_check(k, m);
    if (rc) return rc;
    int total = k + m;
    if (size == 0) return ORC_E_EMPTY_SHARD;
    int number_present = 0;
    for (int i = 0; i < total; ++i) number_present += present[i] ? 1 : 0;
    if (number_present == total) return ORC_OK;
    if (number_present < k) return ORC_E_TOO_FEW_SHARDS_PRESENT;

    uint8_t* mat = (uint8_t*)malloc((size_t)total * k);
    uint8_t* sub = (uint8_t*)malloc((size_t)k * k);
    uint8_t* dec = (uint8_t*)malloc((size_t)k * k);
    int* valid = (int*)malloc(sizeof(int) * total);
    int* invalid = (int*)malloc(sizeof(int) * total);
    int nvalid = 0, ninvalid = 0;
    rc = orc_rs_matrix(k, m, mat);
    if (rc) goto out;

    for (int r = 0; r < total; ++r) {
        if (present[r]) {
            if (nvalid < k) valid[nvalid++] = r;
        } else if (!(r >= k && data_only)) {
            memset(shards[r], 0, size); /* get_or_initialize */
            invalid[ninvalid++] = r;
        } else {
            invalid[ninvalid++] = r;
        }
    }
    for (int r = 0; r < k; ++r) memcpy(sub + r * k, mat + (size_t)valid[r] * k, (size_t)k);
    rc = orc_matrix_invert(k, sub, dec);
    if (rc) goto out;

    {
        const uint8_t** rows = (const uint8_t**)malloc(sizeof(uint8_t*) * total);
        const uint8_t** ins = (const uint8_t**)malloc(sizeof(uint8_t*) * total);
        uint8_t** outs = (uint8_t**)malloc(sizeof(uint8_t*) * total);
        int nout = 0;
        for (int v = 0; v < k; ++v) ins[v] = shards[valid[v]];
        for (int t = 0; t < ninvalid && invalid[t] < k; ++t) {
            rows[nout] = dec + (size_t)invalid[t] * k;
            outs[nout++] = shards[invalid[t]];
        }
        if (nout) code_some_slices(k, nout, rows, ins, outs, size);
        if (!data_only) {
            /* all data shards are now intact in shards[0..k) */
            nout = 0;
            for (int t = 0; t < ninvalid; ++t) {
                if (invalid[t] < k) continue;
                rows[nout] = mat + (size_t)invalid[t] * k;
                outs[nout++] = shards[invalid[t]];
            }
            if (nout) code_some_slices(k, nout, rows, (const uint8_t* const*)shards, outs, size);
        }
        for (int t = 0; t < ninvalid; ++t)
            if (invalid[t] < k || !data_only) present[invalid[t]] = 1;
        free(rows);
        free(ins);
        free(outs);
    }
out:
    free(mat);
    free(sub);
    free(dec);
    free(valid);
    free(invalid);
    return rc;
}

/* filesystem.rs:1084-1145 without the disk: guard k+m>255 (:1095), pad each
 * data chunk to chunk_size (:1108-1113), zeroed parity (:1116-1118),
 * ReedSolomon::new + encode (:1121-1124), sha256 of each full parity shard
 * (:1131).  Data digests are write_chunk's (:1070) over unpadded bytes. */
/* The digest function of the composite calls: the scalar restatement (the
 * checker) or, for the timed CPU baseline, the SHA-NI form sha2 0.10.9
 * auto-selects on x86-64 (orc_sha256_fast; scalar where the host lacks it). */
static void sha_scalar(const uint8_t* p, size_t n, uint8_t out[32]) { orc_sha256(p, n, out); }
static void sha_ni(const uint8_t* p, size_t n, uint8_t out[32]) { (void)orc_sha256_fast(p, n, out); }

int orc_compute_parity_ex(int k, int m, size_t chunk_size,
                          const uint8_t* const* data, const size_t* data_len,
                          uint8_t* const* parity, uint8_t* sha_out, int use_sha_ni) {
    void (*sha)(const uint8_t*, size_t, uint8_t*) = use_sha_ni ? sha_ni : sha_scalar;
    if (k + m > 255) return ORC_E_TOO_MANY_SHARDS_255;
    int rc = orc_rs_check(k, m);
    if (rc) return rc;
    uint8_t** shards = (uint8_t**)malloc(sizeof(uint8_t*) * (k + m));
    for (int j = 0; j < k; ++j) {
        if (data_len[j] > chunk_size) { rc = ORC_E_INVALID_ARG; break; }
        shards[j] = (uint8_t*)calloc(chunk_size ? chunk_size : 1, 1);
        memcpy(shards[j], data[j], data_len[j]);
        if (sha_out) sha(data[j], data_len[j], sha_out + 32 * j);
    }
    if (rc == ORC_OK) {
        for (int i = 0; i < m; ++i) {
            shards[k + i] = parity[i];
            memset(parity[i], 0, chunk_size);
        }
        rc = orc_rs_encode(k, m, chunk_size, shards);
        if (rc == ORC_OK && sha_out)
            for (int i = 0; i < m; ++i) sha(parity[i], chunk_size, sha_out + 32 * (k + i));
    }
    for (int j = 0; j < k; ++j) free(shards[j]);
    free(shards);
    return rc;
}

int orc_compute_parity(int k, int m, size_t chunk_size,
                       const uint8_t* const* data, const size_t* data_len,
                       uint8_t* const* parity, uint8_t* sha_out) {
    return orc_compute_parity_ex(k, m, chunk_size, data, data_len, parity, sha_out, 0);
}

/* chunk_reader.rs:157-226 without the disk: every shard is hashed and
 * compared to the manifest digest (:176-196); mismatches / missing files
 * become None; present ones are padded to shard_size; present < k is an
 * error (:199-208); reconstruct (:211); return target truncated (:216-222). */
int orc_try_reconstruct_data_chunk_ex(int k, int m, size_t shard_size,
                                      const uint8_t* const* shards,
                                      const size_t* shard_len,
                                      const uint8_t* expected_sha,
                                      const uint64_t* chunk_sizes, int target,
                                      uint8_t* out, int* n_present, int use_sha_ni) {
    void (*sha)(const uint8_t*, size_t, uint8_t*) = use_sha_ni ? sha_ni : sha_scalar;
    int rc = orc_rs_check(k, m);
    if (rc) return rc;
    if (target < 0 || target >= k + m) return ORC_E_INVALID_INDEX;
    int total = k + m;
    uint8_t** bufs = (uint8_t**)malloc(sizeof(uint8_t*) * total);
    uint8_t* present = (uint8_t*)calloc((size_t)total, 1);
    int np = 0;
    for (int i = 0; i < total; ++i) {
        bufs[i] = (uint8_t*)calloc(shard_size ? shard_size : 1, 1);
        if (!shards[i]) continue;
        uint8_t d[32];
        sha(shards[i], shard_len[i], d);
        if (memcmp(d, expected_sha + 32 * i, 32) != 0) continue;
        /* Vec::resize(shard_size): pad, or truncate if longer */
        size_t n = shard_len[i] < shard_size ? shard_len[i] : shard_size;
        memcpy(bufs[i], shards[i], n);
        present[i] = 1;
        ++np;
    }
    if (n_present) *n_present = np;
    if (np < k) {
        rc = ORC_E_TOO_FEW_SHARDS_PRESENT;
    } else {
        rc = orc_rs_reconstruct(k, m, shard_size, bufs, present, 0);
        if (rc == ORC_OK) {
            size_t real = (size_t)chunk_sizes[target];
            if (real > shard_size) real = shard_size;
            memcpy(out, bufs[target], real);
        }
    }
    for (int i = 0; i < total; ++i) free(bufs[i]);
    free(bufs);
    free(present);
    return rc;
}

int orc_try_reconstruct_data_chunk(int k, int m, size_t shard_size,
                                   const uint8_t* const* shards,
                                   const size_t* shard_len,
                                   const uint8_t* expected_sha,
                                   const uint64_t* chunk_sizes, int target,
                                   uint8_t* out, int* n_present) {
    return orc_try_reconstruct_data_chunk_ex(k, m, shard_size, shards, shard_len, expected_sha, chunk_sizes,
                                             target, out, n_present, 0);
}

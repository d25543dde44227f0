/* put_get.c — a plain C99 client of libmaxio_ec, as MaxIO's Rust FFI would
 * drive it: PutObject with --erasure-coding into chunk files
 * plus manifest.json, lose / rot shards, GetObject through the verified
 * reader, compare.  Built and run by tests/test_c_client.py.
 *
 *   put_get <scratch dir>      exit 0 and "c client ok" on success
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "maxio_ec.h"

#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                  \
            fprintf(stderr, " (%s)\n", mxec_last_error()); \
            exit(1);                                       \
        }                                                  \
    } while (0)

static uint8_t* body_of(size_t n, uint32_t seed) {
    uint8_t* b = malloc(n ? n : 1);
    uint64_t x = 0x9E3779B97F4A7C15ull ^ seed;
    for (size_t i = 0; i < n; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        b[i] = (uint8_t)(x >> 24);
    }
    return b;
}

/* GET through the pull reader in 256 KiB reads (ReaderStream's size,
 * object.rs:906) and compare with want[offset, offset + length). */
static void get_and_compare(mxec_ctx* ctx, const char* dir, const uint8_t* want, uint64_t offset,
                            uint64_t length) {
    mxec_reader* r = NULL;
    int rc = mxec_reader_open(ctx, dir, offset, length, 0, &r);
    CHECK(rc == 0, "reader_open %s rc=%d", dir, rc);
    uint8_t* buf = malloc(256 << 10);
    uint64_t got = 0;
    for (;;) {
        int64_t n = mxec_reader_read(r, buf, 256 << 10);
        CHECK(n >= 0, "reader_read %s rc=%lld", dir, (long long)n);
        if (n == 0) break;
        CHECK(got + (uint64_t)n <= length, "reader overran the range");
        CHECK(memcmp(buf, want + offset + got, (size_t)n) == 0, "GET bytes differ at %llu",
              (unsigned long long)(offset + got));
        got += (uint64_t)n;
    }
    CHECK(got == length, "GET returned %llu of %llu bytes", (unsigned long long)got,
          (unsigned long long)length);
    mxec_reader_close(r);
    free(buf);
}

static void path(char* out, size_t cap, const char* dir, const char* leaf) {
    snprintf(out, cap, "%s/%s", dir, leaf);
}

int main(int argc, char** argv) {
    CHECK(argc == 2, "usage: put_get <scratch dir>");
    mxec_ctx* ctx = mxec_open(1, 2);
    CHECK(ctx != NULL, "mxec_open");
    char dir[4096], f[4200];

    /* BASELINE configs[0]: one 10 MiB object, --chunk-size 10485760
     * --parity-shards 2; delete shard 000000; GET rebuilds it. */
    {
        const size_t n = 10u << 20;
        uint8_t* body = body_of(n, 1);
        snprintf(dir, sizeof dir, "%s/cfg1.ec", argv[1]);
        mxec_body_sums sums;
        int rc = mxec_put_object_chunked_sums(ctx, dir, 10485760, 2, body, n,
                                              MXEC_SUM_MD5 | MXEC_SUM_CRC32C, &sums);
        CHECK(rc == 0, "put cfg1 rc=%d", rc);
        path(f, sizeof f, dir, "000002");
        struct stat st;
        CHECK(stat(f, &st) == 0 && (size_t)st.st_size == n, "parity file 000002");
        path(f, sizeof f, dir, "000000");
        CHECK(unlink(f) == 0, "delete 000000");
        get_and_compare(ctx, dir, body, 0, n);
        free(body);
    }
    /* 3.5 MiB at 1 MiB chunks, 2 parity: bitrot in chunk 1, a deleted parity
     * shard, then full and ranged GETs. */
    {
        const size_t n = (7u << 20) / 2;
        uint8_t* body = body_of(n, 2);
        snprintf(dir, sizeof dir, "%s/rot.ec", argv[1]);
        int rc = mxec_put_object_chunked(ctx, dir, 1 << 20, 2, body, n);
        CHECK(rc == 0, "put rot rc=%d", rc);
        path(f, sizeof f, dir, "000001");
        FILE* fp = fopen(f, "r+b");
        CHECK(fp != NULL, "open 000001");
        fseek(fp, 12345, SEEK_SET);
        fputc(0x5A ^ body[(1 << 20) + 12345], fp);
        fclose(fp);
        path(f, sizeof f, dir, "000005");
        CHECK(unlink(f) == 0, "delete 000005");
        get_and_compare(ctx, dir, body, 0, n);
        get_and_compare(ctx, dir, body, 1000000, 1500000);
        uint8_t* whole = malloc(n);
        uint64_t got = 0;
        rc = mxec_get_object_chunked(ctx, dir, 0, UINT64_MAX, whole, n, &got);
        CHECK(rc == 0 && got == n && memcmp(whole, body, n) == 0, "get_object_chunked rc=%d", rc);
        /* three chunks lost of a 4 + 2 object: the reference's error */
        path(f, sizeof f, dir, "000000"); unlink(f);
        path(f, sizeof f, dir, "000002"); unlink(f);
        rc = mxec_get_object_chunked(ctx, dir, 0, UINT64_MAX, whole, n, &got);
        CHECK(rc != 0, "GET with 4 of 6 shards gone must fail");
        free(whole);
        free(body);
    }
    mxec_close(ctx);
    printf("c client ok\n");
    return 0;
}

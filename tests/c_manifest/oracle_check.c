/* oracle_check — runs the C oracle (the oracle/ sources, test infrastructure) under
 * -fsanitize=address,undefined: RS encode + every 1- and 2-erasure
 * reconstruct at 8+4 and 4+2 with ragged sizes, the chunk-level helpers,
 * SHA-256 / SHA-1 / MD5 / CRC32 / CRC32C at every length 0..300, and an
 * AES-256-GCM round trip.  Built by tests/test_manifest_strict.py.  Prints
 * "oracle_check ok" and exits 0 when every internal consistency check holds. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/oracle.h"

static unsigned long long st = 0x6D6178696FULL;
static uint8_t rnd(void) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return (uint8_t)st;
}

static int rs_case(int k, int m, size_t size) {
    int n = k + m, fails = 0;
    uint8_t** sh = calloc((size_t)n, sizeof(uint8_t*));
    uint8_t** orig = malloc(sizeof(uint8_t*) * (size_t)n);
    for (int i = 0; i < n; ++i) {
        sh[i] = malloc(size);
        orig[i] = malloc(size);
        for (size_t b = 0; b < size; ++b) sh[i][b] = rnd();
    }
    if (orc_rs_encode(k, m, size, sh) != ORC_OK) fails++;
    for (int i = 0; i < n; ++i) memcpy(orig[i], sh[i], size);
    uint8_t* present = malloc((size_t)n);
    for (int a = 0; a < n; ++a)
        for (int b = a; b < n; ++b) {
            for (int i = 0; i < n; ++i) present[i] = 1;
            present[a] = present[b] = 0;
            memset(sh[a], 0, size);
            memset(sh[b], 0, size);
            if (orc_rs_reconstruct(k, m, size, sh, present, 0) != ORC_OK) fails++;
            for (int i = 0; i < n; ++i)
                if (memcmp(sh[i], orig[i], size)) fails++;
        }
    /* too few present */
    for (int i = 0; i < n; ++i) present[i] = i < k - 1;
    if (orc_rs_reconstruct(k, m, size, sh, present, 0) != ORC_E_TOO_FEW_SHARDS_PRESENT) fails++;
    /* chunk-level: compute_parity over ragged data, then try_reconstruct */
    size_t* dl = malloc(sizeof(size_t) * (size_t)k);
    uint64_t* cs = malloc(sizeof(uint64_t) * (size_t)n);
    size_t* sl = malloc(sizeof(size_t) * (size_t)n);
    for (int j = 0; j < k; ++j) dl[j] = j == k - 1 ? size / 3 + 1 : size;
    uint8_t* sha = malloc(32 * (size_t)n);
    if (orc_compute_parity(k, m, size, (const uint8_t* const*)orig, dl, sh + k, sha) != ORC_OK) fails++;
    for (int i = 0; i < n; ++i) {
        cs[i] = i < k ? dl[i] : size;
        sl[i] = (size_t)cs[i];
    }
    const uint8_t** in = malloc(sizeof(uint8_t*) * (size_t)n);
    for (int i = 0; i < n; ++i) in[i] = i < k ? orig[i] : sh[i];
    in[0] = NULL;
    uint8_t* out = malloc(size);
    int np = 0;
    if (orc_try_reconstruct_data_chunk(k, m, size, in, sl, sha, cs, 0, out, &np) != ORC_OK || memcmp(out, orig[0], dl[0]))
        fails++;
    free(out);
    free(in);
    free(sha);
    free(sl);
    free(cs);
    free(dl);
    free(present);
    for (int i = 0; i < n; ++i) {
        free(sh[i]);
        free(orig[i]);
    }
    free(sh);
    free(orig);
    return fails;
}

int main(void) {
    int fails = 0;
    fails += rs_case(4, 2, 1000);
    fails += rs_case(8, 4, 4096 + 17);
    fails += rs_case(10, 4, 333);
    fails += rs_case(1, 2, 64);
    if (orc_rs_check(200, 57) != ORC_E_TOO_MANY_SHARDS) fails++; /* crate: k+m > 256 */
    uint8_t buf[300], d1[32], d2[32], h20[20], h16[16];
    for (int i = 0; i < 300; ++i) buf[i] = rnd();
    for (size_t n = 0; n <= 300; ++n) {
        orc_sha256(buf, n, d1);
        if (orc_sha256_fast(buf, n, d2) == 0 && memcmp(d1, d2, 32)) fails++;
        orc_sha1(buf, n, h20);
        orc_md5(buf, n, h16);
        if (orc_crc32c_append(0, buf, n) != orc_crc32c_append_fast(0, buf, n)) fails++;
        (void)orc_crc32(buf, n);
    }
    uint8_t key[32], iv[12], aad[40], ct[300], pt[300], tag[16];
    for (int i = 0; i < 32; ++i) key[i] = rnd();
    for (int i = 0; i < 12; ++i) iv[i] = rnd();
    for (int i = 0; i < 40; ++i) aad[i] = rnd();
    if (orc_gcm_encrypt(key, iv, aad, 40, buf, 300, ct, tag) != 0) fails++;
    if (orc_gcm_decrypt(key, iv, aad, 40, ct, 300, tag, pt) != 0 || memcmp(pt, buf, 300)) fails++;
    tag[0] ^= 1;
    if (orc_gcm_decrypt(key, iv, aad, 40, ct, 300, tag, pt) == 0) fails++;
    if (fails) {
        printf("oracle_check FAILED: %d\n", fails);
        return 1;
    }
    printf("oracle_check ok\n");
    return 0;
}

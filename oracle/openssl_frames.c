/*
 * openssl_frames.c — CPU BASELINE ONLY (see oracle.h): FrameEncryptor's work
 * (crypto.rs:94-117) through OpenSSL's EVP_aes_256_gcm (AES-NI + PCLMUL, the
 * same instruction paths the aes-gcm crate autodetects), looped in C so a
 * multi-threaded timing is not serialised by the Python interpreter.
 * Never a checker: the frame oracle is gcm_oracle.c.
 */
#include <openssl/evp.h>
#include <stdint.h>
#include <string.h>

int orc_ssl_frames_encrypt(const uint8_t key[32], const uint8_t prefix[4], const uint8_t* aad, size_t aad_len,
                           size_t frame_size, const uint8_t* pt, size_t len, uint8_t* out) {
    EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
    if (!c) return -1;
    int rc = 0;
    if (EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), NULL, key, NULL) != 1) rc = -1;
    size_t f = 0;
    for (size_t off = 0; rc == 0 && off < len; off += frame_size, ++f) {
        const size_t n = len - off < frame_size ? len - off : frame_size;
        uint8_t* fr = out + f * (frame_size + 28);
        memcpy(fr, prefix, 4);
        for (int j = 0; j < 8; ++j) fr[4 + j] = (uint8_t)((uint64_t)f >> (8 * j));
        int outl = 0;
        if (EVP_EncryptInit_ex(c, NULL, NULL, NULL, fr) != 1) rc = -1;
        if (rc == 0 && aad_len && EVP_EncryptUpdate(c, NULL, &outl, aad, (int)aad_len) != 1) rc = -1;
        if (rc == 0 && EVP_EncryptUpdate(c, fr + 12, &outl, pt + off, (int)n) != 1) rc = -1;
        if (rc == 0 && EVP_EncryptFinal_ex(c, fr + 12 + outl, &outl) != 1) rc = -1;
        if (rc == 0 && EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, fr + 12 + n) != 1) rc = -1;
    }
    EVP_CIPHER_CTX_free(c);
    return rc;
}

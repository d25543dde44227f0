"""CPU: pin the encrypt-then-EC frame oracle (oracle/gcm_oracle.c) — AES-256
(FIPS-197), GCM (SP 800-38D) and the crypto.rs frame layout — against the
published vectors and against OpenSSL's EVP_aes_256_gcm (an independent
implementation, loaded from the system libcrypto).  No GPU."""
from __future__ import annotations

import numpy as np
import pytest

import openssl_gcm
import oracle

needs_openssl = pytest.mark.skipif(openssl_gcm.lib() is None, reason="libcrypto not loadable")


def _rand(n: int, seed: int) -> bytes:
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def test_fips197_aes256_vector():
    # FIPS-197 Appendix C.3
    key = bytes(range(32))
    assert oracle.aes256_block(key, bytes.fromhex("00112233445566778899aabbccddeeff")).hex() == \
        "8ea2b7ca516745bfeafc49904b496089"


def test_gcm_published_cases():
    # McGrew & Viega GCM spec, test cases 13 and 14 (AES-256, zero key and IV).
    key, iv = bytes(32), bytes(12)
    ct, tag = oracle.gcm_encrypt(key, iv, b"")
    assert ct == b"" and tag.hex() == "530f8afbc74536b9a963b4f1c4cb738b"
    ct, tag = oracle.gcm_encrypt(key, iv, bytes(16))
    assert ct.hex() == "cea7403d4d606b6e074ec5d3baf39d18"
    assert tag.hex() == "d0d1c8a799996bf0265b98b5d48ab919"


@needs_openssl
@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 100, 4096, 65536, 65537])
@pytest.mark.parametrize("aad_len", [0, 20, 32])
def test_gcm_matches_openssl(n, aad_len):
    key, iv = _rand(32, 1 + n), _rand(12, 2 + n)
    pt, aad = _rand(n, 3 + n), _rand(aad_len, 4 + n)
    ct, tag = oracle.gcm_encrypt(key, iv, pt, aad)
    assert (ct, tag) == openssl_gcm.encrypt(key, iv, pt, aad)
    assert oracle.gcm_decrypt(key, iv, ct, tag, aad) == pt
    bad = bytes([tag[0] ^ 1]) + tag[1:]
    assert oracle.gcm_decrypt(key, iv, ct, bad, aad) is None
    assert openssl_gcm.decrypt(key, iv, ct, bad, aad) is None


def test_gf128_mul_is_commutative_and_distributive():
    a, b, c = _rand(16, 5), _rand(16, 6), _rand(16, 7)
    assert oracle.gf128_mul(a, b) == oracle.gf128_mul(b, a)
    bc = bytes(x ^ y for x, y in zip(b, c))
    lhs = oracle.gf128_mul(a, bc)
    rhs = bytes(x ^ y for x, y in zip(oracle.gf128_mul(a, b), oracle.gf128_mul(a, c)))
    assert lhs == rhs


@needs_openssl
@pytest.mark.parametrize("n", [0, 23, 65536, 2 * 65536 + 1000])
def test_frames_layout_and_round_trip(n):
    """crypto.rs tests round_trip_small/empty/multi_frame: frame = nonce(prefix
    || index LE) || ciphertext || tag; len = n + 28 per frame; each frame is
    an independent AES-256-GCM message (checked with OpenSSL)."""
    key, prefix = bytes([0x42]) * 32, bytes([1, 2, 3, 4])
    pt = bytes(i % 256 for i in range(n))
    fs = oracle.FRAME_CHUNK_SIZE
    nfr = (n + fs - 1) // fs
    aads = [oracle.frame_aad(oracle.object_aad_prefix("bkt", "obj/key", None), i) for i in range(nfr)]
    out = oracle.frames_encrypt(key, prefix, pt, aads)
    assert len(out) == n + 28 * nfr
    for i in range(nfr):
        fr = out[i * (fs + 28):(i + 1) * (fs + 28)]
        ln = min(fs, n - i * fs)
        assert fr[:12] == prefix + i.to_bytes(8, "little")
        ct, tag = openssl_gcm.encrypt(key, fr[:12], pt[i * fs:i * fs + ln], aads[i])
        assert fr[12:12 + ln] == ct and fr[12 + ln:12 + ln + 16] == tag
    rc, back = oracle.frames_decrypt(key, out, n, aads)
    assert rc == 0 and back == pt


def test_frames_errors():
    key, prefix = bytes([7]) * 32, b"abcd"
    pt = _rand(3 * 1000, 9)
    out = bytearray(oracle.frames_encrypt(key, prefix, pt, frame_size=1000))
    # frame swap -> index mismatch (crypto.rs:330-340)
    f0, f1 = bytes(out[:1028]), bytes(out[1028:2056])
    swapped = f1 + f0 + bytes(out[2056:])
    assert oracle.frames_decrypt(key, swapped, 3000, frame_size=1000)[0] == -44
    # flipped ciphertext bit -> authentication error (:355-360)
    out[1028 + 12 + 5] ^= 0x10
    assert oracle.frames_decrypt(key, bytes(out), 3000, frame_size=1000)[0] == -41
    # wrong AAD (cross-object swap) -> authentication error
    good = oracle.frames_encrypt(key, prefix, pt[:500], [b"A" * 32], frame_size=1000)
    assert oracle.frames_decrypt(key, good, 500, [b"B" * 32], frame_size=1000)[0] == -41

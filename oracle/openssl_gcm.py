# TEST / BASELINE INFRASTRUCTURE ONLY (see oracle.h): never imported by maxio_amd.
"""AES-256-GCM through the system OpenSSL (libcrypto.so.3, EVP API) via
ctypes — an independent implementation used only to pin the oracle
(tests/test_oracle_gcm.py).  None if libcrypto is not loadable."""
from __future__ import annotations

import ctypes
import ctypes.util
from typing import Optional

_lib = None


def lib():
    global _lib
    if _lib is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        try:
            L = ctypes.CDLL(name)
        except OSError:
            return None
        L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        L.EVP_aes_256_gcm.restype = ctypes.c_void_p
        for fn in ("EVP_EncryptInit_ex", "EVP_DecryptInit_ex"):
            getattr(L, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                       ctypes.c_char_p]
        for fn in ("EVP_EncryptUpdate", "EVP_DecryptUpdate"):
            getattr(L, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                       ctypes.c_char_p, ctypes.c_int]
        for fn in ("EVP_EncryptFinal_ex", "EVP_DecryptFinal_ex"):
            getattr(L, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _lib = L
    return _lib


EVP_CTRL_GCM_GET_TAG = 0x10
EVP_CTRL_GCM_SET_TAG = 0x11


def encrypt(key: bytes, iv: bytes, pt: bytes, aad: bytes = b"") -> tuple[bytes, bytes]:
    L = lib()
    c = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_EncryptInit_ex(c, L.EVP_aes_256_gcm(), None, key, iv) == 1
        n = ctypes.c_int(0)
        if aad:
            assert L.EVP_EncryptUpdate(c, None, ctypes.byref(n), aad, len(aad)) == 1
        out = ctypes.create_string_buffer(len(pt) + 16)
        assert L.EVP_EncryptUpdate(c, out, ctypes.byref(n), pt, len(pt)) == 1
        total = n.value
        assert L.EVP_EncryptFinal_ex(c, ctypes.byref(out, total), ctypes.byref(n)) == 1
        tag = ctypes.create_string_buffer(16)
        assert L.EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, tag) == 1
        return out.raw[:total], tag.raw
    finally:
        L.EVP_CIPHER_CTX_free(c)


def decrypt(key: bytes, iv: bytes, ct: bytes, tag: bytes, aad: bytes = b"") -> Optional[bytes]:
    L = lib()
    c = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_DecryptInit_ex(c, L.EVP_aes_256_gcm(), None, key, iv) == 1
        n = ctypes.c_int(0)
        if aad:
            assert L.EVP_DecryptUpdate(c, None, ctypes.byref(n), aad, len(aad)) == 1
        out = ctypes.create_string_buffer(len(ct) + 16)
        assert L.EVP_DecryptUpdate(c, out, ctypes.byref(n), ct, len(ct)) == 1
        total = n.value
        t = ctypes.create_string_buffer(tag, 16)
        assert L.EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, t) == 1
        if L.EVP_DecryptFinal_ex(c, ctypes.byref(out, total), ctypes.byref(n)) != 1:
            return None
        return out.raw[:total]
    finally:
        L.EVP_CIPHER_CTX_free(c)


_ssl_frames = None


def frames_encrypt_fn():
    """orc_ssl_frames_encrypt from oracle/build/liboracle_ssl.so (CPU baseline),
    or None."""
    global _ssl_frames
    if _ssl_frames is None:
        import os

        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "liboracle_ssl.so")
        try:
            L = ctypes.CDLL(path)
        except OSError:
            return None
        f = L.orc_ssl_frames_encrypt
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        f.restype = ctypes.c_int
        _ssl_frames = f
    return _ssl_frames

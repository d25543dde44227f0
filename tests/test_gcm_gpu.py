"""GPU: encrypt-then-EC frames (mxec_frames_*, gcm_kernel.hip) against the
oracle (oracle/gcm_oracle.c, pinned to OpenSSL and the published vectors by
tests/test_oracle_gcm.py) — bit-exact frame streams, and the decryptor's
error cases from crypto.rs (index mismatch, tag mismatch, truncation)."""
from __future__ import annotations

import numpy as np
import pytest

import maxio_amd
import oracle

pytestmark = pytest.mark.gpu

FS = oracle.FRAME_CHUNK_SIZE


def _rand(n: int, seed: int) -> bytes:
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 23, 1000, FS - 1, FS, FS + 1, 2 * FS + 1000, 5 * FS])
@pytest.mark.parametrize("aad", ["none", "object"])
def test_frames_encrypt_matches_oracle(ctx, n, aad):
    key, prefix = _rand(32, n), bytes([1, 2, 3, 4])
    pt = _rand(n, 100 + n)
    nfr = (n + FS - 1) // FS
    aads = None
    if aad == "object":
        aads = [oracle.frame_aad(oracle.object_aad_prefix("bucket", "k/e/y", "v1"), i) for i in range(nfr)] or None
    got = ctx.frames_encrypt(key, prefix, pt, aads)
    assert got == oracle.frames_encrypt(key, prefix, pt, aads)
    assert ctx.frames_decrypt(key, got, n, aads) == pt


def test_frame_aads_match_reference_builder(ctx):
    pre = oracle.object_aad_prefix("bkt", "photos/a.jpg", None)
    assert ctx.frame_aads(pre, 7, 5) == [oracle.frame_aad(pre, 7 + i) for i in range(5)]
    part = b"PART\0" + b"upload-1" + b"\0" + (3).to_bytes(4, "little") + b"\0"
    assert ctx.frame_aads(part, 0, 3) == [oracle.frame_aad(part, i) for i in range(3)]


def test_small_frames_and_first_index(ctx):
    """frame_size 1024 (the decryptor takes chunk_size as a parameter) and a
    stream starting at index 5 (range reads start mid-object)."""
    key, prefix = _rand(32, 1), b"wxyz"
    pt = _rand(10 * 1024 + 77, 2)
    aads = [bytes([i]) * 32 for i in range(11)]
    got = ctx.frames_encrypt(key, prefix, pt, aads, first_index=5, frame_size=1024)
    assert got == oracle.frames_encrypt(key, prefix, pt, aads, first_index=5, frame_size=1024)
    assert ctx.frames_decrypt(key, got, len(pt), aads, first_index=5, frame_size=1024) == pt


def test_large_frames_long_counters(ctx):
    """Frames of more than 65534 blocks (counters past 2^16) take the generic
    AES path instead of the per-frame counter constants; both must match."""
    key, prefix = _rand(32, 9), b"LONG"
    fs = 65535 * 16  # 65535 blocks: the last counter is 65536
    pt = _rand(fs + 4096 + 5, 10)
    got = ctx.frames_encrypt(key, prefix, pt, first_index=2, frame_size=fs)
    assert got == oracle.frames_encrypt(key, prefix, pt, first_index=2, frame_size=fs)
    assert ctx.frames_decrypt(key, got, len(pt), first_index=2, frame_size=fs) == pt


def test_decrypt_errors(ctx):
    key, prefix = _rand(32, 3), b"abcd"
    pt = _rand(3 * 1000, 4)
    fr = bytearray(ctx.frames_encrypt(key, prefix, pt, frame_size=1008))
    fl = 1008 + 28
    # frames 0 and 1 swapped: index check first (crypto.rs:330-340)
    sw = bytes(fr[fl:2 * fl]) + bytes(fr[:fl]) + bytes(fr[2 * fl:])
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.frames_decrypt(key, sw, len(pt), frame_size=1008)
    assert e.value.name == "Integrity" and "frame index mismatch: expected 0, got 1" in str(e.value)
    # one flipped ciphertext bit (:355-360)
    bad = bytearray(fr)
    bad[fl + 12 + 100] ^= 4
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.frames_decrypt(key, bytes(bad), len(pt), frame_size=1008)
    assert "AES-GCM decryption failed: authentication error" in str(e.value)
    # wrong AAD: a frame moved to another object does not authenticate
    with pytest.raises(maxio_amd.RSError):
        ctx.frames_decrypt(key, bytes(fr), len(pt), [b"x" * 32] * 3, frame_size=1008)
    # truncated stream
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.frames_decrypt(key, bytes(fr[:-1]), len(pt), frame_size=1008)
    assert "truncated encrypted frame" in str(e.value)


def test_device_batch_many_objects(ctx):
    """Several objects with their own keys in one launch; decrypt status per job."""
    import torch

    jobs, refs, bufs = [], [], []
    sizes = [1, 4000, FS, 3 * FS + 5, 100_000]
    for i, n in enumerate(sizes):
        key, pre = _rand(32, 50 + i), bytes([i, 0, 0, 1])
        pt = _rand(n, 60 + i)
        total = oracle.frames_len(n)
        src = torch.frombuffer(bytearray(pt), dtype=torch.uint8).cuda()
        dst = torch.zeros(total, dtype=torch.uint8, device="cuda")
        bufs += [src, dst]
        jobs.append({"key": key, "nonce_prefix": pre, "in_dev": src.data_ptr(), "len": n,
                     "out_dev": dst.data_ptr(), "first_index": i})
        refs.append((key, pre, pt, dst, i))
    ctx.frames_device(jobs)
    torch.cuda.synchronize()
    back_jobs = []
    for key, pre, pt, dst, first in refs:
        got = dst.cpu().numpy().tobytes()
        assert got == oracle.frames_encrypt(key, pre, pt, first_index=first)
        out = torch.zeros(max(1, len(pt)), dtype=torch.uint8, device="cuda")
        bufs.append(out)
        back_jobs.append({"key": key, "in_dev": dst.data_ptr(), "len": len(pt), "out_dev": out.data_ptr(),
                          "first_index": first})
    # corrupt job 2's ciphertext
    refs[2][3][12 + 7] ^= 1
    st = ctx.frames_device(back_jobs, decrypt=True)
    assert st[2] != 0 and all(s == 0 for i, s in enumerate(st) if i != 2)
    for (key, pre, pt, dst, first), j in zip(refs, back_jobs):
        if first != 2:
            got = bufs[-len(back_jobs) + first][:len(pt)].cpu().numpy().tobytes()
            assert got == pt


def test_device_batch_full_chip_every_frame(ctx):
    """Enough frames to keep every workgroup busy for many iterations (the
    bench's shape, scaled down): 48 objects x 41 frames with per-frame AADs,
    every frame of every object compared with the oracle.  Catches races
    between a workgroup's waves (they drift apart over a long grid-stride)."""
    import torch

    n_obj, n = 48, 40 * FS + 1234
    rng = np.random.default_rng(7)
    nfr = (n + FS - 1) // FS
    pt = torch.randint(0, 256, (n_obj, n), dtype=torch.uint8, device="cuda")
    fl = oracle.frames_len(n)
    fr = torch.zeros((n_obj, fl), dtype=torch.uint8, device="cuda")
    aad = torch.from_numpy(rng.integers(0, 256, (n_obj, nfr, 32), dtype=np.uint8)).cuda()
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(n_obj)]
    jobs = [{"key": keys[o], "nonce_prefix": bytes([o, 1, 2, 3]), "aad_dev": aad[o].data_ptr(), "aad_len": 32,
             "in_dev": pt[o].data_ptr(), "len": n, "out_dev": fr[o].data_ptr()} for o in range(n_obj)]
    for _ in range(2):  # twice: the second run starts with warm tables and clocks
        fr.zero_()
        ctx.frames_device(jobs)
        torch.cuda.synchronize()
        host_pt, host_fr, host_aad = pt.cpu().numpy(), fr.cpu().numpy(), aad.cpu().numpy()
        for o in range(n_obj):
            want = oracle.frames_encrypt(keys[o], bytes([o, 1, 2, 3]), host_pt[o],
                                         [bytes(x) for x in host_aad[o]])
            assert host_fr[o].tobytes() == want, o

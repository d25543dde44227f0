"""GPU: the stream form of SHA-256 (sha256_kernel.hip sha256_stream_kernel:
persistent waves, each message's chain cut into 32 KiB segments handed from
wave to wave) against hashlib — the digests the reference computes with
Sha256::digest at filesystem.rs:1070/:1131 and chunk_reader.rs:108/:184.

It is chosen for batches of more 64-message groups than the chip has SIMDs
(config 3c's combined verification); MXEC_SHA_FORM=stream forces it for any
batch (in a child process: the choice is read once per process)."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

import maxio_amd
import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEG = 512 * 64  # bytes per segment

CHILD = r'''
import hashlib, sys
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/oracle"]
import maxio_amd, oracle
rng = np.random.default_rng(71)
SEG = 512 * 64
lens = [0, 1, 55, 56, 63, 64, 119, 120, SEG - 64, SEG - 1, SEG, SEG + 1, SEG + 64, 2 * SEG, 3 * SEG - 9,
        (1 << 20), (1 << 20) + 5, 5 * SEG + 100]
lens += [int(x) for x in rng.integers(0, 4 * SEG, 150)]
bufs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
with maxio_amd.Context(streams_per_device=2) as c:
    got = c.sha256(bufs)
    assert got == [hashlib.sha256(b).digest() for b in bufs], "stream-form digests differ from hashlib"
    # verify + rebuild through mxec_reconstruct (expected digests, one corrupt shard)
    k, m, S = 6, 3, 3 * SEG + 17
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    par, dig = c.encode(data, m, S)
    want, want_dig, rc = oracle.compute_parity(data, m, S)
    assert dig == want_dig and all(np.array_equal(par[i], want[i]) for i in range(m))
    shards = [d.tobytes() for d in data] + [p.tobytes() for p in par]
    inp = list(shards)
    inp[2] = bytes(S)
    out, present = c.reconstruct(inp, k, m, S, expected=dig)
    assert present.all() and out[2].tobytes() == shards[2]
print("stream child ok", len(bufs))
'''


def test_stream_form_forced_matches_hashlib():
    env = dict(os.environ, MXEC_SHA_FORM="stream")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "stream child ok" in r.stdout


def test_stream_form_chosen_for_oversubscribed_batch(ctx):
    """More 64-message groups than SIMDs (65 600 messages > 1 024 x 64): the
    combined launch takes the stream form by itself.  Mostly short messages,
    every 97th one several segments long."""
    rng = np.random.default_rng(72)
    n = 65_600
    lens = rng.integers(0, 4096, n)
    lens[::97] = rng.integers(SEG, 5 * SEG, len(lens[::97]))
    lens[1] = 0
    lens[2] = SEG
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8).tobytes()
    bufs, o = [], 0
    for x in lens:
        bufs.append(blob[o:o + int(x)])
        o += int(x)
    got = ctx.sha256(bufs)
    want = [hashlib.sha256(b).digest() for b in bufs]
    bad = [i for i in range(n) if got[i] != want[i]]
    assert not bad, f"{len(bad)} digests differ, first {bad[:5]}"


def test_stream_form_device_verify_and_rebuild(ctx):
    """Device-resident verification of 7 000 objects of 8+4 x 64 KiB (two
    segments per shard) with two erasures and one silent corruption per
    object: the 70 000 present shards are more 64-message groups than SIMDs,
    so the combined launch takes the stream form; mismatches become erasures
    and every object is rebuilt exactly (chunk_reader.rs:176-211)."""
    import torch

    k, m, S, n = 8, 4, 65536, 7000
    g = torch.Generator(device="cuda").manual_seed(73)
    obj = torch.randint(0, 256, (n, k + m, S), dtype=torch.uint8, device="cuda", generator=g)
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.encode_strided_device(k, m, S, n, obj.data_ptr(), (k + m) * S, S, obj[:, k:].data_ptr(), (k + m) * S, S,
                              digests_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    ref = obj.clone()
    h = ref[n - 1].cpu().numpy()
    want, want_dig, rc = oracle.compute_parity(list(h[:k]), m, S)
    assert [bytes(x) for x in dig[n - 1].cpu().numpy()] == want_dig
    rng = np.random.default_rng(74)
    present = np.ones(n * (k + m), np.uint8)
    for o in range(n):
        lost = rng.choice(k + m, 3, replace=False)
        for i in lost[:2]:
            present[o * (k + m) + i] = 0
            obj[o, i].zero_()
        obj[o, lost[2], 1000] ^= 0x01  # silent corruption
    torch.cuda.synchronize()
    rc, status = ctx.reconstruct_strided_device(k, m, S, n, obj.data_ptr(), (k + m) * S, S, present,
                                                expected_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    assert rc == 0 and present.all()
    assert torch.equal(obj, ref)

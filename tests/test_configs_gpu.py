"""GPU: the BASELINE workload shapes end to end against the oracle, every
object checked (not a sample):

* configs[1] — 4+2 at 10 MiB: every object's parity bytes and parity digests
  equal the oracle's (filesystem.rs:1108-1131);
* configs[4] — mixed 4+2 / 8+4 / 10+4 at 64 KiB .. 10 MiB with short last
  chunks, encoded then reconstructed with 1..m seeded erasures in one stream,
  per class (the bench's layout) and as one mixed-shape launch;
* configs[3] — 10+4 at 1 MiB, one object per device, on eight logical
  devices of one GPU (mxec_open_test logical_devices=8, each with its own streams,
  arenas and pipeline, as MaxIO's one process would open eight MI355X), and
  the literal reading k=64 m=4.

Reference: filesystem.rs:1084-1145 (encode), chunk_reader.rs:157-226
(reconstruct); SURVEY §8(d) maps the configs."""
from __future__ import annotations

import re

import hashlib

import numpy as np
import pytest

import maxio_amd
import oracle

pytestmark = pytest.mark.gpu

SEED = 0x6D6178696F


def _torch():
    import torch

    return torch


def test_config2_every_object_parity_and_digest(ctx):
    torch = _torch()
    k, m, s, n = 4, 2, 10 << 20, 6
    g = torch.Generator(device="cuda").manual_seed(12)
    data = torch.randint(0, 256, (n, k, s), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.zeros((n, m, s), dtype=torch.uint8, device="cuda")
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.encode_strided_device(k, m, s, n, data.data_ptr(), k * s, s, par.data_ptr(), m * s, s,
                              digests_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    hd, hp, hg = data.cpu().numpy(), par.cpu().numpy(), dig.cpu().numpy()
    for o in range(n):
        want, want_dig, rc = oracle.compute_parity(list(hd[o]), m, s)
        assert rc == 0
        for i in range(m):
            assert np.array_equal(hp[o, i], want[i]), (o, i)
        assert [bytes(x) for x in hg[o]] == want_dig, o


def _mixed_classes(rng, per_class_objects=2):
    kms = [(4, 2), (8, 4), (10, 4)]
    sizes = [64 << 10, 256 << 10, 1 << 20, 4 << 20, 10 << 20]
    out = []
    for (k, m) in kms:
        for S in sizes:
            last = int(rng.integers(1, S))
            out.append((k, m, S, per_class_objects, [S] * (k - 1) + [last]))
    return out


def test_config5_mixed_stream_encode_then_reconstruct(ctx):
    """Per class: encode with a short last chunk (zero padded, never
    materialised), check every object's parity against the oracle, erase
    1..m seeded shards (data and parity), reconstruct on the same stream, and
    the whole object equals its encoded state."""
    torch = _torch()
    rng = np.random.default_rng(SEED)
    st = torch.cuda.Stream()
    classes = []
    for (k, m, S, n, dl) in _mixed_classes(rng):
        t = torch.randint(0, 256, (n, k + m, S), dtype=torch.uint8, device="cuda")
        # bytes past a short chunk's length are not part of it; zero them so
        # the stored object is exactly what the reference would hold
        t[:, k - 1, dl[-1]:] = 0
        classes.append((k, m, S, n, dl, t))
    torch.cuda.synchronize()
    for (k, m, S, n, dl, t) in classes:
        ctx.encode_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, t[:, k:].data_ptr(), (k + m) * S, S,
                                  data_len=dl, stream=st.cuda_stream)
    st.synchronize()
    refs = [c[5].clone() for c in classes]
    torch.cuda.synchronize()
    for (k, m, S, n, dl, t), ref in zip(classes, refs):
        h = ref.cpu().numpy()
        for o in range(n):
            want = oracle.encode([h[o][j][:dl[j]] for j in range(k)], m, S)
            for i in range(m):
                assert np.array_equal(h[o][k + i], want[i]), (k, m, S, o, i)
    pres = []
    for (k, m, S, n, dl, t) in classes:
        p = np.ones(n * (k + m), np.uint8)
        for o in range(n):
            for i in rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False):
                p[o * (k + m) + i] = 0
                t[o, i].fill_(0xA5)
        pres.append(p)
    torch.cuda.synchronize()
    for (k, m, S, n, dl, t), p in zip(classes, pres):
        rc, status = ctx.reconstruct_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, p,
                                                    shard_len=dl + [S] * m, stream=st.cuda_stream)
        assert rc == 0 and p.all() and not status.any()
    st.synchronize()
    for (k, m, S, n, dl, t), ref in zip(classes, refs):
        # a rebuilt short chunk is written at its length; the bytes past it
        # in the slot are not part of the chunk
        t[:, k - 1, dl[-1]:] = 0
        assert torch.equal(t, ref), (k, m, S)


def test_config5_one_mixed_launch(ctx):
    """The same classes as ONE mxec_encode_batch_device call (objects of
    different (k, m, S) in one batch), parity equal to the oracle's."""
    torch = _torch()
    rng = np.random.default_rng(SEED + 1)
    objs, dptr, pptr, dlen, bufs = [], [], [], [], []
    for (k, m, S, n, dl) in _mixed_classes(rng, 1):
        d = torch.randint(0, 256, (k, S), dtype=torch.uint8, device="cuda")
        p = torch.zeros((m, S), dtype=torch.uint8, device="cuda")
        objs.append((k, m, S))
        dptr += [d[j].data_ptr() for j in range(k)]
        pptr += [p[i].data_ptr() for i in range(m)]
        dlen += dl
        bufs.append((d, p, dl))
    dig = torch.zeros((sum(k + m for k, m, _ in objs), 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.encode_batch_device(objs, dptr, pptr, data_len=dlen, digests_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    hdig = dig.cpu().numpy()
    row = 0
    for (k, m, S), (d, p, dl) in zip(objs, bufs):
        hd, hp = d.cpu().numpy(), p.cpu().numpy()
        want, want_dig, rc = oracle.compute_parity([hd[j][:dl[j]] for j in range(k)], m, S)
        assert rc == 0
        for i in range(m):
            assert np.array_equal(hp[i], want[i]), (k, m, S, i)
        assert [bytes(hdig[row + t]) for t in range(k + m)] == want_dig
        row += k + m


@pytest.fixture()
def ctx8(monkeypatch, capfd):
    """Eight logical devices of the one card, with the debug affinity check
    on (MXEC_DEBUG_AFFINITY: every launch and copy asserts that its stream,
    slot, arena and pointers belong to the launching logical device); the
    totals printed at close must show checks and no violation."""
    monkeypatch.setenv("MXEC_DEBUG_AFFINITY", "1")
    c = maxio_amd.Context(device_mask=1, streams_per_device=1, test={"logical_devices": 8})
    assert c.device_ids() == [0] * 8
    yield c
    c.close()
    err = capfd.readouterr().err
    m = re.search(r"maxio_ec affinity: (\d+) checks, (\d+) violations", err)
    assert m and int(m.group(1)) > 0 and m.group(2) == "0", err[-2000:]


@pytest.mark.parametrize("k,m,n_obj", [(10, 4, 8), (10, 4, 13), (64, 4, 8)])
def test_config4_one_object_per_device(ctx8, k, m, n_obj):
    """configs[3]: objects of k=10 (or 64) 1 MiB chunks + 4 parity, dealt one
    per device over eight devices (object i -> device i mod 8), from host
    memory, with digests; every parity chunk and digest equals the oracle's
    and hashlib's."""
    S = 1 << 20
    rng = np.random.default_rng(SEED + k + n_obj)
    objs, dptr, pptr, dlen, keep = [], [], [], [], []
    for o in range(n_obj):
        chunks = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        if o % 3 == 2:
            chunks[-1] = chunks[-1][: int(rng.integers(1, S))].copy()
        outs = [np.full(S, 0xEE, np.uint8) for _ in range(m)]
        objs.append((k, m, S))
        dptr += [c.ctypes.data for c in chunks]
        dlen += [c.size for c in chunks]
        pptr += [x.ctypes.data for x in outs]
        keep.append((chunks, outs))
    dig = np.zeros(n_obj * (k + m) * 32, np.uint8)
    st = ctx8.encode_batch_host(objs, dptr, pptr, data_len=dlen, digests=dig)
    assert not st.any()
    for o, (chunks, outs) in enumerate(keep):
        want, want_dig, rc = oracle.compute_parity(chunks, m, S)
        assert rc == 0
        for i in range(m):
            assert np.array_equal(outs[i], want[i]), (o, i)
        got = [dig[(o * (k + m) + t) * 32:(o * (k + m) + t + 1) * 32].tobytes() for t in range(k + m)]
        assert got == want_dig, o
        assert got[0] == hashlib.sha256(chunks[0].tobytes()).digest()


def test_config5_mixed_host_batch_over_eight_devices(ctx8):
    """configs[4]'s mixed stream as a host batch (mxec_encode_batch_host) over
    eight devices: 4+2 / 8+4 / 10+4 at 64 KiB .. 10 MiB chunks with short last
    chunks, dealt by bytes (deal.hpp; the balance itself is unit-tested on
    the CPU, tests/test_host_planning.py).  Every parity chunk and digest
    equals the oracle's, with the affinity check on."""
    rng = np.random.default_rng(SEED + 55)
    kms = [(4, 2), (8, 4), (10, 4)]
    sizes = [64 << 10, 256 << 10, 1 << 20, 4 << 20, 10 << 20]
    objs, dptr, pptr, dlen, keep = [], [], [], [], []
    for o in range(20):
        k, m = kms[o % 3]
        S = sizes[int(rng.integers(0, len(sizes)))] if o >= 5 else sizes[o]
        chunks = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        chunks[-1] = chunks[-1][: int(rng.integers(1, S + 1))].copy()
        outs = [np.full(S, 0xEE, np.uint8) for _ in range(m)]
        objs.append((k, m, S))
        dptr += [c.ctypes.data for c in chunks]
        dlen += [c.size for c in chunks]
        pptr += [x.ctypes.data for x in outs]
        keep.append((chunks, outs, m, S))
    n_msgs = sum(k + m for (k, m, S) in objs)
    dig = np.zeros(n_msgs * 32, np.uint8)
    st = ctx8.encode_batch_host(objs, dptr, pptr, data_len=dlen, digests=dig)
    assert not st.any()
    row = 0
    for o, (chunks, outs, m, S) in enumerate(keep):
        want, want_dig, rc = oracle.compute_parity(chunks, m, S)
        assert rc == 0
        for i in range(m):
            assert np.array_equal(outs[i], want[i]), (o, i)
        k = len(chunks)
        got = [dig[(row + t) * 32:(row + t + 1) * 32].tobytes() for t in range(k + m)]
        assert got == want_dig, o
        row += k + m


def test_config3_host_reconstruct_over_eight_devices(ctx8):
    """configs[2]'s GET side from host memory (mxec_reconstruct_batch_host)
    over eight devices, mixed with configs[4]'s shapes: 8+4 x 1 MiB objects
    with two erasures and a silently corrupt shard, 4+2 / 10+4 at 64 KiB and
    256 KiB with short last chunks; verified against the manifest digests.
    Every object comes back bit-exact (oracle parity, hashlib digests), with
    the affinity check on."""
    rng = np.random.default_rng(SEED + 77)
    objs, ptrs, lens, present, expected, originals, bufs = [], [], [], [], [], [], []
    shapes = [(8, 4, 1 << 20)] * 8 + [(4, 2, 64 << 10), (10, 4, 256 << 10)] * 6
    for o, (k, m, S) in enumerate(shapes):
        chunks = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        if o % 2:
            chunks[-1] = chunks[-1][: int(rng.integers(1, S))].copy()
        par, dig, rc = oracle.compute_parity(chunks, m, S)
        assert rc == 0
        shards = list(chunks) + [np.asarray(p, np.uint8) for p in par]
        originals.append([x.copy() for x in shards])
        lost = set(int(x) for x in rng.choice(k + m, 2 if m > 2 else 1, replace=False))
        keep = [i for i in range(k + m) if i not in lost]
        bad = int(rng.choice(keep))
        objs.append((k, m, S))
        for i, x in enumerate(shards):
            b = np.empty(max(1, x.size), np.uint8)
            b[:x.size] = 0xEE if i in lost else x
            if i == bad:
                b[0] ^= 0x80
            bufs.append(b)
            ptrs.append(b.ctypes.data)
            lens.append(x.size)
            present.append(0 if i in lost else 1)
            expected.append(np.frombuffer(dig[i], np.uint8))
    present = np.array(present, np.uint8)
    rc, status = ctx8.reconstruct_batch_host(objs, ptrs, present, shard_len=lens,
                                             expected=np.concatenate(expected).copy())
    assert rc == 0 and not status.any() and present.all()
    g = 0
    for o, (k, m, S) in enumerate(objs):
        for i in range(k + m):
            assert np.array_equal(bufs[g + i][:lens[g + i]], originals[o][i]), (o, i)
        g += k + m

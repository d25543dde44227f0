"""GPU: mixed-shape device batches — objects of different (k, m) and chunk
sizes in ONE call each way (BASELINE configs[4]'s continuous encode + decode
stream): `mxec_encode_batch_device` (one grouped launch per m) and
`mxec_reconstruct_batch_device` (one grouped launch per number of shards to
rebuild), checked object by object against the oracle.

Reference: filesystem.rs:1084-1145 (encode of each object),
chunk_reader.rs:157-226 (verify -> erasure -> reconstruct of each object)."""
from __future__ import annotations

import re

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

SEED = 0x6D6178696F
DATA_ONLY = 1
E_TOO_FEW_PRESENT = -10


def _torch():
    import torch

    return torch


def _classes(rng, sizes=(64 << 10, 256 << 10, 1 << 20), kms=((4, 2), (8, 4), (10, 4)), n=2):
    out = []
    for (k, m) in kms:
        for S in sizes:
            out.append((k, m, S, n, [S] * (k - 1) + [int(rng.integers(1, S))]))
    return out


class Batch:
    """Object-major tensors per class ([n][k+m][S]); the flat per-object
    arrays the mixed entry points take."""

    def __init__(self, torch, classes):
        self.classes = []
        self.objs, self.dptr, self.pptr, self.dlen, self.sptr, self.slen = [], [], [], [], [], []
        for (k, m, S, n, dl) in classes:
            t = torch.randint(0, 256, (n, k + m, S), dtype=torch.uint8, device="cuda")
            t[:, k - 1, dl[-1]:] = 0  # bytes past the short chunk are not part of it
            self.classes.append((k, m, S, n, dl, t))
            for o in range(n):
                self.objs.append((k, m, S))
                self.dptr += [t[o, j].data_ptr() for j in range(k)]
                self.pptr += [t[o, k + i].data_ptr() for i in range(m)]
                self.dlen += dl
                self.sptr += [t[o, i].data_ptr() for i in range(k + m)]
                self.slen += dl + [S] * m
        self.total = len(self.sptr)

    def check_parity(self):
        for (k, m, S, n, dl, t) in self.classes:
            h = t.cpu().numpy()
            for o in range(n):
                want = oracle.encode([h[o][j][:dl[j]] for j in range(k)], m, S)
                for i in range(m):
                    assert np.array_equal(h[o][k + i], want[i]), (k, m, S, o, i)


@pytest.mark.parametrize("multi", ["1", "0"])
def test_mixed_encode_then_reconstruct_one_call_each(ctx_with, multi):
    """Encode every class in one call (digests too), erase 1..m seeded
    shards per object (data and parity) and silently corrupt a present shard
    of every third object, then one verified reconstruct call: every object
    equals its encoded state, the corrupted shards were caught.  multi=1: the
    r = 1..4 groups of each call run as one multi-r launch (rs_apply_multi,
    the default); 0: one grouped launch per r."""
    ctx = ctx_with(MXEC_RS_MULTI=multi)  # read at mxec_open
    torch = _torch()
    rng = np.random.default_rng(SEED)
    b = Batch(torch, _classes(rng) + [(4, 2, 10 << 20, 1, [10 << 20] * 3 + [777])])
    dig = torch.zeros((b.total, 32), dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    ctx.encode_batch_device(b.objs, b.dptr, b.pptr, data_len=b.dlen, digests_ptr=dig.data_ptr(),
                            stream=st.cuda_stream)
    st.synchronize()
    b.check_parity()
    refs = [c[5].clone() for c in b.classes]
    present = np.ones(b.total, np.uint8)
    corrupted = []
    g = 0
    ob = 0
    for (k, m, S, n, dl, t) in b.classes:
        for o in range(n):
            e = int(rng.integers(1, m + 1))
            if ob % 3 == 0:
                e = min(e, m - 1)
            miss = rng.choice(k + m, e, replace=False)
            for i in miss:
                present[g + i] = 0
                t[o, i].fill_(0xA5)
            if ob % 3 == 0:
                keep = [i for i in range(k + m) if i not in miss]
                c = int(rng.choice(keep))
                t[o, c, 0] ^= 0x01
                corrupted.append(g + c)
            g += k + m
            ob += 1
    torch.cuda.synchronize()
    p = present.copy()
    rc, status = ctx.reconstruct_batch_device(b.objs, b.sptr, p, shard_len=b.slen, expected_ptr=dig.data_ptr(),
                                              stream=st.cuda_stream)
    st.synchronize()
    assert rc == 0 and not status.any() and p.all()
    for (k, m, S, n, dl, t), ref in zip(b.classes, refs):
        t[:, k - 1, dl[-1]:] = 0  # a rebuilt short chunk is written at its length
        assert torch.equal(t, ref), (k, m, S)
    assert corrupted


def test_mixed_reconstruct_without_verify_and_data_only(ctx):
    """No expected digests: the masks as given; with MXEC_F_DATA_ONLY only the
    missing data shards are rebuilt (crate reconstruct_data) and missing
    parity stays missing."""
    torch = _torch()
    rng = np.random.default_rng(SEED + 1)
    b = Batch(torch, _classes(rng, sizes=(64 << 10, 1 << 20)))
    torch.cuda.synchronize()
    ctx.encode_batch_device(b.objs, b.dptr, b.pptr, data_len=b.dlen)
    torch.cuda.synchronize()
    refs = [c[5].clone() for c in b.classes]
    present = np.ones(b.total, np.uint8)
    g = 0
    for (k, m, S, n, dl, t) in b.classes:
        for o in range(n):
            # one data shard and one parity shard missing
            for i in (int(rng.integers(0, k)), k + int(rng.integers(0, m))):
                present[g + i] = 0
                t[o, i].fill_(0x5A)
            g += k + m
    torch.cuda.synchronize()
    p = present.copy()
    rc, status = ctx.reconstruct_batch_device(b.objs, b.sptr, p, shard_len=b.slen, data_only=True)
    torch.cuda.synchronize()
    assert rc == 0 and not status.any()
    g = 0
    for (k, m, S, n, dl, t), ref in zip(b.classes, refs):
        t[:, k - 1, dl[-1]:] = 0
        for o in range(n):
            for i in range(k + m):
                if i < k:
                    assert p[g + i] == 1
                    assert torch.equal(t[o, i], ref[o, i]), (k, m, S, o, i)
                else:
                    assert p[g + i] == present[g + i]
            g += k + m
    # now the parity too
    rc, status = ctx.reconstruct_batch_device(b.objs, b.sptr, p, shard_len=b.slen)
    torch.cuda.synchronize()
    assert rc == 0 and p.all()
    for (k, m, S, n, dl, t), ref in zip(b.classes, refs):
        assert torch.equal(t, ref), (k, m, S)


def test_mixed_reconstruct_too_few_shards(ctx):
    """An object missing m+1 shards fails alone (status -10, the reference's
    message); the others of the batch are rebuilt."""
    torch = _torch()
    rng = np.random.default_rng(SEED + 2)
    b = Batch(torch, _classes(rng, sizes=(64 << 10,), n=3))
    torch.cuda.synchronize()
    ctx.encode_batch_device(b.objs, b.dptr, b.pptr, data_len=b.dlen)
    torch.cuda.synchronize()
    refs = [c[5].clone() for c in b.classes]
    present = np.ones(b.total, np.uint8)
    bad = 4  # object index in batch order
    g = 0
    ob = 0
    for (k, m, S, n, dl, t) in b.classes:
        for o in range(n):
            e = m + 1 if ob == bad else 1
            for i in rng.choice(k + m, e, replace=False):
                present[g + i] = 0
                if ob != bad:
                    t[o, i].fill_(0x33)
            g += k + m
            ob += 1
    torch.cuda.synchronize()
    p = present.copy()
    rc, status = ctx.reconstruct_batch_device(b.objs, b.sptr, p, shard_len=b.slen)
    torch.cuda.synchronize()
    assert rc == E_TOO_FEW_PRESENT
    assert [i for i, s in enumerate(status) if s] == [bad] and status[bad] == E_TOO_FEW_PRESENT
    for (k, m, S, n, dl, t), ref in zip(b.classes, refs):
        t[:, k - 1, dl[-1]:] = 0
        assert torch.equal(t, ref), (k, m, S)


def test_mixed_batches_unaligned_and_wide(ctx):
    """Shapes the grouped launch does not take fall back per (k, S) inside the
    same calls: a shard size that is not a multiple of 16 (unaligned shard
    pointers), m > 8 (row groups), beside aligned objects of the same m."""
    torch = _torch()
    rng = np.random.default_rng(SEED + 3)
    classes = [(3, 2, 5000, 2, [5000, 5000, 1234]), (4, 2, 64 << 10, 2, [64 << 10] * 3 + [100]),
               (20, 10, 4096, 2, [4096] * 19 + [4000]), (6, 10, 8192, 1, [8192] * 6)]
    b = Batch(torch, classes)
    torch.cuda.synchronize()
    ctx.encode_batch_device(b.objs, b.dptr, b.pptr, data_len=b.dlen)
    torch.cuda.synchronize()
    b.check_parity()
    refs = [c[5].clone() for c in b.classes]
    present = np.ones(b.total, np.uint8)
    g = 0
    for (k, m, S, n, dl, t) in b.classes:
        for o in range(n):
            for i in rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False):
                present[g + i] = 0
                t[o, i].fill_(0x77)
            g += k + m
    torch.cuda.synchronize()
    p = present.copy()
    rc, status = ctx.reconstruct_batch_device(b.objs, b.sptr, p, shard_len=b.slen)
    torch.cuda.synchronize()
    assert rc == 0 and p.all() and not status.any()
    for (k, m, S, n, dl, t), ref in zip(b.classes, refs):
        t[:, k - 1, dl[-1]:] = 0
        assert torch.equal(t, ref), (k, m, S)


def test_mixed_reconstruct_async_matches(ctx):
    """mxec_reconstruct_batch_device_async (ticket + eventfd): the same
    rebuild as the blocking call, the pointer arrays copied at submission
    (the caller's lists are dropped before the ticket completes)."""
    torch = _torch()
    rng = np.random.default_rng(SEED + 4)
    b = Batch(torch, _classes(rng, sizes=(64 << 10, 1 << 20)))
    dig = torch.zeros((b.total, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.encode_batch_device(b.objs, b.dptr, b.pptr, data_len=b.dlen, digests_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    refs = [c[5].clone() for c in b.classes]
    present = np.ones(b.total, np.uint8)
    g = 0
    for (k, m, S, n, dl, t) in b.classes:
        for o in range(n):
            for i in rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False):
                present[g + i] = 0
                t[o, i].fill_(0x11)
            g += k + m
    torch.cuda.synchronize()
    p = present.copy()
    sptr, slen = list(b.sptr), list(b.slen)
    tk = ctx.reconstruct_batch_device_async(b.objs, sptr, p, shard_len=slen, expected_ptr=dig.data_ptr())
    del sptr, slen
    status = tk.wait()
    tk.close()
    torch.cuda.synchronize()
    assert not status.any() and p.all()
    for (k, m, S, n, dl, t), ref in zip(b.classes, refs):
        t[:, k - 1, dl[-1]:] = 0
        assert torch.equal(t, ref), (k, m, S)


@pytest.fixture()
def ctx8(monkeypatch, capfd):
    """Eight logical devices of the one card, with the debug affinity check
    on (MXEC_DEBUG_AFFINITY: every launch and copy asserts that its stream,
    slot, arena and pointers belong to the launching logical device); the
    totals printed at close must show checks and no violation."""
    import maxio_amd

    monkeypatch.setenv("MXEC_DEBUG_AFFINITY", "1")
    c = maxio_amd.Context(device_mask=1, streams_per_device=1, test={"logical_devices": 8})
    assert c.device_ids() == [0] * 8
    yield c
    c.close()
    err = capfd.readouterr().err
    m = re.search(r"maxio_ec affinity: (\d+) checks, (\d+) violations", err)
    assert m and int(m.group(1)) > 0 and m.group(2) == "0", err[-2000:]


def test_mixed_batches_over_eight_devices(ctx8):
    """configs[4] as eight GPUs would run it: the mixed objects dealt object
    i -> device i mod 8; each device's share is one encode and
    then one verified reconstruct batch call from its own host thread on its
    own stream (per-device slots, descriptor rings, coefficient arenas).
    Every parity equals the oracle's and every object its encoded state."""
    import threading

    torch = _torch()
    rng = np.random.default_rng(SEED + 5)
    b = Batch(torch, _classes(rng, sizes=(64 << 10, 256 << 10, 1 << 20), n=3))
    where, spans, g = [], [], 0  # object -> (class tensor, index in class), (first global shard, k, m)
    for (k, m, S, n, dl, t) in b.classes:
        for o in range(n):
            where.append((t, o))
            spans.append((g, k, m))
            g += k + m
    D = 8
    mine = [[o for o in range(len(b.objs)) if o % D == d] for d in range(D)]
    streams = [torch.cuda.Stream() for _ in range(D)]
    dig = torch.zeros((b.total, 32), dtype=torch.uint8, device="cuda")
    errors = []

    def arrays(d):
        gi = [gg for o in mine[d] for gg in range(spans[o][0], spans[o][0] + spans[o][1] + spans[o][2])]
        return [b.objs[o] for o in mine[d]], gi

    def encode(d):
        try:
            oo, gi = arrays(d)
            dp = [b.sptr[spans[o][0] + j] for o in mine[d] for j in range(spans[o][1])]
            pp = [b.sptr[spans[o][0] + spans[o][1] + i] for o in mine[d] for i in range(spans[o][2])]
            dl = [b.slen[spans[o][0] + j] for o in mine[d] for j in range(spans[o][1])]
            # this device's digests: rows gi of `dig`, contiguous per object in batch order
            dg = torch.zeros((len(gi), 32), dtype=torch.uint8, device="cuda")
            ctx8.encode_batch_device(oo, dp, pp, data_len=dl, digests_ptr=dg.data_ptr(), dev=d,
                                     stream=streams[d].cuda_stream)
            streams[d].synchronize()
            dig[gi] = dg
        except Exception as e:  # noqa: BLE001
            errors.append(("encode", d, repr(e)))

    def reconstruct(d, present):
        try:
            oo, gi = arrays(d)
            pr = present[gi].copy()
            dg = dig[gi].contiguous()
            torch.cuda.synchronize()
            rc, status = ctx8.reconstruct_batch_device(oo, [b.sptr[x] for x in gi], pr,
                                                       shard_len=[b.slen[x] for x in gi],
                                                       expected_ptr=dg.data_ptr(), dev=d,
                                                       stream=streams[d].cuda_stream)
            streams[d].synchronize()
            if rc != 0 or status.any() or not pr.all():
                errors.append(("reconstruct", d, rc, status.tolist()))
        except Exception as e:  # noqa: BLE001
            errors.append(("reconstruct", d, repr(e)))

    torch.cuda.synchronize()
    ths = [threading.Thread(target=encode, args=(d,)) for d in range(D)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    b.check_parity()
    refs = [c[5].clone() for c in b.classes]
    present = np.ones(b.total, np.uint8)
    for o, (g0, k, m) in enumerate(spans):
        t, oi = where[o]
        for i in rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False):
            present[g0 + int(i)] = 0
            t[oi, int(i)].fill_(0xC3)
    torch.cuda.synchronize()
    ths = [threading.Thread(target=reconstruct, args=(d, present)) for d in range(D)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    for (k, m, S, n, dl, t), ref in zip(b.classes, refs):
        t[:, k - 1, dl[-1]:] = 0
        assert torch.equal(t, ref), (k, m, S)


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_mixed_random_shapes(ctx, seed):
    """60 objects of random k (1-24), m (1-10) and shard size (16 B-320 KiB,
    a few not a multiple of 16), ragged last chunks, in one encode and one
    reconstruct call (grouped launches and the per-(k, S) fallbacks mixed):
    every parity equals the oracle's, every object with <= m erasures comes
    back bit-exact, every object with more fails alone."""
    torch = _torch()
    rng = np.random.default_rng(seed)
    objs, tens, dls = [], [], []
    for _ in range(60):
        k, m = int(rng.integers(1, 25)), int(rng.integers(1, 11))
        S = int(rng.integers(1, 20001)) * 16 if rng.random() < 0.85 else int(rng.integers(1, 4000)) * 16 + 7
        dl = [S] * (k - 1) + [int(rng.integers(1, S + 1))]
        t = torch.randint(0, 256, (k + m, S), dtype=torch.uint8, device="cuda")
        t[k - 1, dl[-1]:] = 0
        objs.append((k, m, S))
        tens.append(t)
        dls.append(dl)
    dptr = [t[j].data_ptr() for (k, m, S), t in zip(objs, tens) for j in range(k)]
    pptr = [t[k + i].data_ptr() for (k, m, S), t in zip(objs, tens) for i in range(m)]
    dlen = [x for dl in dls for x in dl]
    torch.cuda.synchronize()
    ctx.encode_batch_device(objs, dptr, pptr, data_len=dlen)
    torch.cuda.synchronize()
    for (k, m, S), t, dl in zip(objs, tens, dls):
        h = t.cpu().numpy()
        want = oracle.encode([h[j][:dl[j]] for j in range(k)], m, S)
        for i in range(m):
            assert np.array_equal(h[k + i], want[i]), (k, m, S, i)
    refs = [t.clone() for t in tens]
    present, sptr, slen, fail = [], [], [], []
    for o, ((k, m, S), t, dl) in enumerate(zip(objs, tens, dls)):
        e = int(rng.integers(1, m + 1)) if o % 7 else min(k + m, m + 1)
        p = np.ones(k + m, np.uint8)
        for i in rng.choice(k + m, e, replace=False):
            p[i] = 0
            t[int(i)].fill_(0x99)
        if e > m:
            fail.append(o)
        present.append(p)
        sptr += [t[i].data_ptr() for i in range(k + m)]
        slen += dl + [S] * m
    pres = np.concatenate(present)
    torch.cuda.synchronize()
    rc, status = ctx.reconstruct_batch_device(objs, sptr, pres, shard_len=slen)
    torch.cuda.synchronize()
    assert [o for o, st in enumerate(status) if st] == fail
    assert rc == (E_TOO_FEW_PRESENT if fail else 0)
    for o, ((k, m, S), t, dl, ref) in enumerate(zip(objs, tens, dls, refs)):
        if o in fail:
            continue
        t[k - 1, dl[-1]:] = 0
        assert torch.equal(t, ref), (o, k, m, S)


def test_mixed_large_batch_side_stream_tables(ctx):
    """4 000 objects of 64 KiB shards (4+2 and 8+4) in one call each way: the
    descriptor tables pass 256 KiB, so they are copied on the slot's side
    stream the launch waits for (runtime.cpp DescWriter::commit); every
    object's round trip is exact and a sample's parity equals the oracle's."""
    torch = _torch()
    rng = np.random.default_rng(SEED + 6)
    S = 64 << 10
    specs = [(4, 2, 2500), (8, 4, 1500)]
    b = Batch(torch, [(k, m, S, n, [S] * (k - 1) + [int(rng.integers(1, S + 1))]) for (k, m, n) in specs])
    assert len(b.objs) == 4000
    torch.cuda.synchronize()
    ctx.encode_batch_device(b.objs, b.dptr, b.pptr, data_len=b.dlen)
    torch.cuda.synchronize()
    for (k, m, S_, n, dl, t) in b.classes:
        h = t[[0, n // 2, n - 1]].cpu().numpy()
        for row in h:
            want = oracle.encode([row[j][:dl[j]] for j in range(k)], m, S_)
            for i in range(m):
                assert np.array_equal(row[k + i], want[i]), (k, m, i)
    refs = [c[5].clone() for c in b.classes]
    present = np.ones(b.total, np.uint8)
    g = 0
    for (k, m, S_, n, dl, t) in b.classes:
        for o in range(n):
            for i in rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False):
                present[g + int(i)] = 0
            g += k + m
    g = 0
    for (k, m, S_, n, dl, t) in b.classes:
        mask = torch.from_numpy(present[g:g + n * (k + m)].reshape(n, k + m) == 0).cuda()
        t[mask] = 0x3C
        g += n * (k + m)
    torch.cuda.synchronize()
    p = present.copy()
    rc, status = ctx.reconstruct_batch_device(b.objs, b.sptr, p, shard_len=b.slen)
    torch.cuda.synchronize()
    assert rc == 0 and p.all() and not status.any()
    for (k, m, S_, n, dl, t), ref in zip(b.classes, refs):
        t[:, k - 1, dl[-1]:] = 0
        assert torch.equal(t, ref), (k, m)


def test_mixed_zero_length_and_tile_edge_chunks(ctx):
    """Data chunks of length 0 (read as all zero, never loaded), lengths
    that end exactly on a 16 KiB tile edge or one byte past it, and shard
    sizes that are not a tile multiple, in one grouped launch: parity equals
    the oracle's zero-padded encode."""
    torch = _torch()
    T = 16 << 10
    cases = [(4, 2, 3 * T, [0, 3 * T, T, T + 1]), (4, 2, 3 * T + 48, [T, 0, 0, 1]),
             (8, 4, 2 * T, [2 * T] * 6 + [T - 16, 0]), (6, 4, 5 * T + 16, [5 * T + 16, 2 * T, 16, 0, T, 3 * T])]
    objs, tens = [], []
    for (k, m, S, dl) in cases:
        t = torch.randint(0, 256, (k + m, S), dtype=torch.uint8, device="cuda")
        for j in range(k):
            t[j, dl[j]:] = 0
        objs.append((k, m, S))
        tens.append((t, dl))
    dptr = [t[j].data_ptr() for (k, m, S), (t, dl) in zip(objs, tens) for j in range(k)]
    pptr = [t[k + i].data_ptr() for (k, m, S), (t, dl) in zip(objs, tens) for i in range(m)]
    dlen = [x for (t, dl) in tens for x in dl]
    torch.cuda.synchronize()
    ctx.encode_batch_device(objs, dptr, pptr, data_len=dlen)
    torch.cuda.synchronize()
    for (k, m, S), (t, dl) in zip(objs, tens):
        h = t.cpu().numpy()
        want = oracle.encode([h[j][:dl[j]] for j in range(k)], m, S)
        for i in range(m):
            assert np.array_equal(h[k + i], want[i]), (k, m, S, dl, i)


def test_mixed_batch_argument_errors(ctx):
    """Crate argument errors answer before any work (k = 0, k + m > 256, a
    zero shard size)."""
    import maxio_amd

    present = np.ones(8, np.uint8)
    for objs, code in (([(0, 2, 64)], -3), ([(250, 10, 64)], -2), ([(4, 2, 0)], -11)):
        rc, _ = ctx.reconstruct_batch_device(objs, [0] * 8, present)
        assert rc == code, (objs, rc)
    with pytest.raises(maxio_amd.RSError):
        ctx.encode_batch_device([(0, 2, 64)], [0], [0, 0])
    # a NULL output (a missing shard's buffer, a parity buffer) is refused, not written
    rc, _ = ctx.reconstruct_batch_device([(2, 1, 64)], [0, 0, 0], np.array([1, 0, 1], np.uint8))
    assert rc == -21
    with pytest.raises(maxio_amd.RSError):
        ctx.encode_batch_device([(2, 1, 64)], [0, 0], [0])

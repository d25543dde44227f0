"""GPU: the RS kernels' grid-stride loop past its first iteration.

Every RS launch walks its tiles grid-stride (rs_kernel.hip rs_apply_fast,
rs_apply_multi, rs_apply_edge).  At BASELINE sizes most bytes are carried by
iterations >= 2 (configs[1]: 655 360 tiles over <= 262 144 workgroups), and
the grouped kernels prefetch the NEXT iteration's tile record
(`next = tiles[tile + gridDim.x]`).  Here the context caps every RS launch at
a handful of workgroups (mxec_open_test rs_grid_cap), so each
workgroup walks dozens of tiles across object boundaries, and EVERY object's
outputs are compared with the oracle:

* uniform encode, R = 1..8 and 12 (row groups 8 + 4), short last chunk;
* grouped encode (one m, mixed k and shard size), R = 1..8;
* multi-r encode (m = 1..4 in one launch), and per-r grouped launches;
* reconstruct: uniform, grouped and multi-r (mixed erasure counts);
* the edge kernel (unaligned pointers).

Reference: filesystem.rs:1121-1124 (encode), chunk_reader.rs:211
(reconstruct) — the crate's code_some_slices over every byte column.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

GRIDS = [7, 61]  # workgroups per launch: 7 walks ~every 7th tile, 61 is prime against every tile count


def _torch():
    import torch

    return torch


@pytest.fixture(params=GRIDS, ids=lambda g: f"grid{g}")
def gctx(request, ctx_with):
    return ctx_with(MXEC_TEST_RS_GRID=request.param)


def _round(x, a=256):
    return (x + a - 1) // a * a


@pytest.mark.parametrize("m", [1, 2, 3, 4, 5, 6, 7, 8, 12])
def test_uniform_encode_every_object(gctx, m):
    torch = _torch()
    k = {1: 3, 2: 4, 3: 5, 4: 8, 5: 4, 6: 10, 7: 2, 8: 6, 12: 9}[m]
    S = 5 * 16384 + 4096 + 48  # 6 tiles at V = 4 (11 at V = 2), the last one cut
    Sp = _round(S)
    n = 6
    g = torch.Generator(device="cuda").manual_seed(100 + m)
    t = torch.randint(0, 256, (n, k + m, Sp), dtype=torch.uint8, device="cuda", generator=g)
    t[:, k:].fill_(0x77)
    dl = [S] * (k - 1) + [S - 5000]  # the short last chunk: zero padded, never materialised
    torch.cuda.synchronize()
    gctx.encode_strided_device(k, m, S, n, t.data_ptr(), (k + m) * Sp, Sp, t.data_ptr() + k * Sp,
                               (k + m) * Sp, Sp, data_len=dl)
    torch.cuda.synchronize()
    h = t.cpu().numpy()
    for o in range(n):
        want = oracle.encode([h[o, j, :dl[j]] for j in range(k)], m, S)
        for i in range(m):
            assert np.array_equal(h[o, k + i, :S], want[i]), (m, o, i)
            assert (h[o, k + i, S:] == 0x77).all(), (m, o, i)  # nothing past the shard


def _mixed_objects(rng, ms, n_per=3):
    """(k, m, S, dl) per object: k and S vary so no two neighbours share a shape."""
    objs = []
    for m in ms:
        for t in range(n_per):
            k = int(rng.integers(1, 11))
            S = int(rng.integers(3, 40)) * 4096 + int(rng.integers(0, 4096))
            last = int(rng.integers(1, S + 1))
            objs.append((k, m, S, [S] * (k - 1) + [last]))
    return objs


class DevObjs:
    """One device buffer per object: k + m shard slots, 256-byte aligned."""

    def __init__(self, torch, objs, seed):
        self.objs = objs
        self.t = []
        g = torch.Generator(device="cuda").manual_seed(seed)
        self.dptr, self.pptr, self.dlen, self.sptr, self.slen = [], [], [], [], []
        for (k, m, S, dl) in objs:
            Sp = _round(S)
            t = torch.randint(0, 256, (k + m, Sp), dtype=torch.uint8, device="cuda", generator=g)
            t[k:].fill_(0x77)
            t[k - 1, dl[-1]:] = 0
            self.t.append(t)
            self.dptr += [t[j].data_ptr() for j in range(k)]
            self.pptr += [t[k + i].data_ptr() for i in range(m)]
            self.dlen += dl
            self.sptr += [t[i].data_ptr() for i in range(k + m)]
            self.slen += dl + [S] * m

    def shapes(self):
        return [(k, m, S) for (k, m, S, _) in self.objs]

    def check_parity(self):
        for (k, m, S, dl), t in zip(self.objs, self.t):
            h = t.cpu().numpy()
            want = oracle.encode([h[j, :dl[j]] for j in range(k)], m, S)
            for i in range(m):
                assert np.array_equal(h[k + i, :S], want[i]), (k, m, S, i)
                assert (h[k + i, S:] == 0x77).all(), (k, m, S, i)


@pytest.mark.parametrize("m", [1, 2, 3, 4, 5, 6, 7, 8])
def test_grouped_encode_every_object(gctx, m):
    """One m, mixed k and shard sizes: rs_apply_fast<GRP> with its
    one-iteration-ahead tile-record prefetch."""
    torch = _torch()
    b = DevObjs(torch, _mixed_objects(np.random.default_rng(200 + m), [m], n_per=5), 300 + m)
    torch.cuda.synchronize()
    gctx.encode_batch_device(b.shapes(), b.dptr, b.pptr, data_len=b.dlen)
    torch.cuda.synchronize()
    b.check_parity()


@pytest.mark.parametrize("multi", ["1", "0"])
def test_multi_r_encode_every_object(ctx_with, multi):
    """m = 1..4 in one call: one rs_apply_multi launch (multi=1) or one
    grouped launch per m (multi=0), both capped at 7 workgroups."""
    ctx = ctx_with(MXEC_TEST_RS_GRID=7, MXEC_RS_MULTI=multi)
    torch = _torch()
    rng = np.random.default_rng(400)
    objs = _mixed_objects(rng, [1, 2, 3, 4], n_per=3)
    order = rng.permutation(len(objs))
    b = DevObjs(torch, [objs[i] for i in order], 401)
    torch.cuda.synchronize()
    ctx.encode_batch_device(b.shapes(), b.dptr, b.pptr, data_len=b.dlen)
    torch.cuda.synchronize()
    b.check_parity()


@pytest.mark.parametrize("mode", ["uniform", "mixed"])
def test_reconstruct_every_object(gctx, mode):
    """Encode, erase seeded shards (data and parity), rebuild in one call:
    uniform (one shape, two data erasures each: one launch, R = 2) or mixed
    (shapes and 1..m erasures: multi-r / grouped launches).  Every object
    equals its encoded state and the oracle's reconstruct of its survivors."""
    torch = _torch()
    rng = np.random.default_rng(500 if mode == "uniform" else 501)
    if mode == "uniform":
        S = 9 * 16384 + 333
        objs = [(8, 4, S, [S] * 7 + [S - 777])] * 7
    else:
        objs = _mixed_objects(rng, [1, 2, 3, 4, 6], n_per=3)
    b = DevObjs(torch, objs, 502)
    torch.cuda.synchronize()
    gctx.encode_batch_device(b.shapes(), b.dptr, b.pptr, data_len=b.dlen)
    torch.cuda.synchronize()
    refs = [t.clone() for t in b.t]
    present = np.ones(len(b.sptr), np.uint8)
    g = 0
    for (k, m, S, dl), t in zip(b.objs, b.t):
        e = 2 if mode == "uniform" else int(rng.integers(1, m + 1))
        miss = rng.choice(k, 2, replace=False) if mode == "uniform" else rng.choice(k + m, e, replace=False)
        for i in miss:
            present[g + i] = 0
            t[i].fill_(0xA5)
        g += k + m
    survivors = [t.cpu().numpy() for t in b.t]
    torch.cuda.synchronize()
    p = present.copy()
    rc, status = gctx.reconstruct_batch_device(b.shapes(), b.sptr, p, shard_len=b.slen)
    torch.cuda.synchronize()
    assert rc == 0 and not status.any() and p.all()
    g = 0
    for (k, m, S, dl), t, ref, h in zip(b.objs, b.t, refs, survivors):
        t[k - 1, dl[-1]:] = 0  # a rebuilt short chunk is written at its length
        # the oracle's reconstruct of this object's survivors (first k present)
        shards = [h[i, :b.slen[g + i]] if present[g + i] else None for i in range(k + m)]
        bufs, pres, orc = oracle.reconstruct(shards, k, m, S)
        assert orc == 0
        got = t.cpu().numpy()
        for i in range(k + m):
            L = b.slen[g + i]
            assert np.array_equal(got[i, :L], bufs[i][:L]), (k, m, S, i)
        assert torch.equal(t[:, :S], ref[:, :S]), (k, m, S)
        g += k + m


def test_edge_kernel_unaligned(gctx):
    """Unaligned shard pointers send every tile to the byte-exact edge
    kernel (rs_apply_edge), also grid-stride: 4+2 and 10+4 objects at odd
    offsets, every object against the oracle."""
    torch = _torch()
    for (k, m) in [(4, 2), (10, 4)]:
        n, S = 5, 3 * 16384 + 999
        slot = _round(S + 16)
        t = torch.randint(0, 256, (n, k + m, slot), dtype=torch.uint8, device="cuda",
                          generator=torch.Generator(device="cuda").manual_seed(601 + k))
        t[:, k:].fill_(0x77)
        off = 3
        dl = [S] * (k - 1) + [S - 123]
        objs = [(k, m, S)] * n
        dptr = [t[o, j].data_ptr() + off for o in range(n) for j in range(k)]
        pptr = [t[o, k + i].data_ptr() + off for o in range(n) for i in range(m)]
        torch.cuda.synchronize()
        gctx.encode_batch_device(objs, dptr, pptr, data_len=dl * n)
        torch.cuda.synchronize()
        h = t.cpu().numpy()
        for o in range(n):
            want = oracle.encode([h[o, j, off:off + dl[j]] for j in range(k)], m, S)
            for i in range(m):
                assert np.array_equal(h[o, k + i, off:off + S], want[i]), (k, m, o, i)
                assert (h[o, k + i, :off] == 0x77).all() and (h[o, k + i, off + S:] == 0x77).all()

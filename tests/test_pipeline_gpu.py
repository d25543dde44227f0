"""GPU: the end-to-end host-memory batch encode (mxec_encode_batch_host) is
bit-identical to the oracle for pageable and pinned buffers, mixed shapes,
short last chunks, and reports per-object errors like the reference guards."""
from __future__ import annotations

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _objects(rng, specs):
    objs, data, dlen, parity, chunks_of = [], [], [], [], []
    for (k, m, s, last) in specs:
        chunks = [rng.integers(0, 256, s, dtype=np.uint8) for _ in range(k)]
        if last is not None:
            chunks[-1] = chunks[-1][:last].copy()
        objs.append((k, m, s))
        data += [c.ctypes.data for c in chunks]
        dlen += [c.size for c in chunks]
        outs = [np.full(s, 0xEE, np.uint8) for _ in range(m)]
        parity += [o.ctypes.data for o in outs]
        chunks_of.append((chunks, outs))
    return objs, data, dlen, parity, chunks_of


def _check(objs, chunks_of, digests):
    row = 0
    for (k, m, s), (chunks, outs) in zip(objs, chunks_of):
        want, want_dig, rc = oracle.compute_parity(chunks, m, s)
        assert rc == 0
        for i in range(m):
            assert np.array_equal(outs[i], want[i]), (k, m, s, i)
        if digests is not None:
            got = [digests[(row + t) * 32:(row + t + 1) * 32].tobytes() for t in range(k + m)]
            assert got == want_dig
        row += k + m


def test_batch_host_pageable_mixed(ctx):
    rng = np.random.default_rng(31)
    specs = [(4, 2, 65536, None), (8, 4, 1 << 20, 1000), (10, 4, 4096 + 16, None),
             (4, 2, 65536, 17), (1, 2, 3000, None), (3, 5, 100, 1)] * 3
    objs, data, dlen, parity, chunks_of = _objects(rng, specs)
    digests = np.zeros(sum(k + m for (k, m, _) in objs) * 32, np.uint8)
    status = ctx.encode_batch_host(objs, data, parity, data_len=dlen, digests=digests)
    assert (status == 0).all()
    _check(objs, chunks_of, digests)


def test_batch_host_pinned_buffers(ctx):
    torch = pytest.importorskip("torch")
    k, m, s, n = 4, 2, 1 << 20, 24
    host = torch.randint(0, 256, (n, k, s), dtype=torch.uint8).pin_memory()
    par = torch.zeros((n, m, s), dtype=torch.uint8).pin_memory()
    objs = [(k, m, s)] * n
    data = [host[o, j].data_ptr() for o in range(n) for j in range(k)]
    parity = [par[o, i].data_ptr() for o in range(n) for i in range(m)]
    digests = np.zeros(n * (k + m) * 32, np.uint8)
    status = ctx.encode_batch_host(objs, data, parity, digests=digests)
    assert (status == 0).all()
    h, p = host.numpy(), par.numpy()
    chunks_of = [([h[o, j] for j in range(k)], [p[o, i] for i in range(m)]) for o in range(n)]
    _check(objs, chunks_of, digests)


def test_batch_host_without_digests(ctx):
    rng = np.random.default_rng(32)
    objs, data, dlen, parity, chunks_of = _objects(rng, [(8, 4, 8192, None)] * 5)
    status = ctx.encode_batch_host(objs, data, parity, data_len=dlen)
    assert (status == 0).all()
    _check(objs, chunks_of, None)


def test_batch_host_per_object_errors(ctx):
    import maxio_amd

    rng = np.random.default_rng(33)
    objs, data, dlen, parity, chunks_of = _objects(rng, [(4, 2, 256, None)])
    bad = [(250, 6, 4)]
    bad_data = [np.zeros(4, np.uint8) for _ in range(250)]
    bad_par = [np.zeros(4, np.uint8) for _ in range(6)]
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.encode_batch_host(objs + bad, data + [b.ctypes.data for b in bad_data],
                              parity + [b.ctypes.data for b in bad_par],
                              data_len=dlen + [4] * 250)
    assert e.value.name == "TooManyShards255"
    _check(objs, chunks_of, None)  # the valid object was still encoded

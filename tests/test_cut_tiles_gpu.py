"""RS tiles that a length boundary cuts, run inside the fast kernel.

The fast kernel masks a cut shard's 16-byte vectors at its length: inputs
read as zero past it (the crate's zero padding of a short last chunk,
filesystem.rs:1111), outputs are written up to it and not one byte further
(a rebuilt short chunk, chunk_reader.rs:216-222).  These sweeps put the
boundary at every interesting offset of a tile -- 1, 15, 16, 17 bytes, one
vector short of a tile, exactly a tile, a tile plus one, the shard end -- for
several (k, m), shard sizes that are and are not tile multiples, every input
and output width R the launches use, and compare with the oracle bit for
bit.  The shard stride is a multiple of 16 so the launches stay aligned (the
fast path); unaligned launches are the edge kernel's, covered elsewhere."""
from __future__ import annotations

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

TILE = 256 * 16 * 4  # rs_kernel.hip fast tile at V = 4 (r_total <= 4)


def _torch():
    import torch

    assert torch.cuda.is_available(), "HIP device visible to libmaxio_ec but not to torch"
    return torch


def _lengths(S):
    c = [1, 15, 16, 17, 4095, 4096, 4097, TILE - 16, TILE - 1, TILE, TILE + 1, TILE + 4101, S - 17, S - 1, S]
    return sorted({x for x in c if 0 < x <= S})


@pytest.mark.parametrize("k,m,S", [(4, 2, 3 * TILE), (8, 4, 2 * TILE + 48), (10, 4, TILE + 4096 + 32),
                                   (3, 7, 2 * TILE), (5, 3, 40_000)])
def test_short_data_chunk_at_every_offset(ctx, k, m, S):
    """One object per boundary offset, the short chunk at a different data
    index each time; encode, then lose that chunk and (when m > 1) one more
    shard and rebuild."""
    torch = _torch()
    lens = _lengths(S)
    stride = (S + 15) // 16 * 16
    rng = np.random.default_rng(k * 100 + m)
    for t, last in enumerate(lens):
        short = t % k
        dl = [S] * k
        dl[short] = last
        n = 3
        host = np.zeros((n, k + m, stride), np.uint8)
        host[:, :k, :S] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
        host[:, short, last:] = 0
        for o in range(n):
            want, _, rc = oracle.compute_parity([host[o, j, :dl[j]] for j in range(k)], m, S)
            assert rc == 0
            host[o, k:, :S] = np.stack(want)
        dev = torch.from_numpy(host).cuda()
        # Bytes past a short chunk's end hold garbage on the device: the
        # kernel must read them as zero, never load them into the parity.
        dev[:, short, last:S].fill_(0xA5)
        dev[:, k:].fill_(0x33)
        torch.cuda.synchronize()
        ctx.encode_strided_device(k, m, S, n, dev.data_ptr(), (k + m) * stride, stride, dev[:, k:].data_ptr(),
                                  (k + m) * stride, stride, data_len=dl)
        torch.cuda.synchronize()
        got = dev.cpu().numpy()
        assert np.array_equal(got[:, k:, :S], host[:, k:, :S]), (k, m, S, short, last)
        # rebuild the short chunk (and one parity shard): written to `last` only
        present = np.ones(n * (k + m), np.uint8)
        lost = [short] + ([k + m - 1] if m > 1 else [])
        for o in range(n):
            for i in lost:
                present[o * (k + m) + i] = 0
        dev[:, short].fill_(0x77)
        dev[:, k + m - 1].fill_(0x77)
        torch.cuda.synchronize()
        rc, st = ctx.reconstruct_strided_device(k, m, S, n, dev.data_ptr(), (k + m) * stride, stride, present,
                                                shard_len=dl + [S] * m)
        torch.cuda.synchronize()
        assert rc == 0 and (st == 0).all()
        got = dev.cpu().numpy()
        assert np.array_equal(got[:, short, :last], host[:, short, :last]), (k, m, S, short, last)
        assert (got[:, short, last:] == 0x77).all(), (k, m, S, short, last)  # not one byte past the end
        if m > 1:
            assert np.array_equal(got[:, k + m - 1, :S], host[:, k + m - 1, :S])


@pytest.mark.parametrize("r", [1, 2, 3, 4, 5, 6, 8])
def test_rebuild_r_short_shards_at_once(ctx, r):
    """r shards rebuilt in one launch (R = r), every one of them short by a
    different amount, k = 8, m = r."""
    torch = _torch()
    k, m, S = 8, r, 2 * TILE + 160
    stride = S
    lens_pool = _lengths(S)
    rng = np.random.default_rng(r)
    n = 4
    dl = [S] * k
    for i in range(r):
        dl[i] = lens_pool[(3 * i + r) % len(lens_pool)]
    host = np.zeros((n, k + m, stride), np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    for j in range(k):
        host[:, j, dl[j]:] = 0
    for o in range(n):
        want, _, rc = oracle.compute_parity([host[o, j, :dl[j]] for j in range(k)], m, S)
        host[o, k:] = np.stack(want)
    dev = torch.from_numpy(host).cuda()
    present = np.ones(n * (k + m), np.uint8)
    for o in range(n):
        for i in range(r):
            present[o * (k + m) + i] = 0
    for i in range(r):
        dev[:, i].fill_(0x5C)
    torch.cuda.synchronize()
    rc, st = ctx.reconstruct_strided_device(k, m, S, n, dev.data_ptr(), (k + m) * stride, stride, present,
                                            shard_len=dl + [S] * m)
    torch.cuda.synchronize()
    assert rc == 0 and (st == 0).all()
    got = dev.cpu().numpy()
    for i in range(r):
        assert np.array_equal(got[:, i, :dl[i]], host[:, i, :dl[i]]), (r, i, dl[i])
        assert (got[:, i, dl[i]:] == 0x5C).all(), (r, i, dl[i])

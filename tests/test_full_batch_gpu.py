"""GPU: BASELINE configs[1] and configs[2] at their full batch sizes, with
the shipping grid (no cap): most tiles run in grid-stride iterations >= 2.

* configs[1] — RS encode 4+2, 10 MiB chunks, 1024 objects (40 GiB in, 20 GiB
  out): 655 360 tiles over at most 262 144 workgroups.  Every object is
  checked by a round trip (two data shards of every object erased and
  rebuilt from the parity just written — a wrong parity byte anywhere
  changes the rebuilt data), and a strided sample that lands in every
  grid-stride iteration of both grids the tuner may pick is compared byte
  for byte with the oracle.
* configs[2] — reconstruct 8+4 with 2 seeded data erasures per object and
  per-chunk SHA-256 verification of the 10 survivors, 1 MiB chunks, 8192
  data chunks (1024 objects): every rebuilt shard equals the original, and
  the sample's rebuilt bytes equal the oracle's reconstruct.

Reference: filesystem.rs:1121-1124 (encode), chunk_reader.rs:176-211
(verify -> erasure -> reconstruct).
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

N_OBJ = 1024


def _torch():
    import torch

    return torch


def _iteration_sample(tiles_per_obj, n_obj, n_cus):
    """Objects on both sides of every grid-stride iteration boundary, for
    the grids the shipping kernel runs at (1024 / 512 / 256 workgroups per
    CU), plus the first and last object."""
    s = {0, n_obj - 1}
    for bpc in (1024, 512, 256):
        grid = bpc * n_cus
        b = grid
        while b < tiles_per_obj * n_obj:
            o = b // tiles_per_obj
            s.update({o, min(o + 1, n_obj - 1), max(o - 1, 0)})
            b += grid
    return sorted(s)


def test_config1_full_batch(ctx):
    torch = _torch()
    k, m, S, n = 4, 2, 10 << 20, N_OBJ
    dev = torch.device("cuda", 0)
    n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    g = torch.Generator(device="cuda").manual_seed(0x6D6178696F)
    t = torch.empty((n, k + m, S), dtype=torch.uint8, device="cuda")
    t[:, :k].random_(0, 256, generator=g)
    t[:, k:].fill_(0)
    torch.cuda.synchronize()
    # the bench's layout: [n][k+m][S], parity at k*S of each object
    ctx.encode_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, t.data_ptr() + k * S, (k + m) * S, S)
    torch.cuda.synchronize()
    # every grid-stride iteration against the oracle
    sample = _iteration_sample(S // 16384, n, n_cus)
    assert len(sample) >= 6
    for o in sample:
        h = t[o].cpu().numpy()
        want = oracle.encode(list(h[:k]), m, S)
        for i in range(m):
            assert np.array_equal(h[k + i], want[i]), (o, i)
    # every object: erase data shards 0 and 2, rebuild them from the parity
    keep = t[:, [0, 2]].clone()
    t[:, [0, 2]].fill_(0xA5)
    present = np.ones(n * (k + m), np.uint8)
    present.reshape(n, k + m)[:, [0, 2]] = 0
    torch.cuda.synchronize()
    rc, status = ctx.reconstruct_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, present)
    torch.cuda.synchronize()
    assert rc == 0 and not status.any() and present.all()
    assert torch.equal(t[:, [0, 2]], keep), "round trip through the parity of some object differs"
    del t, keep
    torch.cuda.empty_cache()


def test_config2_full_batch(ctx):
    torch = _torch()
    k, m, S, n = 8, 4, 1 << 20, N_OBJ
    dev = torch.device("cuda", 0)
    n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    g = torch.Generator(device="cuda").manual_seed(0x6D6178696F + 3)
    t = torch.empty((n, k + m, S), dtype=torch.uint8, device="cuda")
    t[:, :k].random_(0, 256, generator=g)
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.encode_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, t.data_ptr() + k * S, (k + m) * S, S,
                              digests_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    ref = t.clone()
    # two seeded data erasures per object, garbage in their slots
    rng = np.random.default_rng(0x6D6178696F)
    present = np.ones((n, k + m), np.uint8)
    miss = np.stack([rng.choice(k, 2, replace=False) for _ in range(n)])
    for o in range(n):
        present[o, miss[o]] = 0
    idx = torch.from_numpy(miss).to(dev)
    rows = torch.arange(n, device=dev).unsqueeze(1)
    t[rows, idx] = 0x5A
    torch.cuda.synchronize()
    p = present.reshape(-1).copy()
    rc, status = ctx.reconstruct_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, p,
                                                expected_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    assert rc == 0 and not status.any() and p.all()
    assert torch.equal(t, ref), "some rebuilt shard differs from the encoded object"
    # the sample's rebuilt bytes against the oracle's reconstruct of its
    # survivors (the R = 2 decode runs 16 KiB tiles: 64 per object)
    for o in _iteration_sample(S // 16384, n, n_cus):
        h = ref[o].cpu().numpy()
        shards = [None if not present[o, i] else h[i] for i in range(k + m)]
        bufs, pres, orc = oracle.reconstruct(shards, k, m, S)
        assert orc == 0
        got = t[o].cpu().numpy()
        for i in miss[o]:
            assert np.array_equal(got[i], bufs[i]), (o, i)
        for i in range(k + m):
            assert hashlib.sha256(got[i].tobytes()).digest() == bytes(dig[o, i].cpu().numpy()), (o, i)
    del t, ref
    torch.cuda.empty_cache()

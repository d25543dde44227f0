"""GPU: mxec_batch_alloc, the placement-probing allocator for device-resident
batches (placement.cpp): it returns HBM laid out [n][k+m][shard_stride] with
the stride one of its candidates, probe times for the candidates it tried,
and an encode over the batch through mxec_encode_strided_device is bit-exact
against the oracle (reference: the crate's encode at filesystem.rs:1121-1124,
per object).  Errors: the k + m > 255 guard, a zero-object batch, freeing a
pointer it did not hand out."""
from __future__ import annotations

import numpy as np
import pytest

import maxio_amd
import oracle

pytestmark = pytest.mark.gpu

M = 1 << 20


class _DevMem:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 2, "strides": None}


@pytest.mark.parametrize("k,m,S,n", [(4, 2, 4 * M + 48, 24), (8, 4, M, 40), (10, 4, 3000, 7)])
def test_batch_alloc_layout_and_encode(ctx, k, m, S, n):
    import torch

    p, stride, probe = ctx.batch_alloc(k, m, S, n)
    try:
        pads = [(2 << 20) + (64 << 10), 6 << 20] if S >= 4 * M else [0, 256 << 10]
        assert stride - S in pads, (stride, pads)
        assert sum(1 for x in probe if x > 0) >= 2 and all(x == -1 or x > 0 for x in probe), probe
        buf = torch.as_tensor(_DevMem(p, n * (k + m) * stride), device="cuda").view(n, k + m, stride)
        g = torch.Generator(device="cuda").manual_seed(k * 1000 + n)
        buf[:, :k, :S] = torch.randint(0, 256, (n, k, S), dtype=torch.uint8, device="cuda", generator=g)
        torch.cuda.synchronize()
        ctx.encode_strided_device(k, m, S, n, p, (k + m) * stride, stride, p + k * stride, (k + m) * stride, stride)
        torch.cuda.synchronize()
        host = buf[:, :, :S].cpu().numpy()
        for o in sorted({0, n // 2, n - 1}):
            want = oracle.encode(list(host[o, :k]), m, S)
            for i in range(m):
                assert np.array_equal(host[o, k + i], want[i]), (o, i)
        del buf
    finally:
        ctx.batch_free(p)


def test_batch_alloc_errors(ctx):
    with pytest.raises(maxio_amd.RSError):
        ctx.batch_alloc(250, 10, M, 4)  # filesystem.rs:1095's k + m > 255 guard
    with pytest.raises(maxio_amd.RSError):
        ctx.batch_alloc(4, 2, M, 0)
    with pytest.raises(maxio_amd.RSError):
        ctx.batch_free(0x1000)

"""GPU: the failing-object contract of the batched, verifying reconstructs
(VERDICT r2 item 8).

The reference rebuilds one object per call and returns before touching
anything when fewer than k shards survive verification
(chunk_reader.rs:199-208).  The batched device calls keep going for the other
objects of the batch, so the contract pinned here is:

* the call returns MXEC_E_TOO_FEW_SHARDS_PRESENT (-10) and its message, the
  failing objects get -10 in status_out, every other object 0;
* every healthy object is rebuilt bit-exact (parity from the oracle, the
  crate's algorithm);
* a failing object's present mask comes back as its input mask minus the
  shards whose digest mismatched;
* a failing object's bytes are untouched except, on the strided call (whose
  decode runs speculatively beside the hash), the shards that were already
  missing in its input mask -- and only when that mask alone had k shards,
  since a decode needs k; the corrupt shards themselves are never written.
  mxec_reconstruct_batch_device verifies before it rebuilds, so there the
  failing object is untouched entirely.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

K, M, S, N = 8, 4, 1 << 16, 12
CORRUPT_OBJ, SHORT_OBJ = 7, 4  # > m bad after verify / < k present before it


def _batch():
    rng = np.random.default_rng(0xC0)
    host = rng.integers(0, 256, (N, K + M, S), dtype=np.uint8)
    for o in range(N):
        host[o, K:] = np.stack(oracle.encode(list(host[o, :K]), M, S))
    digests = np.stack([[np.frombuffer(hashlib.sha256(host[o, i].tobytes()).digest(), np.uint8)
                         for i in range(K + M)] for o in range(N)])
    given = host.copy()  # what the call receives
    present = np.ones((N, K + M), np.uint8)
    for o in range(N):
        for i in rng.choice(K + M, int(rng.integers(0, 3)), replace=False):
            present[o, i] = 0
    # CORRUPT_OBJ: 2 missing + 3 silently corrupt present shards -> 7 < k after verify,
    # but 10 >= k in the mask as given (the speculative decode runs for it)
    present[CORRUPT_OBJ] = 1
    present[CORRUPT_OBJ, [0, 9]] = 0
    corrupt = [1, 2, 10]
    for i in corrupt:
        given[CORRUPT_OBJ, i, 123 * i] ^= 0x5A
    # SHORT_OBJ: 5 missing -> 7 present before verification (no decode at all)
    present[SHORT_OBJ] = 1
    present[SHORT_OBJ, [0, 3, 5, 8, 11]] = 0
    for o in range(N):
        for i in range(K + M):
            if not present[o, i]:
                given[o, i] = 0xEE  # a missing shard's buffer: the rebuild target
    return host, digests, given, present, corrupt


def _check(host, given, out, present_in, present_out, status, rc, msg, corrupt, speculative):
    assert rc == -10, rc
    assert "too many missing/corrupt shards" in msg
    for o in range(N):
        if o in (CORRUPT_OBJ, SHORT_OBJ):
            assert status[o] == -10, (o, status[o])
            continue
        assert status[o] == 0, (o, status[o])
        assert present_out[o].all(), o
        assert np.array_equal(out[o], host[o]), o  # bit-exact vs the oracle's parity
    # present mask: input minus mismatches
    want = present_in[CORRUPT_OBJ].copy()
    want[corrupt] = 0
    assert np.array_equal(present_out[CORRUPT_OBJ], want)
    assert np.array_equal(present_out[SHORT_OBJ], present_in[SHORT_OBJ])
    # bytes: nothing but the speculatively decoded missing shards may change
    for i in range(K + M):
        if speculative and not present_in[CORRUPT_OBJ, i]:
            continue  # may hold the speculative decode (from corrupt inputs)
        assert np.array_equal(out[CORRUPT_OBJ, i], given[CORRUPT_OBJ, i]), ("corrupt obj shard", i)
    assert np.array_equal(out[SHORT_OBJ], given[SHORT_OBJ])


def test_failing_object_contract_strided(ctx):
    import torch

    host, digests, given, present, corrupt = _batch()
    dev = torch.from_numpy(given.copy()).cuda()
    dig = torch.from_numpy(digests).cuda()
    pres = present.reshape(-1).copy()
    torch.cuda.synchronize()
    rc, status = ctx.reconstruct_strided_device(K, M, S, N, dev.data_ptr(), (K + M) * S, S, pres,
                                                expected_ptr=dig.data_ptr())
    msg = ctx._lib.mxec_last_error().decode()
    torch.cuda.synchronize()
    _check(host, given, dev.cpu().numpy(), present, pres.reshape(N, K + M), status, rc, msg, corrupt,
           speculative=True)


def test_failing_object_contract_mixed_batch(ctx):
    import torch

    host, digests, given, present, corrupt = _batch()
    dev = torch.from_numpy(given.copy()).cuda()
    dig = torch.from_numpy(digests).cuda()
    pres = present.reshape(-1).copy()
    base, ss = dev.data_ptr(), S
    ptrs = [base + (o * (K + M) + i) * ss for o in range(N) for i in range(K + M)]
    torch.cuda.synchronize()
    rc, status = ctx.reconstruct_batch_device([(K, M, S)] * N, ptrs, pres, expected_ptr=dig.data_ptr())
    msg = ctx._lib.mxec_last_error().decode()
    torch.cuda.synchronize()
    _check(host, given, dev.cpu().numpy(), present, pres.reshape(N, K + M), status, rc, msg, corrupt,
           speculative=False)

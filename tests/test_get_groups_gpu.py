"""GPU: the verified host GET, as one verification group, as the count the
library picks per wave (the default) and as pipelined groups (MXEC_GET_VGROUPS; pipeline.cpp verify_cuts / verify_enqueue
/ verify_collect): group j + 1's pieces go up and hash while the host
collects group j's verdicts, rebuilds it and sends its shards down.  Reference: try_reconstruct_data_chunk,
chunk_reader.rs:157-226, per object.

160 objects of 8+4 x 1 MiB (some shards shorter) from page-locked memory, two
erasures each, silent corruption in objects on both sides of every group
boundary, and two objects (one early, one late) with more bad shards than
parity: every rebuilt shard equals the original, every failing object's
present shards are untouched (its missing shards' buffers are undefined: the
speculative rebuild, MXEC_GET_SPECULATE, wrote them before the verdict) and
its status is MXEC_E_TOO_FEW_SHARDS_PRESENT, and mxec_ctx_pipe_stats shows
the wave ran as that many groups.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M = 1 << 20
TOO_FEW_SHARDS_PRESENT = -10  # include/maxio_ec.h MXEC_E_TOO_FEW_SHARDS_PRESENT


@pytest.mark.parametrize("groups", [0, 1, 3])
def test_verified_get_in_groups_matches_originals(ctx_with, groups):
    """groups 0: the per-wave choice (pipeline.cpp verify_cuts), which keeps
    this batch -- a 34 ms upload against a 19 ms chain -- as one group."""
    ctx = ctx_with(MXEC_GET_VGROUPS=str(groups))
    k, m, n = 8, 4, 160
    S = M
    rng = np.random.default_rng(4242)
    buf = ctx.host_array(n * (k + m) * S).reshape(n, k + m, S)
    flat = buf.reshape(-1)
    step = 256 * M
    for o in range(0, flat.size, step):
        flat[o:o + min(step, flat.size - o)] = np.frombuffer(rng.bytes(min(step, flat.size - o)), np.uint8)
    dl = [S] * (k - 1) + [S - 4097]
    objs = [(k, m, S)] * n
    dig = np.zeros(n * (k + m) * 32, np.uint8)
    st = ctx.encode_batch_host(objs, [buf[o, j].ctypes.data for o in range(n) for j in range(k)],
                               [buf[o, k + i].ctypes.data for o in range(n) for i in range(m)],
                               data_len=dl * n, digests=dig)
    assert (st == 0).all()
    for o in (0, n // 2, n - 1):  # the digests the GET checks against
        for j in range(k + m):
            L = dl[j] if j < k else S
            assert dig[(o * (k + m) + j) * 32:][:32].tobytes() == hashlib.sha256(buf[o, j, :L].tobytes()).digest()
    ref = buf.copy()
    lens = dl + [S] * m
    present = np.ones((n, k + m), np.uint8)
    for o in range(n):
        for i in rng.choice(k + m, 2, replace=False):
            present[o, i] = 0
            buf[o, i] = 0x5A
    # silent corruption of a present shard: near every third of the batch (the
    # model picks a few groups here) and at both ends
    corrupt = [0, 1, 52, 53, 54, 105, 106, 107, n - 2, n - 1]
    for o in corrupt:
        c = int(np.flatnonzero(present[o])[o % 3])
        buf[o, c, 1000 + o] ^= 0x10
    # more bad shards than parity: 2 erased + 3 corrupt -> fails, untouched
    failing = [17, 140]
    for o in failing:
        for c in np.flatnonzero(present[o])[:3]:
            buf[o, int(c), 7] ^= 0xFF
    before_fail = {o: buf[o].copy() for o in failing}
    s0 = ctx.pipe_stats()
    pr = present.reshape(-1).copy()
    rc, status = ctx.reconstruct_batch_host(objs, [buf[o, i].ctypes.data for o in range(n) for i in range(k + m)],
                                            pr, shard_len=lens * n, expected=dig)
    s1 = ctx.pipe_stats()
    assert rc == TOO_FEW_SHARDS_PRESENT, rc  # the batch's first failing object
    assert s1["verify_waves"] > s0["verify_waves"]
    want = groups or 1
    assert s1["verify_groups"] - s0["verify_groups"] == want * (s1["verify_waves"] - s0["verify_waves"]), (s0, s1)
    for o in range(n):
        if o in failing:
            assert status[o] == TOO_FEW_SHARDS_PRESENT, (o, status[o])
            for i in np.flatnonzero(present[o]):
                assert np.array_equal(buf[o, i], before_fail[o][i]), f"failing object {o}'s shard {i} was written"
            continue
        assert status[o] == 0, (o, status[o])
        assert pr[o * (k + m):(o + 1) * (k + m)].all(), o
        for i in range(k + m):  # erased and silently corrupted shards alike come back exact
            assert np.array_equal(buf[o, i, :lens[i]], ref[o, i, :lens[i]]), (o, i)
    ctx.host_free(buf)

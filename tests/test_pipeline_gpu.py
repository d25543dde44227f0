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


@pytest.mark.parametrize("piece_mb", ["1", "2", "4", "0", ""])
def test_batch_host_digests_in_pieces(ctx_with, piece_mb):
    """With digests the wave runs piece-major (MXEC_PIPE_PIECE_MB; unset
    ("") = chosen per wave among 1 / 2 / 4 MiB; 0 = the group form):
    every chunk is hashed piece by piece, its chain carried in a device
    state slot from launch to launch.  Shards over several pieces and off
    the piece grid, last chunks that end mid-piece, on a piece boundary
    (the first one included), one byte into a piece, empty, and objects of
    one piece beside them: parity and every digest equal to the oracle and
    hashlib."""
    ctx = ctx_with(MXEC_PIPE_PIECE_MB=piece_mb)
    rng = np.random.default_rng(40 + int(piece_mb or 9))
    M = 1 << 20
    specs = [(4, 2, 3 * M + 100, None), (4, 2, 3 * M + 100, 2 * M + 17), (8, 4, 2 * M, M),
             (10, 4, M + 64, M + 1), (4, 2, 3 * M + 100, 0), (1, 2, 5 * M + 3, None),
             (4, 2, 65536, 17), (3, 5, 100, 1), (4, 2, M + M // 4, M // 4), (4, 2, 2 * M + M // 4, None),
             (4, 2, 2 * M, 960 << 10), (4, 2, 192 << 10, 64 << 10), (4, 2, 960 << 10, None)]
    objs, data, dlen, parity, chunks_of = _objects(rng, specs)
    digests = np.zeros(sum(k + m for (k, m, _) in objs) * 32, np.uint8)
    status = ctx.encode_batch_host(objs, data, parity, data_len=dlen, digests=digests)
    assert (status == 0).all()
    _check(objs, chunks_of, digests)


@pytest.mark.parametrize("ramp_kb,copy2d", [("", ""), ("0", "1"), ("256", "1"), ("64", "1"), ("64", "0")])
def test_batch_host_pinned_pieces_2d(ctx_with, ramp_kb, copy2d):
    """Page-locked bodies in pieces, defaults (uniform pieces, 1D copies)
    and the lab knobs (lab builds only): the same piece of an object's k
    chunks (and of its m parity chunks) as one 2D copy (MXEC_PIPE_COPY2D=1),
    a ramp of pieces from MXEC_PIPE_RAMP_KB up to 1 MiB;
    shards off the piece grid.  Parity and digests equal to the oracle."""
    from conftest import lab_build

    torch = pytest.importorskip("torch")
    if (ramp_kb or copy2d) and not lab_build():
        pytest.skip("MXEC_PIPE_RAMP_KB / MXEC_PIPE_COPY2D exist in lab builds only")
    ctx = ctx_with(MXEC_PIPE_RAMP_KB=ramp_kb, MXEC_PIPE_COPY2D=copy2d)
    k, m, s, n = 4, 2, 3 * (1 << 20) + 128, 6
    host = torch.randint(0, 256, (n, k, s), dtype=torch.uint8).pin_memory()
    par = torch.zeros((n, m, s), dtype=torch.uint8).pin_memory()
    objs = [(k, m, s)] * n
    data = [host[o, j].data_ptr() for o in range(n) for j in range(k)]
    parity = [par[o, i].data_ptr() for o in range(n) for i in range(m)]
    digests = np.zeros(n * (k + m) * 32, np.uint8)
    status = ctx.encode_batch_host(objs, data, parity, digests=digests)
    assert (status == 0).all()
    h, p = host.numpy(), par.numpy()
    _check(objs, [([h[o, j] for j in range(k)], [p[o, i] for i in range(m)]) for o in range(n)], digests)


def test_batch_host_digests_past_quad_capacity(ctx):
    """A wave of more chunks than the lag quad form holds (64 per CU: 16 384
    on 256 CUs) takes the group form (whole chunks, one launch after the
    upload) instead of pieces: 2 800 objects of 4+2 x 4 KiB = 16 800 chunks,
    parity and digests against the oracle for a sample, every digest against
    hashlib; then the verified GET of the same objects with one erasure and
    one corrupt shard in a few of them."""
    import hashlib

    rng = np.random.default_rng(61)
    k, m, s, n = 4, 2, 4096, 2800
    data = rng.integers(0, 256, (n, k, s), dtype=np.uint8)
    par = np.zeros((n, m, s), np.uint8)
    objs = [(k, m, s)] * n
    digests = np.zeros(n * (k + m) * 32, np.uint8)
    status = ctx.encode_batch_host(objs, [data[o, j].ctypes.data for o in range(n) for j in range(k)],
                                   [par[o, i].ctypes.data for o in range(n) for i in range(m)], digests=digests)
    assert (status == 0).all()
    sample = [0, 1, n // 2, n - 1]
    _check([objs[o] for o in sample], [([data[o, j] for j in range(k)], [par[o, i] for i in range(m)])
                                       for o in sample], None)
    for o in range(0, n, 97):
        for t in range(k + m):
            x = data[o, t] if t < k else par[o, t - k]
            assert digests[(o * (k + m) + t) * 32:(o * (k + m) + t + 1) * 32].tobytes() == hashlib.sha256(x).digest()
    shards = np.concatenate([data, par], axis=1).copy()
    want = shards.copy()
    present = np.ones(n * (k + m), np.uint8)
    for o in range(0, n, 211):
        present[o * (k + m) + 1] = 0
        shards[o, 1] = 0xEE
        shards[o, 4, 7] ^= 0x10  # silently corrupt: verification turns it into an erasure
    ptrs = [shards[o, i].ctypes.data for o in range(n) for i in range(k + m)]
    rc, st = ctx.reconstruct_batch_host(objs, ptrs, present, expected=digests)
    assert rc == 0 and not st.any()
    assert np.array_equal(shards[:, :k], want[:, :k])


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


# ---- mxec_reconstruct_batch_host (GET from host memory) -------------------------------


def _rec_batch(rng, specs, pinned=None):
    """Encoded objects (oracle parity, hashlib digests) with seeded erasures
    (buffers of missing shards filled with 0xEE), silently corrupt shards as
    given: returns (objs, ptrs, lens, present, expected, originals, buffers)."""
    import hashlib

    objs, ptrs, lens, present, expected, originals, bufs = [], [], [], [], [], [], []
    for (k, m, s, last, lost, corrupt) in specs:
        chunks = [rng.integers(0, 256, s, dtype=np.uint8) for _ in range(k)]
        if last is not None:
            chunks[-1] = chunks[-1][:last].copy()
        par, dig, rc = oracle.compute_parity(chunks, m, s)
        assert rc == 0
        shards = [c.copy() for c in chunks] + [np.asarray(p, np.uint8).copy() for p in par]
        originals.append([x.copy() for x in shards])
        objs.append((k, m, s))
        for i, x in enumerate(shards):
            b = pinned(x.size) if pinned else np.empty(max(1, x.size), np.uint8)
            b[:x.size] = x
            if i in lost:
                b[:x.size] = 0xEE
            if i in corrupt:
                b[x.size // 2] ^= 0x40
            bufs.append(b)
            ptrs.append(b.ctypes.data)
            lens.append(x.size)
            present.append(0 if i in lost else 1)
            expected.append(np.frombuffer(dig[i], np.uint8))
    return (objs, ptrs, lens, np.array(present, np.uint8), np.concatenate(expected).copy(), originals, bufs)


@pytest.mark.parametrize("verify", [True, False])
def test_reconstruct_batch_host_mixed(ctx, verify):
    """Mixed shapes, short last chunks, 1..m erasures (data and parity), and
    with verification a silently corrupt present shard per object that still
    has room: every object comes back bit-exact (oracle parity), present
    all 1."""
    rng = np.random.default_rng(41)
    specs = []
    for t in range(18):
        k, m = [(4, 2), (8, 4), (10, 4), (1, 2)][t % 4]
        s = [4096, 65536 + 16, 1 << 20, 300][t % 4]
        last = None if t % 3 else int(rng.integers(1, s))
        e = int(rng.integers(1, m + 1)) - (1 if verify and m > 1 else 0)
        lost = set(int(x) for x in rng.choice(k + m, max(1, e), replace=False))
        keep = [i for i in range(k + m) if i not in lost]
        corrupt = {int(rng.choice(keep))} if verify and len(lost) < m else set()
        specs.append((k, m, s, last, lost, corrupt))
    objs, ptrs, lens, present, expected, originals, bufs = _rec_batch(rng, specs)
    rc, status = ctx.reconstruct_batch_host(objs, ptrs, present, shard_len=lens,
                                            expected=expected if verify else None)
    assert rc == 0 and not status.any() and present.all()
    g = 0
    for o, (k, m, s) in enumerate(objs):
        for i in range(k + m):
            n = lens[g + i]
            assert np.array_equal(bufs[g + i][:n], originals[o][i]), (o, i)
        g += k + m


@pytest.mark.parametrize("piece_mb", ["1", "2", "4", "0", ""])
def test_reconstruct_batch_host_verify_in_pieces(ctx_with, piece_mb):
    """With verification the present shards go up and are hashed piece by
    piece (MXEC_PIPE_PIECE_MB; 0 = one launch after the whole upload):
    shards over several pieces and off the piece grid, short and empty last
    chunks, a corrupt present shard caught as an erasure, an object that
    fails (its present shards untouched; with whole-chunk hashing, piece 0,
    nothing of it written), the rest bit-exact."""
    ctx = ctx_with(MXEC_PIPE_PIECE_MB=piece_mb)
    rng = np.random.default_rng(50 + int(piece_mb or 9))
    M = 1 << 20
    specs = [(4, 2, 3 * M + 100, None, {1}, {4}), (4, 2, 3 * M + 100, 2 * M + 17, {0, 5}, set()),
             (8, 4, 2 * M, M, {3}, {9}), (4, 2, 3 * M + 100, 0, {2}, {0}),
             (4, 2, 2 * M + 64, None, {0, 1}, {2}),  # fails: 3 of 6 gone
             (1, 2, 5 * M + 3, None, {1}, set()), (4, 2, 65536, 17, {3}, set()),
             (4, 2, M + M // 4, M // 4, {5}, {3}), (4, 2, 2 * M, 960 << 10, {0}, {3})]
    objs, ptrs, lens, present, expected, originals, bufs = _rec_batch(rng, specs)
    before = [b.copy() for b in bufs]
    p = present.copy()
    rc, status = ctx.reconstruct_batch_host(objs, ptrs, p, shard_len=lens, expected=expected)
    assert rc == -10 and list(status) == [0, 0, 0, 0, -10, 0, 0, 0, 0]
    g = 0
    for o, (k, m, s) in enumerate(objs):
        for i in range(k + m):
            if o == 4:
                if present[g + i] or piece_mb == "0":  # the speculative rebuild may have written the missing ones
                    assert np.array_equal(bufs[g + i], before[g + i])
            else:
                assert np.array_equal(bufs[g + i][:lens[g + i]], originals[o][i]), (o, i)
        g += k + m


def test_reconstruct_batch_host_failing_object(ctx):
    """An object with more than m shards lost or corrupt: -10 for it and the
    call, its present shards untouched (its missing shards' buffers are
    undefined: rebuilt speculatively before the verdict), the present mask
    minus the mismatches; the other objects bit-exact
    (chunk_reader.rs:199-208)."""
    rng = np.random.default_rng(42)
    specs = [(4, 2, 8192, None, {0}, set()), (4, 2, 8192, None, {1, 5}, {0}), (8, 4, 4096, 100, {2}, set())]
    objs, ptrs, lens, present, expected, originals, bufs = _rec_batch(rng, specs)
    before = [b.copy() for b in bufs]
    p = present.copy()
    rc, status = ctx.reconstruct_batch_host(objs, ptrs, p, shard_len=lens, expected=expected)
    assert rc == -10 and list(status) == [0, -10, 0]
    assert "too many missing/corrupt shards" in ctx._lib.mxec_last_error().decode()
    for i in (0, 2, 3, 4):  # the present shards (0 corrupt) of the failing object
        assert np.array_equal(bufs[6 + i], before[6 + i])
    assert list(p[6:12]) == [0, 0, 1, 1, 1, 0]
    for o, g in ((0, 0), (2, 12)):
        k, m, s = objs[o]
        for i in range(k + m):
            assert np.array_equal(bufs[g + i][:lens[g + i]], originals[o][i]), (o, i)


def test_reconstruct_batch_host_pinned_config2_shape(ctx):
    """configs[1]'s shape from page-locked memory (the direct-DMA path):
    8 x 4+2 x 10 MiB, two erasures each, verified: bit-exact."""
    rng = np.random.default_rng(43)
    keep = []

    def pinned(n):
        a = ctx.host_array(max(1, n))
        keep.append(a)
        return a

    specs = [(4, 2, 10 << 20, None, set(int(x) for x in rng.choice(6, 2, replace=False)), set()) for _ in range(8)]
    objs, ptrs, lens, present, expected, originals, bufs = _rec_batch(rng, specs, pinned=pinned)
    rc, status = ctx.reconstruct_batch_host(objs, ptrs, present, shard_len=lens, expected=expected)
    assert rc == 0 and present.all()
    for o in range(8):
        for i in range(6):
            assert np.array_equal(bufs[o * 6 + i][:lens[o * 6 + i]], originals[o][i]), (o, i)


@pytest.mark.parametrize("k,m,s", [(4, 2, 65536), (8, 4, 1024 + 16), (10, 4, 4096 + 48), (1, 2, 300)])
@pytest.mark.parametrize("verify", [False, True])
def test_reconstruct_batch_host_every_pattern(ctx, k, m, s, verify):
    """Every erasure pattern of 1..m shards (data and parity) for the shapes
    MaxIO runs, one object per pattern, all in ONE call: 793 distinct decode
    matrices at 8+4, 1 471 at 10+4, in one grouped launch each wave.  With
    verification every object that has room also gets one silently corrupt
    present shard (chunk_reader.rs:176-198 turns it into an erasure), so the
    effective pattern reaches m.  Every fifth object has a short last chunk.
    Bit-exact against the oracle's parity, present mask all 1 afterwards
    (reed-solomon-erasure 6.0.0 reconstruct, chunk_reader.rs:157-226)."""
    import itertools

    rng = np.random.default_rng(k * 100 + m + (7 if verify else 0))
    pats = [set(p) for e in range(1, m + 1) for p in itertools.combinations(range(k + m), e)]
    specs = []
    for i, lost in enumerate(pats):
        last = int(rng.integers(1, s)) if i % 5 == 0 else None
        keep = [j for j in range(k + m) if j not in lost]
        corrupt = {int(rng.choice(keep))} if verify and len(lost) < m else set()
        specs.append((k, m, s, last, lost, corrupt))
    objs, ptrs, lens, present, expected, originals, bufs = _rec_batch(rng, specs)
    rc, status = ctx.reconstruct_batch_host(objs, ptrs, present, shard_len=lens,
                                            expected=expected if verify else None)
    assert rc == 0 and not status.any() and present.all()
    for o in range(len(objs)):
        for i in range(k + m):
            g = o * (k + m) + i
            assert np.array_equal(bufs[g][:lens[g]], originals[o][i]), (sorted(pats[o]), i)


def test_batch_host_pieces_descriptor_tables_outgrow_first_block(ctx):
    """a piece-major wave's descriptor tables grow with pieces x
    shape classes (each piece re-issues one RS launch per (k, m, S) class and
    one hash launch), past the first block the wave reserves from its
    object count.  150 objects of distinct 64 MiB-class shard sizes (150
    classes x 64 one-MiB pieces: ~3 MB of tables against a ~2.1 MB first
    block) must encode like any other batch (the arena chains another
    block) instead of failing with MXEC_E_OOM.  k = 1: the crate's parity
    is a copy of the data (matrix [[1]]), so the check is cheap."""
    import hashlib

    n, M = 150, 1 << 20
    rng = np.random.default_rng(77)
    data = [rng.integers(0, 256, 4096, dtype=np.uint8) for _ in range(n)]
    sizes = [64 * M + 4096 * o for o in range(n)]
    outs = [np.full(s, 0xEE, np.uint8) for s in sizes]
    objs = [(1, 1, s) for s in sizes]
    digests = np.zeros(n * 2 * 32, np.uint8)
    status = ctx.encode_batch_host(objs, [d.ctypes.data for d in data], [o.ctypes.data for o in outs],
                                   data_len=[4096] * n, digests=digests)
    assert (status == 0).all()
    for o in range(n):
        assert np.array_equal(outs[o][:4096], data[o]) and not outs[o][4096:].any(), o
        assert digests[o * 64:o * 64 + 32].tobytes() == hashlib.sha256(data[o].tobytes()).digest(), o
    for o in range(0, n, 15):  # parity digests over the full (zero-padded) shard
        assert digests[o * 64 + 32:o * 64 + 64].tobytes() == hashlib.sha256(outs[o].tobytes()).digest(), o


@pytest.mark.parametrize("copy", ["auto", "waves", "sdma"])
def test_host_alloc_buffers_copy_modes(ctx_with, copy):
    """mxec_host_alloc buffers (mapped into the GPU's address space) through
    the host batch calls with MXEC_PIPE_COPY=auto (the default: SDMA while a
    timed probe finds it healthy, CU-wave copy kernels, copy_kernel.hip,
    while not), =waves (both by waves) and =sdma: a PUT with digests in pieces, shards off the
    piece grid and short last chunks, then a verified GET with two erasures
    per object and one corrupted present shard -- parity, digests and the
    rebuilt shards equal to the oracle / the originals in both modes."""
    import hashlib

    ctx = ctx_with(MXEC_PIPE_COPY=copy)
    rng = np.random.default_rng(91)
    k, m, n = 4, 2, 7
    S = 3 * (1 << 20) + 4096 + 48
    data = ctx.host_array(n * k * S).reshape(n, k, S)
    par = ctx.host_array(n * m * S).reshape(n, m, S)
    data[:] = rng.integers(0, 256, data.shape, dtype=np.uint8)
    par[:] = 0xEE
    dl = [S] * (k - 1) + [S - 3333]
    objs = [(k, m, S)] * n
    dptr = [data[o, j].ctypes.data for o in range(n) for j in range(k)]
    pptr = [par[o, i].ctypes.data for o in range(n) for i in range(m)]
    dig = np.zeros(n * (k + m) * 32, np.uint8)
    status = ctx.encode_batch_host(objs, dptr, pptr, data_len=dl * n, digests=dig)
    assert (status == 0).all()
    for o in range(n):
        want, want_dig, rc = oracle.compute_parity([data[o, j, :dl[j]] for j in range(k)], m, S)
        assert rc == 0
        for i in range(m):
            assert np.array_equal(par[o, i], want[i]), (copy, o, i)
        assert [dig[(o * (k + m) + t) * 32:(o * (k + m) + t + 1) * 32].tobytes() for t in range(k + m)] == want_dig
    ref_d, ref_p = data.copy(), par.copy()
    present = np.ones((n, k + m), np.uint8)
    for o in range(n):
        for i in rng.choice(k + m, 1 if o == 2 else 2, replace=False):
            present[o, i] = 0
            (data[o, i] if i < k else par[o, i - k])[:] = 0x5A
    # object 2 (one erasure): a present shard silently corrupted, caught, rebuilt
    c = int(np.flatnonzero(present[2])[0])
    (data[2, c] if c < k else par[2, c - k])[77] ^= 1
    sptr, slen = [], []
    for o in range(n):
        sptr += [data[o, j].ctypes.data for j in range(k)] + [par[o, i].ctypes.data for i in range(m)]
        slen += dl + [S] * m
    pr = present.reshape(-1).copy()
    rc, st = ctx.reconstruct_batch_host(objs, sptr, pr, shard_len=slen, expected=dig)
    assert rc == 0 and not st.any() and pr.all()
    for o in range(n):
        for j in range(k):
            assert np.array_equal(data[o, j, :dl[j]], ref_d[o, j, :dl[j]]), (copy, o, j)
        assert np.array_equal(par[o], ref_p[o]), (copy, o)
    assert hashlib.sha256(data[n - 1, 0].tobytes()).digest() == dig[(n - 1) * (k + m) * 32:][:32].tobytes()


@pytest.mark.parametrize("copy", ["waves", "sdma"])
def test_single_request_calls_on_host_alloc_buffers(ctx_with, copy):
    """The single-request entry points with mxec_host_alloc buffers: under
    MXEC_PIPE_COPY=waves the hash and reconstruct calls move them by CU-wave
    copy kernels (runtime.cpp upload_segments / download_segments; under
    auto they do so while the device's last SDMA probe found SDMA slow),
    under sdma by DMAs.  mxec_sha256_batch against hashlib (odd lengths and
    offsets); mxec_reconstruct with verification, two erasures and one
    corrupted shard, rebuilt in place in the caller's page-locked shards."""
    import ctypes
    import hashlib

    import maxio_amd.ec as E

    ctx = ctx_with(MXEC_PIPE_COPY=copy)
    rng = np.random.default_rng(93)
    blob = ctx.host_array(3 << 20)
    blob[:] = rng.integers(0, 256, blob.size, dtype=np.uint8)
    cuts = [(0, 0), (5, 1000), (4096, 1 << 20), (17, (1 << 20) + 333), (2 << 20, 64)]
    got = ctx.sha256([blob[o:o + n] for o, n in cuts])
    assert got == [hashlib.sha256(blob[o:o + n].tobytes()).digest() for o, n in cuts]
    k, m, S = 8, 4, (1 << 20) + 48
    sh = ctx.host_array((k + m) * S).reshape(k + m, S)
    sh[:k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
    par, dig = ctx.encode([sh[j] for j in range(k)], m, S)
    for i in range(m):
        sh[k + i] = par[i]
    ref = sh.copy()
    present = np.ones(k + m, np.uint8)
    for i in (1, 9):
        present[i] = 0
        sh[i] = 0x33
    sh[4, 100] ^= 0x10  # silent corruption: caught by the digest, rebuilt
    exp = np.frombuffer(b"".join(dig), np.uint8).copy()
    npres = ctypes.c_int(0)
    lens = (ctypes.c_size_t * (k + m))(*([S] * (k + m)))
    rc = ctx._lib.mxec_reconstruct(ctx.handle, k, m, S, E._pp([sh[i].ctypes.data for i in range(k + m)]), lens,
                                   exp.ctypes.data_as(E.N.U8P), present.ctypes.data_as(E.N.U8P), 0,
                                   ctypes.byref(npres))
    assert rc == 0 and present.all() and npres.value == k + m - 3
    assert np.array_equal(sh, ref)


@pytest.mark.parametrize("floor,waves", [("0", False), ("100000", True)])
def test_single_request_calls_follow_the_verdict(floor, waves):
    """under MXEC_PIPE_COPY=auto the single-request hash call
    copies mxec_host_alloc buffers by waves exactly while a measured slow
    bracket's hold lasts (capi.cpp copy_waves_get reads the holds).  An
    RS-only host GET with an unreachable floor is judged slow (its upload
    and download brackets); a mxec_sha256_batch issued right after it --
    well inside the 1-2 s holds -- moves its buffers by waves (wave_blocks
    rises); with floor 0 (no brackets, no verdict) it stays on SDMA.
    Digests against hashlib either way."""
    import hashlib

    from conftest import open_ctx

    ctx = open_ctx(2, 0, MXEC_PIPE_COPY="auto", MXEC_PIPE_SDMA_FLOOR=floor)
    try:
        k, m, n, S = 4, 2, 16, 4 * (1 << 20)
        rng = np.random.default_rng(4343)
        buf = ctx.host_array(n * (k + m) * S).reshape(n, k + m, S)
        buf[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
        objs = [(k, m, S)] * n
        st = ctx.encode_batch_host(objs, [buf[o, j].ctypes.data for o in range(n) for j in range(k)],
                                   [buf[o, k + i].ctypes.data for o in range(n) for i in range(m)])
        assert (st == 0).all()
        ref = buf.copy()
        buf[:, [0, 5]] = 0x11
        present = np.ones((n, k + m), np.uint8)
        present[:, [0, 5]] = 0
        pr = present.reshape(-1).copy()
        rc, st = ctx.reconstruct_batch_host(objs, [buf[o, i].ctypes.data for o in range(n) for i in range(k + m)], pr)
        assert rc == 0 and pr.all() and np.array_equal(buf, ref)
        s0 = ctx.pipe_stats()
        cuts = [(0, 1 << 20), (3 << 20, 5 << 20), (4096, 1000)]  # 16-byte phase kept (copy_phase_ok)
        flat = buf.reshape(-1)
        got = ctx.sha256([flat[o:o + ln] for o, ln in cuts])
        s1 = ctx.pipe_stats()
        assert got == [hashlib.sha256(flat[o:o + ln].tobytes()).digest() for o, ln in cuts]
        assert (s0["sdma_slow"] + s0["sdma_down_slow"] > 0) == waves, s0
        assert (s1["wave_blocks"] > s0["wave_blocks"]) == waves, (s0, s1)
        ctx.host_free(buf.reshape(-1))
    finally:
        ctx.close()

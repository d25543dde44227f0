"""GPU: the host pipeline's default copy forms on mxec_host_alloc buffers,
object for object against the oracle (reference: the PUT's parity and
digests, filesystem.rs:1107-1135; the GET's rebuild, chunk_reader.rs:157-226).

* PUT with digests in 2 / 4 MiB pieces (MXEC_PIPE_PIECE_MB, product knob) and
  with the piece size chosen per wave at a batch large enough to be
  upload-bound: the same piece of an object's k data chunks goes up as one
  2D SDMA copy (pipeline.cpp flush_up), its m parity pieces come down as
  one (flush_down).  mxec_ctx_pipe_stats proves the 2D copies ran.  Shards
  off the piece grid; a short and an empty last data chunk break the 2D run
  in the middle of the batch.  EVERY object's parity and all k+m digests
  equal oracle.compute_parity.
* The CU-wave copies (MXEC_PIPE_COPY=waves, or auto once a timed piece of
  uploads ran below MXEC_PIPE_SDMA_FLOOR) with ragged lengths and
  with caller pointers at odd offsets: a segment whose host and device ends
  sit at different offsets modulo 16 goes by SDMA instead (copy_phase_ok),
  one at the same offset moves its head / tail bytewise and the rest as
  vectors (copy_kernel.hip).  Rebuilt shards equal the originals.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

M = 1 << 20


def _random(ctx, shape, seed):
    a = ctx.host_array(int(np.prod(shape))).reshape(shape)
    rng = np.random.default_rng(seed)
    flat = a.reshape(-1)
    step = 256 * M
    for o in range(0, flat.size, step):
        n = min(step, flat.size - o)
        flat[o:o + n] = np.frombuffer(rng.bytes(n), np.uint8)
    return a


def _put_and_check(ctx, n, S, seed, short=None, digests=True, defer=False):
    """n x 4+2 objects of shard size S from host_array memory, PUT with
    digests (or without: the group form); `short` maps object -> length of
    its last data chunk.  Returns the copy-statistics delta (defer=True:
    (delta, a function that checks the objects and frees the buffers))."""
    k, m = 4, 2
    short = short or {}
    data = _random(ctx, (n, k, S), seed)
    par = ctx.host_array(n * m * S).reshape(n, m, S)
    par[:] = 0xEE
    dlen = []
    for o in range(n):
        dlen += [S] * (k - 1) + [short.get(o, S)]
    objs = [(k, m, S)] * n
    dptr = [data[o, j].ctypes.data for o in range(n) for j in range(k)]
    pptr = [par[o, i].ctypes.data for o in range(n) for i in range(m)]
    dig = np.zeros(n * (k + m) * 32, np.uint8)
    before = ctx.pipe_stats()
    status = ctx.encode_batch_host(objs, dptr, pptr, data_len=dlen, digests=dig if digests else None)
    after = ctx.pipe_stats()
    assert (status == 0).all()

    def check(o):
        chunks = [data[o, j, :dlen[o * k + j]] for j in range(k)]
        # SHA-NI digests for the big batch (pinned to the scalar form and
        # FIPS 180-4 in tests/test_oracle.py); the oracle releases the GIL.
        want, want_dig, rc = oracle.compute_parity(chunks, m, S, sha_ni=n >= 100)
        assert rc == 0
        for i in range(m):
            assert np.array_equal(par[o, i], want[i]), (o, i)
        if digests:
            got = [dig[(o * (k + m) + t) * 32:(o * (k + m) + t + 1) * 32].tobytes() for t in range(k + m)]
            assert got == want_dig, o

    def check_all():
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(8) as ex:
            list(ex.map(check, range(n)))
        ctx.host_free(data)
        ctx.host_free(par)

    delta = {key: after[key] - before[key] for key in after}
    if defer:
        return delta, check_all
    check_all()
    return delta


@pytest.mark.parametrize("piece_mb", ["2", "4"])
def test_put_2d_piece_copies_forced_piece(ctx_with, piece_mb):
    """24 objects, 5 MiB + 4160-byte shards (two or three pieces per chunk,
    the last off the grid); object 7's last data chunk ends mid-piece
    (3 MiB + 11), object 13's is empty."""
    ctx = ctx_with(MXEC_PIPE_PIECE_MB=piece_mb)
    S = 5 * M + 4160
    d = _put_and_check(ctx, 24, S, 501 + int(piece_mb), short={7: 3 * M + 11, 13: 0})
    assert d["copies_2d"] > 0 and d["rows_2d"] >= 2 * d["copies_2d"], d


def test_put_2d_piece_copies_default_upload_bound(ctx):
    """The default piece choice at a batch whose upload outlasts one chunk's
    chain (200 x 4+2 x 5 MiB: ~4.2 GB up against a ~105 ms chain), so the
    wave takes 2 or 4 MiB pieces and 2D copies; two ragged objects."""
    S = 5 * M + 4160
    d = _put_and_check(ctx, 200, S, 777, short={0: S - 1, 99: 2 * M + 5, 150: 0})
    assert d["copies_2d"] > 0, d


@pytest.mark.parametrize("copy,floor", [("waves", ""), ("auto", "100000")])
@pytest.mark.parametrize("offset", [0, 3, 16 + 5])
def test_get_wave_copies_ragged_and_odd_offsets(ctx_with, copy, offset, floor):
    """Verified GET of 9 x 4+2 objects whose shards start `offset` bytes
    into page-locked memory and whose last data chunk is S - 3333 bytes, by
    waves (MXEC_PIPE_COPY=waves, and auto, where a verified GET that runs as
    one verification group copies by waves both ways):
    every rebuilt shard equals the original; aligned callers take the wave
    copies (wave_blocks counted), phase-mismatched ones fall back to SDMA."""
    ctx = ctx_with(MXEC_PIPE_COPY=copy, MXEC_PIPE_SDMA_FLOOR=floor)
    k, m, n = 4, 2, 9
    S = 2 * M + 4096 + 48
    rng = np.random.default_rng(900 + offset)
    slot = S + 64
    buf = ctx.host_array(n * (k + m) * slot + 64)
    buf[:] = np.frombuffer(rng.bytes(buf.size), np.uint8)
    shard = [[buf[offset + (o * (k + m) + i) * slot:][:S] for i in range(k + m)] for o in range(n)]
    dl = [S] * (k - 1) + [S - 3333]
    objs = [(k, m, S)] * n
    dig = np.zeros(n * (k + m) * 32, np.uint8)
    st = ctx.encode_batch_host(objs, [shard[o][j].ctypes.data for o in range(n) for j in range(k)],
                               [shard[o][k + i].ctypes.data for o in range(n) for i in range(m)],
                               data_len=dl * n, digests=dig)
    assert (st == 0).all()
    ref = [[shard[o][i][:dl[i] if i < k else S].copy() for i in range(k + m)] for o in range(n)]
    present = np.ones((n, k + m), np.uint8)
    for o in range(n):
        for i in rng.choice(k + m, 2, replace=False):
            present[o, i] = 0
            shard[o][i][:] = 0x5A
    before = ctx.pipe_stats()
    pr = present.reshape(-1).copy()
    rc, st = ctx.reconstruct_batch_host(objs, [shard[o][i].ctypes.data for o in range(n) for i in range(k + m)],
                                        pr, shard_len=(dl + [S] * m) * n, expected=dig)
    after = ctx.pipe_stats()
    assert rc == 0 and not st.any() and pr.all()
    for o in range(n):
        for i in range(k + m):
            L = dl[i] if i < k else S
            assert np.array_equal(shard[o][i][:L], ref[o][i]), (copy, offset, o, i)
    if offset % 16 == 0:
        assert after["wave_blocks"] > before["wave_blocks"], (before, after)
    if copy == "auto":  # a one-group verified GET: waves both ways, no bracket to judge
        assert after["sdma_checks"] == before["sdma_checks"], (before, after)
    ctx.host_free(buf)


@pytest.mark.parametrize("floor,waves", [("0", False), ("", False), ("100000", True)])
def test_auto_copy_engine_follows_the_sdma_watch(floor, waves):
    """MXEC_PIPE_COPY=auto: an RS-only PUT's group uploads are timed (floor
    0: not watched; the default floor: timed, the rate recorded; an
    unreachable floor: the call's brackets are judged slow, and the device's
    next call, issued right after it -- well inside the 2 s hold -- copies
    by waves); parity against the oracle either way.  No assertion on the
    box's own SDMA rate."""
    from conftest import open_ctx

    # a context of its own: a cached one may still hold an earlier call's
    # verdict (waves for 2 s after a slow bracket)
    ctx = open_ctx(2, 0, MXEC_PIPE_COPY="auto", MXEC_PIPE_SDMA_FLOOR=floor)
    S = 3 * M + 4096 + 48
    try:
        s0 = ctx.pipe_stats()
        _, check1 = _put_and_check(ctx, 8, S, 1300 + len(floor), short={3: S - 3333}, digests=False, defer=True)
        s1 = ctx.pipe_stats()
        _, check2 = _put_and_check(ctx, 8, S, 1400 + len(floor), digests=False, defer=True)
        s2 = ctx.pipe_stats()
        check1()
        check2()
    finally:
        ctx.close()
    assert (s1["sdma_checks"] > s0["sdma_checks"]) == (floor != "0"), (s0, s1)
    assert (s1["sdma_slow"] > s0["sdma_slow"]) == waves, (s0, s1)
    assert (s2["wave_blocks"] > s1["wave_blocks"]) == waves, (s1, s2)
    if floor == "":
        assert s1["sdma_last_mbps"] > 0, s1  # a bracket was timed and its rate recorded


@pytest.mark.parametrize("floor", ["", "100000"])
def test_get_download_watch(floor):
    """MXEC_PIPE_COPY=auto times an RS-only GET's downloads (a bracket per
    rebuilt group, opened after the d2h stream's wait for the rebuild) and
    judges them against twice MXEC_PIPE_SDMA_FLOOR, two slow brackets in a
    row making a verdict: with the default floor the brackets are timed;
    with a floor no SDMA reaches they are judged slow (each call here has
    one judged bracket, so the second GET gives the verdict) and the
    device's downloads go by waves for the next 1 s (the third GET).  A
    lone verified GET speculates: its downloads go by SDMA unless a hold is
    on, the wave judged once after the fact from how long its downloads ran
    past the last verdict (pipeline.cpp spec_judge), its uploads by waves.
    16 x 4+2 objects of
    4 MiB + 4 KiB shards, two data shards erased in each: every rebuilt shard
    equals the original every time."""
    from conftest import open_ctx

    ctx = open_ctx(2, 0, MXEC_PIPE_COPY="auto", MXEC_PIPE_SDMA_FLOOR=floor)
    k, m, n = 4, 2, 16
    S = 4 * M + 4096
    try:
        buf = _random(ctx, (n, k + m, S), 4242 + len(floor))
        objs = [(k, m, S)] * n
        dig = np.zeros(n * (k + m) * 32, np.uint8)
        st = ctx.encode_batch_host(objs, [buf[o, j].ctypes.data for o in range(n) for j in range(k)],
                                   [buf[o, k + i].ctypes.data for o in range(n) for i in range(m)], digests=dig)
        assert (st == 0).all()
        s0 = ctx.pipe_stats()
        assert s0["sdma_down_checks"] == 0, s0  # the PUT's downloads are not bracketed
        ref = buf.copy()
        deltas = []
        for call in range(4):  # RS-only x 3, verified
            present = np.ones((n, k + m), np.uint8)
            present[:, [1, 3]] = 0
            buf[:, [1, 3]] = 0x77
            before = ctx.pipe_stats()
            pr = present.reshape(-1).copy()
            rc, st = ctx.reconstruct_batch_host(objs, [buf[o, i].ctypes.data for o in range(n) for i in range(k + m)],
                                                pr, expected=dig if call == 3 else None)
            after = ctx.pipe_stats()
            assert rc == 0 and not st.any() and pr.all()
            assert np.array_equal(buf, ref), call
            deltas.append({key: after[key] - before[key] for key in after} | {"down_mbps": after["sdma_down_last_mbps"]})
        ctx.host_free(buf)
    finally:
        ctx.close()
    d1, d2, d3, d4 = deltas
    assert d1["sdma_down_checks"] > 0 and d1["down_mbps"] > 0, deltas
    assert d4["wave_blocks"] > 0 and d4["spec_pieces"] > 0, deltas  # one group: uploads by waves, speculating
    # judged once after the fact -- or not at all while a download hold is on
    assert d4["sdma_down_checks"] in (0, 1), deltas
    if floor:
        assert d1["sdma_down_slow"] + d2["sdma_down_slow"] > 0, deltas  # two slow brackets in a row
        assert d3["sdma_down_checks"] == 0 and d3["wave_blocks"] > 0, deltas  # within the 1 s download hold

"""GPU: concurrent host-batch calls on one device.

MaxIO serves PUTs (filesystem.rs:686-828) and GETs (chunk_reader.rs:87-226)
at once on a multi-thread tokio runtime (main.rs:81); the library admits up
to MXEC_PIPE_LANES host-batch calls per device at once (pipeline.cpp
PipeHub), their waves interleaving on the device's four pipeline streams.

* A PUT with digests and a verified GET from two threads, started together
  and repeated: every PUT object's parity and k + m digests equal
  oracle.compute_parity; every GET object's shards equal the originals
  (erasures and silently corrupted present shards alike), a failing object
  gets -10 with its present shards unwritten; the counters show that calls
  ran side by side.
* Four threads, each a stream of PUT-with-digests or verified-GET batches of
  mixed shapes (4+2 / 8+4 / 10+4, 64 KiB - 4 MiB shards, short last
  chunks), from page-locked and pageable memory, every result checked.
* The same pair with MXEC_PIPE_LANES=1 (one call at a time) and with
  MXEC_GET_SPECULATE=0 (a failing object's buffers then stay untouched
  entirely).
"""
from __future__ import annotations

import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

M = 1 << 20
TOO_FEW = -10


def _fill(a, rng):
    flat = a.reshape(-1)
    step = 64 * M
    for o in range(0, flat.size, step):
        n = min(step, flat.size - o)
        flat[o:o + n] = np.frombuffer(rng.bytes(n), np.uint8)


class Put:
    """n objects of (k, m, S) from one buffer; check() against the oracle."""

    def __init__(self, ctx, shapes, rng, pinned=True):
        self.ctx, self.shapes = ctx, shapes
        self.pinned = pinned
        self.data, self.par, self.dlen = [], [], []
        for (k, m, S) in shapes:
            d = self._buf(k * S).reshape(k, S)
            _fill(d, rng)
            p = self._buf(m * S).reshape(m, S)
            p[:] = 0xEE
            self.data.append(d)
            self.par.append(p)
            last = int(rng.integers(0, S + 1)) if rng.random() < 0.3 else S
            self.dlen += [S] * (k - 1) + [last]
        self.dig = np.zeros(sum(k + m for k, m, _ in shapes) * 32, np.uint8)

    def _buf(self, n):
        return self.ctx.host_array(n) if self.pinned else np.empty(n, np.uint8)

    def run(self):
        st = self.ctx.encode_batch_host(self.shapes, [d[j].ctypes.data for d in self.data for j in range(d.shape[0])],
                                        [p[i].ctypes.data for p in self.par for i in range(p.shape[0])],
                                        data_len=self.dlen, digests=self.dig)
        assert (st == 0).all()

    def check(self):
        j0 = g0 = 0
        for o, (k, m, S) in enumerate(self.shapes):
            chunks = [self.data[o][j, :self.dlen[j0 + j]] for j in range(k)]
            want, want_dig, rc = oracle.compute_parity(chunks, m, S, sha_ni=True)
            assert rc == 0
            for i in range(m):
                assert np.array_equal(self.par[o][i], want[i]), (o, i)
            got = [self.dig[(g0 + t) * 32:(g0 + t + 1) * 32].tobytes() for t in range(k + m)]
            assert got == want_dig, o
            j0 += k
            g0 += k + m

    def free(self):
        if self.pinned:
            for a in self.data + self.par:
                self.ctx.host_free(a.reshape(-1))


class Get:
    """n encoded objects with two erasures each, except `corrupt` objects:
    one erasure and a silently corrupted present shard; `failing` objects get
    three bad present shards on top (more than m)."""

    def __init__(self, ctx, shapes, rng, corrupt=(), failing=(), pinned=True):
        self.ctx, self.shapes = ctx, shapes
        self.failing = set(failing)
        put = Put(ctx, shapes, rng, pinned)
        put.dlen = [S for (k, m, S) in shapes for _ in range(k)]
        put.run()
        self.put = put
        self.ptrs, self.lens, self.orig = [], [], []
        self.rows = [[put.data[o][j] for j in range(k)] + [put.par[o][i] for i in range(m)]
                     for o, (k, m, S) in enumerate(shapes)]
        self.flips = []  # (object, shard, byte, xor): re-applied before every run
        pres = []
        for o, (k, m, S) in enumerate(shapes):
            rows = self.rows[o]
            self.orig.append([r.copy() for r in rows])
            p = np.ones(k + m, np.uint8)
            for i in rng.choice(k + m, 1 if o in corrupt else 2, replace=False):  # room for the corruption
                p[i] = 0
            live = [int(i) for i in np.flatnonzero(p)]
            if o in corrupt:
                self.flips.append((o, live[o % len(live)], S // 3, 0x08))
            if o in self.failing:
                self.flips += [(o, i, 7, 0xFF) for i in live[:3]]
            self.ptrs += [r.ctypes.data for r in rows]
            self.lens += [S] * (k + m)
            pres.append(p)
        self.present0 = np.concatenate(pres)
        self._damage()
        self.before = {o: [r.copy() for r in self.rows[o]] for o in self.failing}

    def _damage(self):
        """Erased shards scribbled, corruptions applied (a previous run
        rebuilt the corrupted shards of the objects that passed)."""
        g = 0
        for o, (k, m, S) in enumerate(self.shapes):
            for i in range(k + m):
                if not self.present0[g + i]:
                    self.rows[o][i][:] = 0x5A
            g += k + m
        for o, i, b, x in self.flips:
            self.rows[o][i][b] = self.orig[o][i][b] ^ x

    def run(self):
        self._damage()
        self.present = self.present0.copy()
        self.rc, self.status = self.ctx.reconstruct_batch_host(self.shapes, self.ptrs, self.present,
                                                               shard_len=self.lens, expected=self.put.dig)

    def check(self, speculate=True):
        assert self.rc == (TOO_FEW if self.failing else 0), self.rc
        g = 0
        for o, (k, m, S) in enumerate(self.shapes):
            if o in self.failing:
                assert self.status[o] == TOO_FEW, o
                for i in range(k + m):
                    if self.present0[g + i] or not speculate:  # present shards are never written
                        assert np.array_equal(self.rows[o][i], self.before[o][i]), (o, i)
            else:
                assert self.status[o] == 0, (o, self.status[o])
                assert self.present[g:g + k + m].all(), o
                for i in range(k + m):
                    assert np.array_equal(self.rows[o][i], self.orig[o][i]), (o, i)
            g += k + m

    def free(self):
        self.put.free()


def _pair(ctx, rounds, speculate=True, seed=0):
    rng = np.random.default_rng(7000 + seed)
    shapes = [(4, 2, 4 * M + 48)] * 24
    put = Put(ctx, shapes, rng)
    get = Get(ctx, shapes, rng, corrupt=(1, 11, 22), failing=(5, 17))
    s0 = ctx.pipe_stats()
    for _ in range(rounds):
        go = threading.Barrier(2)

        def one(job):
            go.wait()
            job.run()

        with ThreadPoolExecutor(2) as ex:
            list(ex.map(one, (put, get)))
        put.check()
        get.check(speculate)
    s1 = ctx.pipe_stats()
    put.free()
    get.free()
    return {k: s1[k] - s0[k] for k in s1}


def test_put_and_verified_get_side_by_side(ctx_with):
    d = _pair(ctx_with(), 3)
    assert d["calls"] >= 6, d
    assert d["calls_shared"] >= 1, d  # started together, so they overlapped
    assert d["spec_pieces"] > 0 and d["spec_redos"] >= 3 * 5, d  # corrupt + failing objects redone


def test_pair_with_one_lane(ctx_with):
    """MXEC_PIPE_LANES=1: the second call waits for the first (no sharing)."""
    d = _pair(ctx_with(MXEC_PIPE_LANES="1"), 2, seed=1)
    assert d["calls"] >= 4 and d["calls_shared"] == 0, d


def test_pair_without_speculation(ctx_with):
    """MXEC_GET_SPECULATE=0: the rebuild waits for the verdict, and a failing
    object's buffers -- missing shards included -- are not written."""
    d = _pair(ctx_with(MXEC_GET_SPECULATE="0"), 2, speculate=False, seed=2)
    assert d["spec_pieces"] == 0 and d["spec_redos"] == 0, d


def test_four_threads_mixed_shapes_stream(ctx_with):
    """Four threads, three rounds each of PUT-with-digests or verified-GET
    batches of mixed shapes, pinned and pageable, all on one device."""
    ctx = ctx_with()
    kinds = [(4, 2), (8, 4), (10, 4)]
    sizes = [64 << 10, M + 4096, 4 * M, 300 << 10]

    def worker(t):
        rng = np.random.default_rng(8100 + t)
        for r in range(3):
            shapes = [(*kinds[int(rng.integers(0, 3))], sizes[int(rng.integers(0, 4))])
                      for _ in range(int(rng.integers(4, 14)))]
            pinned = (t + r) % 3 != 0
            if t % 2 == 0:
                job = Put(ctx, shapes, rng, pinned)
                job.run()
                job.check()
            else:
                job = Get(ctx, shapes, rng, corrupt=(0, 2), failing=(1,) if r == 1 else (), pinned=pinned)
                job.run()
                job.check()
            job.free()
        return True

    s0 = ctx.pipe_stats()
    with ThreadPoolExecutor(4) as ex:
        assert all(ex.map(worker, range(4)))
    s1 = ctx.pipe_stats()
    assert s1["calls"] - s0["calls"] >= 18, (s0, s1)

"""GPU: the coefficient-table arena's recycle path (runtime.cpp coef_offset,
ops.hpp with_stable_coef).

Every RS launch reads its matrix from a per-device table arena of two
halves; when the current half is full, the next generation takes the other
half after waiting only for the events that fence the launches which read
it (no device-wide wait, and not under the arena's lock); new tables go up
by hipMemcpyAsync on a per-device table stream that the launches wait for
on the GPU.  A test-only arena of a few KiB
(mxec_open_test coef_arena_bytes) makes that happen every few
batches:

* four and sixteen host threads, each on its own stream, rebuild batches whose seeded
  erasure patterns are all different (one decode table each) while the
  others do the same: every object bit-exact, the arena recycled many times;
* the same sequence from one thread, results equal to the oracle's
  reconstruct;
* one batch whose tables alone exceed both halves fails with the arena
  error instead of reading foreign tables.

Reference: chunk_reader.rs:211 -> reed-solomon-erasure's reconstruct, whose
decode matrices sit in an LRU cache per ReedSolomon (the crate's
`data_decode_matrix_cache`).
"""
from __future__ import annotations

import itertools
import threading

import numpy as np
import pytest

import maxio_amd
import oracle

pytestmark = pytest.mark.gpu

K, M, S = 8, 4, 65536


def _torch():
    import torch

    return torch


def _patterns(seed):
    pats = [p for e in (2, 3, 4) for p in itertools.combinations(range(K + M), e)]
    rng = np.random.default_rng(seed)
    rng.shuffle(pats)
    return pats


def _encoded(torch, n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    t = torch.empty((n, K + M, S), dtype=torch.uint8, device="cuda")
    t[:, :K].random_(0, 256, generator=g)
    return t


@pytest.mark.parametrize("n_thr", [4, 16])
def test_recycles_under_threads(ctx_with, n_thr):
    """n_thr threads on their own streams: with 16, a storm of distinct
    erasure patterns where new tables go up asynchronously on the table
    stream (launches wait for them on the GPU) and recycles wait for their
    fences outside the arena's lock."""
    ctx = ctx_with(streams=n_thr, MXEC_TEST_COEF_ARENA_KB=32)  # 8 192 dwords per half: ~10-20 decode tables
    torch = _torch()
    n_obj, rounds = 4, 30
    refs = []
    for th in range(n_thr):
        r = _encoded(torch, n_obj, 700 + th)
        torch.cuda.synchronize()
        ctx.encode_strided_device(K, M, S, n_obj, r.data_ptr(), (K + M) * S, S, r.data_ptr() + K * S,
                                  (K + M) * S, S)
        torch.cuda.synchronize()
        refs.append(r)
    errors = []

    def worker(th):
        try:
            st = torch.cuda.Stream()
            t = torch.empty_like(refs[th])
            pats = _patterns(800 + th)
            for rnd in range(rounds):
                present = np.ones((n_obj, K + M), np.uint8)
                with torch.cuda.stream(st):
                    t.copy_(refs[th])
                    for o in range(n_obj):
                        p = pats[(rnd * n_obj + o) % len(pats)]
                        present[o, list(p)] = 0
                        t[o, list(p)] = 0xEE
                pr = present.reshape(-1).copy()
                rc, status = ctx.reconstruct_strided_device(K, M, S, n_obj, t.data_ptr(), (K + M) * S, S, pr,
                                                            stream=st.cuda_stream)
                st.synchronize()
                if rc != 0 or status.any() or not pr.all():
                    errors.append((th, rnd, rc, maxio_amd.ec.N.lib().mxec_last_error()))
                    return
                if not torch.equal(t, refs[th]):
                    errors.append((th, rnd, "bytes differ"))
                    return
        except Exception as e:  # surfaced below
            errors.append((th, repr(e)))

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(n_thr)]
    for x in ths:
        x.start()
    for x in ths:
        x.join()
    assert not errors, errors[:4]
    stats = ctx.coef_stats()
    assert stats["recycles"] >= 5, stats


def test_recycles_one_thread_against_oracle(ctx_with):
    ctx = ctx_with(MXEC_TEST_COEF_ARENA_KB=16)
    torch = _torch()
    n_obj = 3
    ref = _encoded(torch, n_obj, 900)
    torch.cuda.synchronize()
    ctx.encode_strided_device(K, M, S, n_obj, ref.data_ptr(), (K + M) * S, S, ref.data_ptr() + K * S,
                              (K + M) * S, S)
    torch.cuda.synchronize()
    h = ref.cpu().numpy()
    pats = _patterns(901)
    before = ctx.coef_stats()["recycles"]
    t = torch.empty_like(ref)
    for rnd in range(12):
        t.copy_(ref)
        present = np.ones((n_obj, K + M), np.uint8)
        for o in range(n_obj):
            p = list(pats[rnd * n_obj + o])
            present[o, p] = 0
            t[o, p] = 0x11
        pr = present.reshape(-1).copy()
        torch.cuda.synchronize()
        rc, status = ctx.reconstruct_strided_device(K, M, S, n_obj, t.data_ptr(), (K + M) * S, S, pr)
        torch.cuda.synchronize()
        assert rc == 0 and not status.any() and pr.all()
        got = t.cpu().numpy()
        for o in range(n_obj):
            shards = [h[o, i] if present[o, i] else None for i in range(K + M)]
            bufs, _, orc = oracle.reconstruct(shards, K, M, S)
            assert orc == 0
            for i in range(K + M):
                assert np.array_equal(got[o, i], bufs[i]), (rnd, o, i)
    assert ctx.coef_stats()["recycles"] > before


def test_batch_larger_than_the_arena_fails_cleanly(ctx_with):
    ctx = ctx_with(MXEC_TEST_COEF_ARENA_KB=4)  # 1 024 dwords per half: four 4-erasure tables, 12 needed
    torch = _torch()
    n_obj = 12
    t = _encoded(torch, n_obj, 950)
    present = np.ones((n_obj, K + M), np.uint8)
    for o, p in enumerate(itertools.islice(itertools.combinations(range(K + M), 4), n_obj)):
        present[o, list(p)] = 0
    torch.cuda.synchronize()
    rc, _ = ctx.reconstruct_strided_device(K, M, S, n_obj, t.data_ptr(), (K + M) * S, S,
                                           present.reshape(-1).copy())
    torch.cuda.synchronize()
    assert rc != 0
    assert "table arena" in maxio_amd.ec.N.lib().mxec_last_error().decode()

"""GPU: the in-process multi-device paths of one mxec_ctx, run on a one-GPU
box by opening device 0 as two logical devices (mxec_open_test logical_devices=2, each
with its own slots, streams, coefficient arena, combiner and pipeline):

* mxec_encode_batch_host deals objects to per-device workers (o mod D,
  pipeline.cpp) — odd object counts, mixed (k, m, S), short last chunks and a
  failing object, bit-exact against the oracle, errors aggregated;
* host-API calls round-robin over the devices (ops.hpp DevScope / pick_device)
  from many threads at once;
* the device-pointer entry points address a device by index.

Reference: the path is per object (filesystem.rs:1084-1145,
chunk_reader.rs:157-226); MaxIO is one process, so one context spans the
node's GPUs."""
from __future__ import annotations

import hashlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import maxio_amd
import oracle
from test_pipeline_gpu import _check, _objects

pytestmark = pytest.mark.gpu


@pytest.fixture()
def ctx2(monkeypatch):
    c = maxio_amd.Context(device_mask=1, streams_per_device=3, test={"logical_devices": 2})
    assert c.device_ids() == [0, 0]
    yield c
    c.close()


@pytest.mark.parametrize("n_obj", [1, 7, 12])
def test_encode_batch_host_two_devices_odd_counts(ctx2, n_obj):
    rng = np.random.default_rng(500 + n_obj)
    shapes = [(4, 2, 65536), (8, 4, 1 << 20), (10, 4, 131072), (3, 5, 4096)]
    specs = []
    for o in range(n_obj):
        k, m, s = shapes[o % len(shapes)]
        specs.append((k, m, s, int(rng.integers(1, s)) if o % 3 == 1 else None))
    objs, data, dlen, parity, chunks_of = _objects(rng, specs)
    dig = np.zeros(sum(k + m for k, m, _ in objs) * 32, np.uint8)
    st = ctx2.encode_batch_host(objs, data, parity, data_len=dlen, digests=dig)
    assert list(st) == [0] * n_obj
    _check(objs, chunks_of, dig)


def test_encode_batch_host_two_devices_failing_object(ctx2):
    """One object breaks the reference's k+m > 255 guard (filesystem.rs:1095);
    the rest — on both devices — are still encoded, the call returns that
    object's error and the status array marks only it."""
    rng = np.random.default_rng(77)
    specs = [(4, 2, 8192, None), (6, 3, 16384, 1000), (8, 4, 4096, None), (5, 2, 8192, 17), (2, 2, 4096, None)]
    objs, data, dlen, parity, chunks_of = _objects(rng, specs)
    # object 2 claims 250 parity shards: 8 + 250 > 255
    bad = 2
    objs[bad] = (8, 250, 4096)
    parity_bad = [np.zeros(4096, np.uint8) for _ in range(250)]
    p0 = sum(m for (_, m, _) in objs[:bad])
    parity = parity[:p0] + [p.ctypes.data for p in parity_bad] + parity[p0 + 4:]
    rc, st = ctx2.encode_batch_host(objs, data, parity, data_len=dlen, return_rc=True)
    assert rc == -20, (rc, maxio_amd.lib().mxec_last_error())
    assert "too many shards" in maxio_amd.lib().mxec_last_error().decode()
    assert [int(x) for x in st] == [0, 0, -20, 0, 0]
    good = [i for i in range(len(objs)) if i != bad]
    _check([objs[i] for i in good], [chunks_of[i] for i in good], None)


def test_host_api_round_robin_two_devices(ctx2):
    """Concurrent host-pointer calls from 12 threads land on both logical
    devices; every result matches the oracle / hashlib."""
    k, m, S = 8, 4, 70_001

    def job(t):
        rng = np.random.default_rng(9000 + t)
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        data[-1] = data[-1][: S - 1 - t]
        par, dig = ctx2.encode(data, m, S)
        want, want_dig, rc = oracle.compute_parity(data, m, S)
        if rc != 0 or dig != want_dig or not all(np.array_equal(par[i], want[i]) for i in range(m)):
            return False
        shards = [d.tobytes() for d in data] + [p.tobytes() for p in par]
        lens = [len(x) for x in shards]
        inp = list(shards)
        lost = rng.choice(k + m, 3, replace=False)
        for i in lost[:2]:
            inp[i] = None
        inp[lost[2]] = bytes(lens[lost[2]])  # silent corruption, caught by the digest
        out, present = ctx2.reconstruct(inp, k, m, S, shard_len=lens, expected=dig)
        if not present.all() or any(out[i].tobytes() != shards[i] for i in range(k + m)):
            return False
        return ctx2.sha256(shards[:3]) == [hashlib.sha256(x).digest() for x in shards[:3]]

    with ThreadPoolExecutor(12) as pool:
        assert all(pool.map(job, range(36)))
    # both devices did verification work through their own combiners
    assert ctx2.combiner_stats(0)["messages"] > 0
    assert ctx2.combiner_stats(1)["messages"] > 0


def test_device_entry_points_by_index(ctx2):
    import torch

    k, m, S, n = 4, 2, 65536, 5
    g = torch.Generator(device="cuda").manual_seed(3)
    data = torch.randint(0, 256, (n, k, S), dtype=torch.uint8, device="cuda", generator=g)
    outs = []
    for dev in (0, 1):
        par = torch.zeros((n, m, S), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        ctx2.encode_strided_device(k, m, S, n, data.data_ptr(), k * S, S, par.data_ptr(), m * S, S, dev=dev)
        torch.cuda.synchronize()
        outs.append(par.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    h = data.cpu().numpy()
    for o in range(n):
        want = oracle.encode(list(h[o]), m, S)
        assert all(np.array_equal(outs[0][o][i], want[i]) for i in range(m))
    with pytest.raises(maxio_amd.RSError):
        ctx2.encode_strided_device(k, m, S, n, data.data_ptr(), k * S, S, data.data_ptr(), m * S, S, dev=2)


def test_numa_deal_on_pretend_nodes(ctx2):
    """on a context whose devices sit on two NUMA nodes,
    the host batch calls deal each object to a device on the node of its
    pages, balanced by bytes (deal.hpp deal_objects_numa; the rule itself is
    unit-tested with a fake node map in tests/c_manifest/deal_check.cpp).
    mxec_open_test's two logical copies of the card pretend to sit on nodes
    0 and 1; the objects' pages come from mxec_host_alloc_device(dev = o % 2)
    (on that node where the host has it).  A PUT with digests and a verified
    GET (two erasures, one corrupted present shard) over 12 x 4+2 x 2 MiB:
    every parity chunk, digest and rebuilt shard exact, both devices used."""
    k, m, n, S = 4, 2, 12, (2 << 20) + 48
    rng = np.random.default_rng(606)
    rows = [ctx2.host_array((k + m) * S, dev=o % 2).reshape(k + m, S) for o in range(n)]
    for r in rows:
        r[:k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
    objs = [(k, m, S)] * n
    dig = np.zeros(n * (k + m) * 32, np.uint8)
    c0 = [ctx2.pipe_stats(d) for d in range(2)]
    st = ctx2.encode_batch_host(objs, [r[j].ctypes.data for r in rows for j in range(k)],
                                [r[k + i].ctypes.data for r in rows for i in range(m)], digests=dig)
    assert (st == 0).all()
    for o, r in enumerate(rows):
        want, want_dig, rc = oracle.compute_parity([r[j] for j in range(k)], m, S)
        assert rc == 0 and all(np.array_equal(r[k + i], want[i]) for i in range(m)), o
        assert [dig[(o * (k + m) + t) * 32:][:32].tobytes() for t in range(k + m)] == want_dig, o
    ref = [r.copy() for r in rows]
    present = np.ones((n, k + m), np.uint8)
    for o, r in enumerate(rows):
        lost = rng.choice(k + m, 1 if o == 3 else 2, replace=False)
        present[o, lost] = 0
        r[lost] = 0x5A
    r3 = rows[3]
    r3[int(np.flatnonzero(present[3])[0]), 1234] ^= 0x40  # silently corrupt: caught, rebuilt
    pr = present.reshape(-1).copy()
    rc, st = ctx2.reconstruct_batch_host(objs, [r[i].ctypes.data for r in rows for i in range(k + m)], pr,
                                         expected=dig)
    assert rc == 0 and not st.any() and pr.all()
    for o in range(n):
        assert np.array_equal(rows[o], ref[o]), o
    c1 = [ctx2.pipe_stats(d) for d in range(2)]
    assert all(c1[d]["calls"] - c0[d]["calls"] == 2 for d in range(2)), (c0, c1)
    for r in rows:
        ctx2.host_free(r.reshape(-1))

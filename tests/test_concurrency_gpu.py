"""GPU: many host threads drive every kind of request through ONE context at
once — PUT, healthy / degraded / ranged GET, encrypted PUT + GET, multipart
completion, raw SHA-256 batches and device-batch reconstructs — as MaxIO's
tokio workers would; every result is checked.  Exercises slot locking, the
SHA-256 combiner and the per-device caches under contention."""
from __future__ import annotations

import hashlib
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import maxio_amd
import oracle

pytestmark = pytest.mark.gpu


def _job(ctx, base, t):
    rng = np.random.default_rng(500 + t)
    kind = t % 6
    d = os.path.join(base, f"t{t}")
    if kind == 0:  # PUT + degraded GET
        n = int(rng.integers(1, 3 << 20))
        body = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        ctx.put_object_chunked(d + ".ec", 1 << 18, 2, body)
        k = (n + (1 << 18) - 1) >> 18
        os.unlink(os.path.join(d + ".ec", f"{int(rng.integers(0, k)):06}"))
        return ctx.get_object_chunked(d + ".ec") == body
    if kind == 1:  # PUT + ranged reads through the streaming reader
        n = int(rng.integers(100_000, 2 << 20))
        body = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        ctx.put_object_chunked(d + ".ec", 65536, 3, body)
        off, ln = int(rng.integers(0, n)), int(rng.integers(1, 300_000))
        with ctx.open_reader(d + ".ec", off, ln, batch_bytes=1 << 18) as r:
            got = b""
            while True:
                piece = r.read(77_777)
                if not piece:
                    break
                got += piece
        return got == body[off:off + ln]
    if kind == 2:  # encrypted PUT + ranged GET
        key, pre = rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), b"CONC"
        idp = oracle.object_aad_prefix("b", f"k{t}", None)
        n = int(rng.integers(1, 400_000))
        body = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        ctx.put_object_chunked_encrypted(d + ".ec", 100_000, 2, key, pre, idp, body)
        off = int(rng.integers(0, n))
        return ctx.get_object_chunked_encrypted(d + ".ec", key, idp, off, 5000) == body[off:off + 5000]
    if kind == 3:  # SHA-256 batches of odd lengths
        bufs = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in rng.integers(0, 90_000, 9)]
        return ctx.sha256(bufs) == [hashlib.sha256(b).digest() for b in bufs]
    if kind == 4:  # host encode / reconstruct with verification
        k, m, s = 6, 3, 70_001
        data = [rng.integers(0, 256, s, dtype=np.uint8) for _ in range(k)]
        parity, dig = ctx.encode(data, m, s)
        shards = [x.tobytes() for x in data] + [p.tobytes() for p in parity]
        inp = list(shards)
        inp[1] = None
        inp[7] = bytes(s)  # corrupt: caught by the digest
        out, present = ctx.reconstruct(inp, k, m, s, expected=dig)
        return present.all() and out[1].tobytes() == shards[1] and out[7].tobytes() == shards[7]
    # multipart completion
    sizes = [int(x) for x in rng.integers(1, 200_000, 3)]
    parts = []
    whole = b""
    for i, sz in enumerate(sizes):
        b = rng.integers(0, 256, sz, dtype=np.uint8).tobytes()
        p = f"{d}.part{i}"
        with open(p, "wb") as f:
            f.write(b)
        parts.append({"path": p, "size": sz, "etag": hashlib.md5(b).hexdigest(), "part_number": i + 1})
        whole += b
    etag = ctx.complete_multipart_chunked(d + ".mp", 65536, 2, parts)
    raw = b"".join(bytes.fromhex(p["etag"]) for p in parts)
    return etag == f'"{hashlib.md5(raw).hexdigest()}-3"' and ctx.get_object_chunked(d + ".mp") == whole


def test_mixed_requests_many_threads(tmp_path):
    ctx = maxio_amd.Context(streams_per_device=16)
    try:
        with ThreadPoolExecutor(24) as pool:
            results = list(pool.map(lambda t: _job(ctx, str(tmp_path), t), range(96)))
        assert all(results), [i for i, r in enumerate(results) if not r]
    finally:
        ctx.close()


def test_combined_verify_waits_for_callers_stream_work():
    """The combined SHA-256 launch waits on the device for the work each
    caller queued on its own stream before handing over its shards
    (combiner.cpp: an event per caller, hipStreamWaitEvent): four threads
    each zero their objects, queue a copy that restores them on their own
    stream, and call the device verify + rebuild at once, without a host
    sync.  Hashing before the copies land would see zeros, turn every shard
    into an erasure and fail the call."""
    import torch

    k, m, S, n, W = 8, 4, 1 << 20, 96, 4
    ctx = maxio_amd.Context(streams_per_device=W)
    try:
        streams = [torch.cuda.Stream() for _ in range(W)]
        g = torch.Generator(device="cuda").manual_seed(91)
        objs, refs, digs = [], [], []
        for w in range(W):
            o = torch.randint(0, 256, (n, k + m, S), dtype=torch.uint8, device="cuda", generator=g)
            d = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            ctx.encode_strided_device(k, m, S, n, o.data_ptr(), (k + m) * S, S, o[:, k:].data_ptr(),
                                      (k + m) * S, S, digests_ptr=d.data_ptr())
            torch.cuda.synchronize()
            objs.append(o)
            refs.append(o.clone())
            digs.append(d)
        want = [hashlib.sha256(refs[0][0, i].cpu().numpy().tobytes()).digest() for i in range(k + m)]
        assert [bytes(x) for x in digs[0][0].cpu().numpy()] == want

        def one(w):
            st = streams[w]
            with torch.cuda.stream(st):
                objs[w].zero_()
                objs[w].copy_(refs[w])  # queued, not waited for
            present = np.ones(n * (k + m), np.uint8)
            present[0::k + m] = 0  # one data erasure per object
            rc, _ = ctx.reconstruct_strided_device(k, m, S, n, objs[w].data_ptr(), (k + m) * S, S, present,
                                                   expected_ptr=digs[w].data_ptr(), stream=st.cuda_stream)
            return rc, present

        with ThreadPoolExecutor(W) as pool:
            res = list(pool.map(one, range(W)))
        torch.cuda.synchronize()
        for w, (rc, present) in enumerate(res):
            assert rc == 0, (w, rc)
            assert present.all(), w
            assert torch.equal(objs[w], refs[w]), w
    finally:
        ctx.close()


def test_speculative_rebuild_matches_verify_then_rebuild():
    """mxec_reconstruct_strided_device with expected digests rebuilds
    speculatively beside the hash (capi.cpp); the result must equal verify-
    then-rebuild (chunk_reader.rs:176-211) in every case: no corruption;
    a corrupt data shard among the first k present (the speculative decode
    used it and must be redone); a corrupt parity shard past the first k
    (not used); two corruptions that leave exactly k; corruptions that
    leave fewer than k (the object fails with -10, its present shards
    untouched).  A rebuildable object must come back equal to the object
    as encoded (the reconstruction from any k valid shards is unique), with
    every shard present."""
    import torch

    k, m, S, n = 8, 4, 40_000 + 48, 64
    total = k + m
    rng = np.random.default_rng(95)
    ctx = maxio_amd.Context(streams_per_device=2)
    try:
        g = torch.Generator(device="cuda").manual_seed(96)
        obj = torch.randint(0, 256, (n, total, S), dtype=torch.uint8, device="cuda", generator=g)
        dig = torch.zeros((n, total, 32), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        ctx.encode_strided_device(k, m, S, n, obj.data_ptr(), total * S, S, obj[:, k:].data_ptr(), total * S, S,
                                  digests_ptr=dig.data_ptr())
        torch.cuda.synchronize()
        ref = obj.clone()
        present = np.ones(n * total, np.uint8)
        corrupt = {}
        for o in range(n):
            erased = [int(x) for x in rng.choice(k, 2, replace=False)]
            for i in erased:
                present[o * total + i] = 0
                obj[o, i].fill_(0x5A)
            case = o % 5
            live = [i for i in range(total) if i not in erased]
            if case == 1:
                bad = [live[0]]                       # used by the first-k decode
            elif case == 2:
                bad = [total - 1]                     # a parity shard past the first k
            elif case == 3:
                bad = [live[1], live[5]]              # leaves exactly k
            elif case == 4:
                bad = [live[0], live[2], live[4]]     # leaves k - 1: fails
            else:
                bad = []
            for i in bad:
                obj[o, i, 7] ^= 0x80
            corrupt[o] = (erased, bad)
        before = obj.clone()
        torch.cuda.synchronize()
        rc, status = ctx.reconstruct_strided_device(k, m, S, n, obj.data_ptr(), total * S, S, present,
                                                    expected_ptr=dig.data_ptr())
        torch.cuda.synchronize()
        assert rc == -10  # the first failing object's status
        got = obj.cpu()
        for o in range(n):
            erased, bad = corrupt[o]
            row = present[o * total:(o + 1) * total]
            if len(bad) >= 3:
                assert status[o] == -10, o
                # present shards untouched; the flags show the mismatches
                for i in range(total):
                    if i not in erased and i not in bad:
                        assert row[i] == 1 and torch.equal(got[o, i], before[o, i].cpu()), (o, i)
                    if i in bad:
                        assert row[i] == 0, (o, i)
                continue
            assert status[o] == 0, o
            assert row.all(), o
            assert torch.equal(got[o], ref[o].cpu()), (o, erased, bad)
    finally:
        ctx.close()

"""GPU: the completion-handle forms (mxec_*_async, async.cpp) — what a tokio
caller would await through AsyncFd instead of parking a blocking-pool thread
for a ~30 ms SHA-256 chain (chunk_reader.rs:244-249, main.rs:81).  Results
equal the blocking calls' (oracle / hashlib), errors arrive on the ticket,
the eventfd signals completion, and closing a context drains its queue."""
from __future__ import annotations

import hashlib
import os
import select

import numpy as np
import pytest

import maxio_amd
import oracle

pytestmark = pytest.mark.gpu


def _wait_fds(tickets, timeout=120):
    pending = {t.fd: t for t in tickets}
    while pending:
        r, _, _ = select.select(list(pending), [], [], timeout)
        assert r, "no ticket completed within the timeout"
        for fd in r:
            assert pending.pop(fd).done()


def test_async_mixed_calls_match_oracle(tmp_path):
    rng = np.random.default_rng(81)
    with maxio_amd.Context(streams_per_device=6) as c:
        jobs = []
        for t in range(24):
            kind = t % 4
            if kind == 0:
                k, m, S = 8, 4, 70_000 + t
                data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
                jobs.append(("enc", (data, m, S), c.encode_async(data, m, S)))
            elif kind == 1:
                k, m, S = 4, 2, 50_000 + t
                data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
                par = oracle.encode(data, m, S)
                shards = [d.tobytes() for d in data] + [p.tobytes() for p in par]
                dig = [hashlib.sha256(x).digest() for x in shards]
                inp = list(shards)
                inp[1] = None
                inp[4] = bytes(S)  # corrupt: caught by the digest check
                jobs.append(("rec", shards, c.reconstruct_async(inp, k, m, S, expected=dig)))
            elif kind == 2:
                bufs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 90_000, 5)]
                jobs.append(("sha", bufs, c.sha256_async(bufs)))
            else:
                body = rng.integers(0, 256, 3 * 16384 + t, dtype=np.uint8)
                ec = str(tmp_path / f"o{t}.ec")
                jobs.append(("put", (ec, body), c.put_object_chunked_async(ec, 16384, 2, body)))
        _wait_fds([j[2] for j in jobs])
        for kind, ref, tk in jobs:
            res = tk.wait()
            if kind == "enc":
                data, m, S = ref
                parity, digests = res
                want, want_dig, rc = oracle.compute_parity(data, m, S)
                assert rc == 0 and digests == want_dig
                assert all(np.array_equal(parity[i], want[i]) for i in range(m))
            elif kind == "rec":
                out, present = res
                assert present.all()
                assert [o.tobytes() for o in out] == ref
            elif kind == "sha":
                assert res == [hashlib.sha256(b).digest() for b in ref]
            else:
                ec, body = ref
                g = c.get_object_chunked_async(ec, body.size)
                # deleted while that GET may be reading: either it read the file
                # or it finds it missing and rebuilds it from parity
                os.remove(os.path.join(ec, "000001"))
                assert g.wait() == body.tobytes()
                assert c.get_object_chunked_async(ec, body.size).wait() == body.tobytes()  # rebuilt


def test_async_error_arrives_on_the_ticket(ctx):
    k, m, S = 4, 2, 4096
    t = ctx.reconstruct_async([None, None, None, b"x" * S, b"y" * S, b"z" * S], k, m, S)
    with pytest.raises(maxio_amd.RSError) as ei:
        t.wait()
    assert ei.value.code == -10 and "too many missing" in str(ei.value)
    # rejected before queueing: no ticket, the error right away
    with pytest.raises(maxio_amd.RSError) as ei:
        ctx.encode_async([b"a"], 0, 16)
    assert ei.value.code == -5


def test_close_drains_queued_calls():
    rng = np.random.default_rng(82)
    c = maxio_amd.Context(streams_per_device=2)
    bufs = [rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes() for _ in range(6)]
    tickets = [c.sha256_async(bufs) for _ in range(8)]
    c.close()  # waits for every queued call
    want = [hashlib.sha256(b).digest() for b in bufs]
    for t in tickets:
        assert t.done()
        assert t.wait() == want


def test_async_storage_errors_and_ticket_lifecycle(ctx, tmp_path):
    """File-layer errors come back on the ticket with the blocking call's
    code and message (GET of a missing object: the manifest read fails,
    −40; PUT into a path whose parent is a file: −40), the eventfd is not
    readable before completion and is after, and a ticket freed without a
    wait (close) still waits for its call first."""
    g = ctx.get_object_chunked_async(str(tmp_path / "missing.ec"), 1024)
    with pytest.raises(maxio_amd.RSError) as ei:
        g.wait()
    assert ei.value.code == -40
    blocker = tmp_path / "file"
    blocker.write_bytes(b"x")
    p = ctx.put_object_chunked_async(str(blocker / "obj.ec"), 4096, 2, np.zeros(10000, np.uint8))
    with pytest.raises(maxio_amd.RSError) as ei:
        p.wait()
    assert ei.value.code == -40
    rng = np.random.default_rng(83)
    bufs = [rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes() for _ in range(4)]
    t = ctx.sha256_async(bufs)
    r, _, _ = select.select([t.fd], [], [], 0)
    if not t.done():  # a 1 MiB chain takes ~29 ms: normally still running here
        assert not r, "eventfd readable before the call completed"
    r, _, _ = select.select([t.fd], [], [], 120)
    assert r and t.done()
    assert t.wait() == [hashlib.sha256(b).digest() for b in bufs]
    t2 = ctx.sha256_async(bufs)
    t2.close()  # frees only after the call finished; no crash, no leak of the fd


def test_reconstruct_strided_device_async_matches_blocking(ctx):
    """mxec_reconstruct_strided_device_async (the device verify + rebuild a
    GPU-direct GET stream calls, chunk_reader.rs:176-211) gives the blocking
    call's present flags, statuses and rebuilt bytes; its argument errors
    answer before queueing."""
    import torch

    k, m, S, n = 8, 4, 65536, 96
    total = k + m
    g = torch.Generator(device="cuda").manual_seed(97)
    obj = torch.randint(0, 256, (n, total, S), dtype=torch.uint8, device="cuda", generator=g)
    dig = torch.zeros((n, total, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.encode_strided_device(k, m, S, n, obj.data_ptr(), total * S, S, obj[:, k:].data_ptr(), total * S, S,
                              digests_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    ref = obj.clone()
    rng = np.random.default_rng(98)
    present = np.ones(n * total, np.uint8)
    for o in range(n):
        for i in rng.choice(total, 3, replace=False):
            present[o * total + i] = 0
            obj[o, i].zero_()
        obj[o, int(rng.integers(0, total)), 9] ^= 1  # may hit an erased shard: harmless
    torch.cuda.synchronize()
    t = ctx.reconstruct_strided_device_async(k, m, S, n, obj.data_ptr(), total * S, S, present,
                                             expected_ptr=dig.data_ptr())
    status = t.wait()
    torch.cuda.synchronize()
    assert (status == 0).all() and present.all()
    assert torch.equal(obj, ref)
    with pytest.raises(maxio_amd.RSError) as ei:
        ctx.reconstruct_strided_device_async(0, 2, S, 1, obj.data_ptr(), total * S, S, np.ones(2, np.uint8))
    assert ei.value.code == -3  # TooFewDataShards from the crate's guard, no ticket

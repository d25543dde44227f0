"""GPU parity: the HIP kernels (through the C ABI) against the oracle and the
golden fixtures.  Integer/byte work, so every comparison is bit-exact."""
from __future__ import annotations

import hashlib
import itertools
import os

import numpy as np
import pytest

import maxio_amd
import oracle
from helpers import data_for, sha_vector_inputs

pytestmark = pytest.mark.gpu


# ---- encode ------------------------------------------------------------------


def test_one_encode_crate_vector(ctx, golden):
    kat = golden("rs_kat.json")["one_encode"]
    rs = maxio_amd.ReedSolomon(kat["k"], kat["m"], ctx)
    shards = [bytearray(d) for d in kat["data"]] + [bytearray(2) for _ in range(kat["m"])]
    rs.encode(shards)
    assert [list(s) for s in shards[kat["k"]:]] == kat["parity"]
    assert rs.verify(shards)
    shards[8][0] = (shards[8][0] + 1) % 256
    assert not rs.verify(shards)


def test_encode_golden_vectors(ctx, golden):
    for case in golden("encode_vectors.json")["cases"]:
        data = data_for(case["seed"], case["k"], case["shard_size"], case["last_len"])
        parity, digests = ctx.encode(data, case["m"], case["shard_size"])
        assert [hashlib.sha256(p.tobytes()).hexdigest() for p in parity] == case["parity_sha256"], case
        assert [d.hex() for d in digests] == case["chunk_sha256"], case


@pytest.mark.parametrize("k,m,size,last", [
    (1, 2, 4096, None), (4, 2, 65536, 40000), (8, 4, 1 << 20, None), (10, 4, 100_003, 77),
    (3, 9, 12288, 1), (16, 11, 8192 + 16, None), (64, 4, 8192, 5000), (200, 55, 256, 255),
    (253, 2, 64, None), (2, 1, 1, None), (7, 3, 17, 3),
])
def test_encode_matches_oracle(ctx, k, m, size, last):
    data = data_for(k * 1000 + m, k, size, last)
    parity, digests = ctx.encode(data, m, size)
    want, want_dig, rc = oracle.compute_parity(data, m, size)
    assert rc == 0
    for i in range(m):
        assert np.array_equal(parity[i], want[i]), (k, m, i)
    assert digests == want_dig


def test_encode_errors(ctx):
    d = [np.zeros(8, np.uint8)] * 250
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.encode(d, 6, 8)
    assert e.value.name == "TooManyShards255"
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.encode([b"ab"], 0, 2)
    assert e.value.name == "TooFewParityShards"
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.encode([b"ab"], 2, 0)
    assert e.value.name == "EmptyShard"


# ---- reconstruct ---------------------------------------------------------------


def test_reconstruct_golden_all_patterns(ctx, golden):
    for case in golden("reconstruct_vectors.json")["cases"]:
        k, m, s = case["k"], case["m"], case["shard_size"]
        data = data_for(case["seed"], k, s)
        shards = data + oracle.encode(data, m, s)
        for pat in case["erasure_patterns"]:
            inp = [None if i in pat else shards[i] for i in range(k + m)]
            out, present = ctx.reconstruct(inp, k, m, s)
            assert present.all()
            for i in range(k + m):
                assert np.array_equal(out[i], shards[i]), (k, m, pat, i)
            out, present = ctx.reconstruct(inp, k, m, s, data_only=True)
            for i in range(k):
                assert np.array_equal(out[i], shards[i])
            assert all(present[i] == 0 for i in pat if i >= k)


@pytest.mark.parametrize("k,m,size", [(8, 4, 1 << 20), (10, 4, 65536 + 48), (32, 8, 4096), (5, 5, 333)])
def test_reconstruct_matches_oracle(ctx, k, m, size):
    rng = np.random.default_rng(k * 31 + m)
    data = data_for(k + m, k, size)
    shards = data + oracle.encode(data, m, size)
    for _ in range(3):
        e = int(rng.integers(1, m + 1))
        pat = sorted(rng.choice(k + m, e, replace=False).tolist())
        inp = [None if i in pat else shards[i] for i in range(k + m)]
        want, _, rc = oracle.reconstruct(inp, k, m, size)
        assert rc == 0
        out, present = ctx.reconstruct(inp, k, m, size)
        for i in range(k + m):
            assert np.array_equal(out[i], want[i]), (pat, i)


def test_reconstruct_verify_turns_corruption_into_erasure(ctx):
    k, m, s = 4, 2, 100
    body = bytes([0xEF]) * 350
    data = [np.frombuffer(body[o:o + s], np.uint8) for o in range(0, 350, s)]
    parity, dig = ctx.encode(data, m, s)
    sizes = [100, 100, 100, 50, 100, 100]
    shards = [d.tobytes() for d in data] + [p.tobytes() for p in parity]
    bad = list(shards)
    bad[1] = bytes(100)
    out, present = ctx.reconstruct(bad, k, m, s, shard_len=sizes, expected=dig)
    assert present.all()
    assert out[1].tobytes() == shards[1] and out[3].tobytes() == shards[3]
    want, rc, _ = oracle.try_reconstruct_data_chunk(bad, k, m, s, dig, sizes, 1)
    assert rc == 0 and want == out[1].tobytes()


def test_reconstruct_too_few(ctx):
    data = data_for(5, 4, 64)
    shards = data + oracle.encode(data, 2, 64)
    for pat in itertools.combinations(range(6), 3):
        inp = [None if i in pat else shards[i] for i in range(6)]
        with pytest.raises(maxio_amd.RSError) as e:
            ctx.reconstruct(inp, 4, 2, 64)
        assert e.value.name == "TooFewShardsPresent"


def test_reedsolomon_mirror(ctx):
    rs = maxio_amd.ReedSolomon(10, 4, ctx)
    data = data_for(99, 10, 1000)
    shards = [bytearray(d.tobytes()) for d in data] + [bytearray(1000) for _ in range(4)]
    rs.encode(shards)
    orig = [bytes(s) for s in shards]
    for i in (0, 5, 11, 13):
        shards[i] = None
    rs.reconstruct(shards)
    assert [bytes(s) for s in shards] == orig
    with pytest.raises(maxio_amd.RSError):
        maxio_amd.ReedSolomon(0, 1, ctx)


# ---- SHA-256 ---------------------------------------------------------------------


def test_sha256_golden(ctx, golden):
    sv = golden("sha256_vectors.json")
    lens = [c["len"] for c in sv["cases"]]
    got = ctx.sha256(sha_vector_inputs(sv["seed"], lens))
    assert [g.hex() for g in got] == [c["sha256"] for c in sv["cases"]]
    assert ctx.sha256([b""])[0].hex() == sv["empty"]


def test_sha256_all_tail_lengths(ctx):
    rng = np.random.default_rng(11)
    bufs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in range(0, 300)]
    got = ctx.sha256(bufs)
    assert got == [hashlib.sha256(b).digest() for b in bufs]


# ---- device-resident batches ----------------------------------------------------


def _torch():
    """torch is only the device-memory allocator here; on a GPU box it must
    see the device (a skip would hide the device-resident tests)."""
    import torch

    assert torch.cuda.is_available(), "HIP device visible to libmaxio_ec but not to torch"
    return torch


def test_encode_strided_device_with_digests(ctx):
    torch = _torch()
    k, m, s, n = 4, 2, 65536 + 4096, 7
    rng = np.random.default_rng(5)
    host = rng.integers(0, 256, (n, k, s), dtype=np.uint8)
    data = torch.from_numpy(host).cuda()
    parity = torch.zeros((n, m, s), dtype=torch.uint8, device="cuda")
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.encode_strided_device(k, m, s, n, data.data_ptr(), k * s, s, parity.data_ptr(), m * s, s,
                              digests_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    par = parity.cpu().numpy()
    dg = dig.cpu().numpy()
    for o in range(n):
        want, want_dig, _ = oracle.compute_parity(list(host[o]), m, s)
        for i in range(m):
            assert np.array_equal(par[o, i], want[i])
        assert [dg[o, i].tobytes() for i in range(k + m)] == want_dig


def test_encode_batch_device_mixed(ctx):
    torch = _torch()
    specs = [(4, 2, 65536), (8, 4, 4096), (10, 4, 1 << 20), (4, 2, 65536), (3, 1, 1000)]
    rng = np.random.default_rng(8)
    data_t, par_t, dptr, pptr, dlen, host = [], [], [], [], [], []
    for (k, m, s) in specs:
        h = rng.integers(0, 256, (k, s), dtype=np.uint8)
        host.append(h)
        d = torch.from_numpy(h).cuda()
        p = torch.zeros((m, s), dtype=torch.uint8, device="cuda")
        data_t.append(d)
        par_t.append(p)
        dptr += [d[j].data_ptr() for j in range(k)]
        pptr += [p[i].data_ptr() for i in range(m)]
        dlen += [s] * (k - 1) + [s - 13]
    total = sum(k + m for (k, m, _) in specs)
    dig = torch.zeros((total, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.encode_batch_device(specs, dptr, pptr, data_len=dlen, digests_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    row = 0
    dg = dig.cpu().numpy()
    for (k, m, s), h, p in zip(specs, host, par_t):
        chunks = [h[j] for j in range(k - 1)] + [h[k - 1][: s - 13]]
        want, want_dig, _ = oracle.compute_parity(chunks, m, s)
        got = p.cpu().numpy()
        for i in range(m):
            assert np.array_equal(got[i], want[i])
        assert [dg[row + i].tobytes() for i in range(k + m)] == want_dig
        row += k + m


def test_reconstruct_strided_device_verify(ctx):
    torch = _torch()
    k, m, s, n = 8, 4, 1 << 16, 16
    rng = np.random.default_rng(21)
    host = rng.integers(0, 256, (n, k + m, s), dtype=np.uint8)
    for o in range(n):
        host[o, k:] = np.stack(oracle.encode(list(host[o, :k]), m, s))
    digests = np.stack([[np.frombuffer(hashlib.sha256(host[o, i].tobytes()).digest(), np.uint8)
                         for i in range(k + m)] for o in range(n)])
    dev = torch.from_numpy(host.copy()).cuda()
    dig = torch.from_numpy(digests).cuda()
    present = np.ones(n * (k + m), np.uint8)
    for o in range(n):
        lost = rng.choice(k + m, 2, replace=False)
        for i in lost:
            present[o * (k + m) + i] = 0
            dev[o, i].zero_()
    # silent corruption on object 3, shard 5 (if still present): verify must catch it
    if present[3 * (k + m) + 5]:
        dev[3, 5, 100] ^= 0xFF
    # object 9: three shards lost + one corrupt -> too few
    for i in range(4):
        present[9 * (k + m) + i] = 0
    dev[9, 4, 7] ^= 1
    torch.cuda.synchronize()
    rc, status = ctx.reconstruct_strided_device(k, m, s, n, dev.data_ptr(), (k + m) * s, s,
                                                present, expected_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    assert rc == -10 and status[9] == -10
    out = dev.cpu().numpy()
    for o in range(n):
        if o == 9:
            continue
        assert status[o] == 0
        assert np.array_equal(out[o], host[o]), o


# ---- full-size properties (BASELINE config sizes) ---------------------------------


def test_config2_full_size_roundtrip(ctx):
    """k=4 m=2, 10 MiB chunks: encode -> erase 2 -> reconstruct == original;
    one object also checked byte-for-byte against the oracle."""
    torch = _torch()
    k, m, s, n = 4, 2, 10 << 20, 6
    g = torch.Generator(device="cuda").manual_seed(2)
    obj = torch.randint(0, 256, (n, k + m, s), dtype=torch.uint8, device="cuda", generator=g)
    ctx.encode_strided_device(k, m, s, n, obj.data_ptr(), (k + m) * s, s,
                              obj[:, k:].data_ptr(), (k + m) * s, s)
    torch.cuda.synchronize()
    ref = obj.clone()
    h0 = ref[0].cpu().numpy()
    want = oracle.encode(list(h0[:k]), m, s)
    for i in range(m):
        assert np.array_equal(h0[k + i], want[i])
    present = np.ones(n * (k + m), np.uint8)
    rng = np.random.default_rng(3)
    for o in range(n):
        for i in rng.choice(k + m, 2, replace=False):
            present[o * (k + m) + i] = 0
            obj[o, i].fill_(0x5A)
    rc, status = ctx.reconstruct_strided_device(k, m, s, n, obj.data_ptr(), (k + m) * s, s, present)
    torch.cuda.synchronize()
    assert rc == 0 and present.all()
    assert torch.equal(obj, ref)


def test_config3_full_size_verify_reconstruct(ctx):
    """k=8 m=4, 1 MiB chunks, 2 data erasures + SHA verify of the rest."""
    torch = _torch()
    k, m, s, n = 8, 4, 1 << 20, 64
    g = torch.Generator(device="cuda").manual_seed(4)
    obj = torch.randint(0, 256, (n, k + m, s), dtype=torch.uint8, device="cuda", generator=g)
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
    ctx.encode_strided_device(k, m, s, n, obj.data_ptr(), (k + m) * s, s,
                              obj[:, k:].data_ptr(), (k + m) * s, s, digests_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    ref = obj.clone()
    # digests against hashlib for a sample
    for (o, i) in [(0, 0), (5, 11), (63, 7)]:
        assert dig[o, i].cpu().numpy().tobytes() == hashlib.sha256(ref[o, i].cpu().numpy().tobytes()).digest()
    present = np.ones(n * (k + m), np.uint8)
    rng = np.random.default_rng(6)
    for o in range(n):
        for i in rng.choice(k, 2, replace=False):
            present[o * (k + m) + i] = 0
            obj[o, i].zero_()
    rc, status = ctx.reconstruct_strided_device(k, m, s, n, obj.data_ptr(), (k + m) * s, s, present,
                                                expected_ptr=dig.data_ptr())
    torch.cuda.synchronize()
    assert rc == 0
    assert torch.equal(obj, ref)


def test_sha256_many_messages_throughput_form(ctx):
    """> 32768 messages selects the one-wave-per-64-messages kernel; fewer the
    split producer/consumer kernel.  Both must match hashlib."""
    rng = np.random.default_rng(12)
    lens = rng.integers(0, 300, 40000)
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8).tobytes()
    bufs, o = [], 0
    for n in lens:
        bufs.append(blob[o:o + int(n)])
        o += int(n)
    got = ctx.sha256(bufs)
    assert got == [hashlib.sha256(b).digest() for b in bufs]


@pytest.mark.parametrize("last", [300000, 16384, 1, (1 << 20) - 16])
def test_short_last_chunk_device_encode_and_rebuild(ctx, last):
    """Realistic objects: the last data chunk is short (object size not a
    multiple of chunk_size).  Tiles past its end read it as zero without a
    load; the tile it ends in goes to the edge kernel; a rebuilt short chunk
    is written to its length only (chunk_reader.rs:216-222)."""
    torch = _torch()
    k, m, s, n = 8, 4, 1 << 20, 5
    rng = np.random.default_rng(last)
    host = rng.integers(0, 256, (n, k + m, s), dtype=np.uint8)
    host[:, k - 1, last:] = 0
    dl = [s] * (k - 1) + [last]
    for o in range(n):
        chunks = [host[o, j] for j in range(k - 1)] + [host[o, k - 1, :last]]
        want, _, _ = oracle.compute_parity(chunks, m, s)
        host[o, k:] = np.stack(want)
    dev = torch.from_numpy(host).cuda()
    dev[:, k:].fill_(0x33)  # parity must be fully rewritten
    torch.cuda.synchronize()
    ctx.encode_strided_device(k, m, s, n, dev.data_ptr(), (k + m) * s, s, dev[:, k:].data_ptr(),
                              (k + m) * s, s, data_len=dl)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), host)
    # lose the short chunk and one more; rebuild must write exactly `last` bytes
    present = np.ones(n * (k + m), np.uint8)
    for o in range(n):
        present[o * (k + m) + k - 1] = 0
        present[o * (k + m) + 2] = 0
    dev[:, k - 1].fill_(0x77)
    dev[:, 2].fill_(0x77)
    torch.cuda.synchronize()
    rc, _ = ctx.reconstruct_strided_device(k, m, s, n, dev.data_ptr(), (k + m) * s, s, present,
                                           shard_len=dl + [s] * m)
    torch.cuda.synchronize()
    assert rc == 0
    got = dev.cpu().numpy()
    assert np.array_equal(got[:, k - 1, :last], host[:, k - 1, :last])
    assert (got[:, k - 1, last:] == 0x77).all()  # untouched past the chunk's end
    assert np.array_equal(got[:, 2], host[:, 2])


# MXEC_SHA_FORM pins the SHA-256 kernel (read at mxec_open, so each form has
# its own context).  Shipping forms: lagpair (the auto form up to 64
# messages per CU: the lag quad, four lanes per message behind a producer
# wave, the a-side two rounds behind the e-side, two messages per quad),
# split (producer/consumer waves) and one (one wave per 64 messages).  Lab
# builds (make lab, MXEC_LIB) add lag (one message per quad) and quad (the
# same-round quad form).
SHA_FORMS = ["lagpair", "split", "one", "lag", "quad"]
LAB_SHA_FORMS = {"lag", "quad"}


def _form_ctx(ctx_with, form):
    from conftest import lab_build

    if form in LAB_SHA_FORMS and not lab_build():
        pytest.skip(f"SHA form {form!r} exists in lab builds only")
    return ctx_with(MXEC_SHA_FORM=form)


@pytest.mark.parametrize("form", SHA_FORMS)
def test_sha256_every_kernel_form(ctx_with, form):
    """Every SHA-256 kernel form on mixed lengths (multi-block, tails 0..63,
    unaligned starts)."""
    ctx = _form_ctx(ctx_with, form)
    rng = np.random.default_rng(13)
    lens = list(rng.integers(0, 5000, 300)) + [0, 55, 56, 64, 4096, 100_003]
    blob = rng.integers(0, 256, int(sum(lens)) + 64, dtype=np.uint8).tobytes()
    bufs, o = [], 0
    for i, n in enumerate(lens):
        o += i % 3  # some unaligned starts
        bufs.append(blob[o:o + int(n)])
        o += int(n)
    got = ctx.sha256(bufs)
    assert got == [hashlib.sha256(b).digest() for b in bufs]


@pytest.mark.parametrize("form", SHA_FORMS)
@pytest.mark.parametrize("shift", [0, 16, 3])
def test_sha256_device_messages_ring_edges(ctx_with, form, shift):
    """Device-resident messages straight into the kernel (no staging copy),
    16-byte aligned (shift 0/16: the split form's prefetch-ring path) or not
    (shift 3: its byte-load path): lone messages of 0..9 full blocks (every
    ring phase and tail count), a wave whose lanes end at different blocks,
    empty messages (their lanes borrow a donor lane's address) and a batch
    past one workgroup."""
    ctx = _form_ctx(ctx_with, form)
    torch = _torch()
    rng = np.random.default_rng(21 + shift)
    cases = [[64 * b + t] for b in range(10) for t in (0, 37)]
    cases.append([int(x) for x in rng.integers(0, 64 * 23, 64)])
    cases.append([0, 0, 5 * 64, 0, 64 * 9 + 1])
    cases.append([int(x) for x in rng.integers(0, 3000, 150)])
    for lens in cases:
        stride = (max(lens) + 64 + 15) // 16 * 16
        host = rng.integers(0, 256, stride * len(lens) + 64, dtype=np.uint8)
        dev = torch.from_numpy(host).cuda()
        ptrs = [dev.data_ptr() + i * stride + shift for i in range(len(lens))]
        dig = torch.zeros(len(lens) * 32, dtype=torch.uint8, device="cuda")
        ctx.sha256_batch_device(ptrs, lens, dig.data_ptr())
        torch.cuda.synchronize()
        got = dig.cpu().numpy().reshape(-1, 32)
        for i, n in enumerate(lens):
            o = i * stride + shift
            assert bytes(got[i]) == hashlib.sha256(host[o:o + n].tobytes()).digest(), (lens, i)


def test_concurrent_reconstruct_workers(ctx):
    """Several host threads (tokio workers) reconstruct their own batches on
    their own streams through one context at once (bench config 3c): every
    batch comes back bit-exact, corruption caught per batch."""
    from concurrent.futures import ThreadPoolExecutor

    torch = _torch()
    k, m, s, n, workers = 8, 4, 1 << 16, 24, 4
    c = maxio_amd.Context(streams_per_device=workers)
    try:
        jobs = []
        for w in range(workers):
            g = torch.Generator(device="cuda").manual_seed(100 + w)
            obj = torch.randint(0, 256, (n, k + m, s), dtype=torch.uint8, device="cuda", generator=g)
            dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
            c.encode_strided_device(k, m, s, n, obj.data_ptr(), (k + m) * s, s,
                                    obj[:, k:].data_ptr(), (k + m) * s, s, digests_ptr=dig.data_ptr())
            torch.cuda.synchronize()
            jobs.append((obj, dig, obj.clone(), torch.cuda.Stream(), np.random.default_rng(w)))

        def run(job):
            obj, dig, ref, st, rng = job
            for _ in range(3):
                present = np.ones(n * (k + m), np.uint8)
                with torch.cuda.stream(st):
                    for o in range(n):
                        lost = rng.choice(k + m, 2, replace=False)
                        present[o * (k + m) + lost[0]] = 0
                        obj[o, lost[0]].zero_()
                        obj[o, lost[1], 17] ^= 0x80  # silent corruption: still flagged present
                st.synchronize()
                rc, status = c.reconstruct_strided_device(k, m, s, n, obj.data_ptr(), (k + m) * s, s,
                                                          present, expected_ptr=dig.data_ptr(),
                                                          stream=st.cuda_stream)
                st.synchronize()
                if rc != 0 or not present.all() or not torch.equal(obj, ref):
                    return False
            return True

        with ThreadPoolExecutor(workers) as pool:
            assert all(pool.map(run, jobs))
    finally:
        c.close()


def test_concurrent_small_sha_requests_are_combined(ctx):
    """Many threads hashing a few chunks each (GET verification of small
    objects) share launches through the device's combiner; every digest must
    still land with its own caller."""
    from concurrent.futures import ThreadPoolExecutor

    c = maxio_amd.Context(streams_per_device=12)
    try:
        def job(t):
            rng = np.random.default_rng(1000 + t)
            bufs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()
                    for n in np.random.default_rng(t).integers(0, 70000, 1 + t % 7)]
            for _ in range(4):
                if c.sha256(bufs) != [hashlib.sha256(b).digest() for b in bufs]:
                    return False
            return True

        with ThreadPoolExecutor(12) as pool:
            assert all(pool.map(job, range(48)))
        stats = c.combiner_stats()
        assert stats["messages"] >= 4 * sum(1 + t % 7 for t in range(48))
        assert stats["batches"] <= 4 * 48  # some requests rode in another's launch
    finally:
        c.close()


def test_combiner_after_a_lone_streak_still_combines():
    """A context that first serves lone requests one after another (past the
    combiner's lone streak, where a leader stops waiting for company) still
    gets every digest right, and concurrent callers arriving afterwards
    still share launches (combiner.cpp kLoneStreak)."""
    from concurrent.futures import ThreadPoolExecutor

    c = maxio_amd.Context(streams_per_device=12)
    try:
        rng = np.random.default_rng(77)
        lone = [rng.integers(0, 256, 5000 + 97 * i, dtype=np.uint8).tobytes() for i in range(12)]
        for b in lone:
            assert c.sha256([b]) == [hashlib.sha256(b).digest()]
        before = c.combiner_stats()
        assert before["batches"] == len(lone)

        def job(t):
            bufs = [np.random.default_rng(500 + t).integers(0, 256, 3000 + t, dtype=np.uint8).tobytes()
                    for _ in range(1 + t % 3)]
            for _ in range(4):
                if c.sha256(bufs) != [hashlib.sha256(b).digest() for b in bufs]:
                    return False
            return True

        with ThreadPoolExecutor(12) as pool:
            assert all(pool.map(job, range(48)))
        after = c.combiner_stats()
        assert after["batches"] - before["batches"] < 4 * 48  # some requests rode in another's launch
    finally:
        c.close()


def test_pinned_host_buffers_take_the_direct_dma_path(ctx, tmp_path):
    """Buffers from mxec_host_alloc (Context.host_array) move by DMA straight
    to and from the device: same results as pageable buffers for hashing,
    encode, reconstruct and a file-layer GET into a pinned output."""
    import ctypes

    rng = np.random.default_rng(31)
    k, m, S = 4, 2, 100_003
    pinned = [ctx.host_array(S) for _ in range(k + m)]
    for j in range(k):
        pinned[j][:] = rng.integers(0, 256, S, dtype=np.uint8)
    pageable = [p.copy() for p in pinned[:k]]
    assert ctx.sha256(pinned[:k]) == [hashlib.sha256(p.tobytes()).digest() for p in pageable]
    par_pg, dig_pg = ctx.encode(pageable, m, S)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    ins = (ctypes.c_void_p * k)(*[p.ctypes.data for p in pinned[:k]])
    outs = (ctypes.c_void_p * m)(*[p.ctypes.data for p in pinned[k:]])
    dig = np.zeros((k + m, 32), np.uint8)
    assert maxio_amd.lib().mxec_encode(ctx.handle, k, m, S, ins, None, outs, dig.ctypes.data_as(u8p)) == 0
    for i in range(m):
        assert np.array_equal(pinned[k + i], par_pg[i])
    assert [bytes(d) for d in dig] == dig_pg
    # reconstruct two lost data shards in place, in pinned memory
    want = [p.copy() for p in pinned]
    pinned[1][:] = 0
    pinned[3][:] = 0
    present = np.array([0 if i in (1, 3) else 1 for i in range(k + m)], np.uint8)
    ptrs = (ctypes.c_void_p * (k + m))(*[f.ctypes.data for f in pinned])
    n = ctypes.c_int(0)
    assert maxio_amd.lib().mxec_reconstruct(ctx.handle, k, m, S, ptrs, None, None, present.ctypes.data_as(u8p), 0,
                                            ctypes.byref(n)) == 0
    for i in range(k + m):
        assert np.array_equal(pinned[i], want[i]), i
    # every shard present, nothing to rebuild: returns only after the uploads
    assert maxio_amd.lib().mxec_reconstruct(ctx.handle, k, m, S, ptrs, None, None, present.ctypes.data_as(u8p), 0,
                                            ctypes.byref(n)) == 0
    # file-layer GET into a pinned buffer
    body = rng.integers(0, 256, 5 * 4096 + 17, dtype=np.uint8)
    ec = str(tmp_path / "p.ec")
    ctx.put_object_chunked(ec, 4096, 2, body)
    os.remove(os.path.join(ec, "000002"))
    out = ctx.host_array(body.size)
    got = ctypes.c_uint64(0)
    assert maxio_amd.lib().mxec_get_object_chunked(ctx.handle, ec.encode(), 0, (1 << 64) - 1, out.ctypes.data,
                                                   body.size, ctypes.byref(got)) == 0
    assert got.value == body.size and np.array_equal(out, body)


def test_pinned_error_paths_wait_for_the_dma(ctx):
    """A call whose uploads read the caller's page-locked buffers directly
    returns only after those DMAs finished, on its error paths too: too few
    shards present (no digests given, a routine result) frees the buffers at
    once; the next call on the context still works and its results are
    exact."""
    import ctypes

    u8p = ctypes.POINTER(ctypes.c_uint8)
    k, m, S = 6, 3, 1 << 20
    rng = np.random.default_rng(41)
    for _ in range(4):
        bufs = [ctx.host_array(S) for _ in range(k + m)]
        for b in bufs:
            b[:] = rng.integers(0, 256, S, dtype=np.uint8)
        present = np.array([1] * (k - 1) + [0] * (m + 1), np.uint8)
        ptrs = (ctypes.c_void_p * (k + m))(*[b.ctypes.data for b in bufs])
        n = ctypes.c_int(0)
        rc = maxio_amd.lib().mxec_reconstruct(ctx.handle, k, m, S, ptrs, None, None,
                                              present.ctypes.data_as(u8p), 0, ctypes.byref(n))
        assert rc == -10 and n.value == k - 1
        assert b"too many missing" in maxio_amd.lib().mxec_last_error()
        del bufs, ptrs  # page-locked memory handed back right away
        import gc

        gc.collect()
    data = [rng.integers(0, 256, 4096, dtype=np.uint8) for _ in range(4)]
    par, _ = ctx.encode(data, 2, 4096)
    want = oracle.encode(data, 2, 4096)
    assert all(np.array_equal(par[i], want[i]) for i in range(2))


def test_sha256_mixed_pinned_and_pageable(ctx):
    """One batch with page-locked and pageable buffers (the staging path takes
    the whole call) and a range that starts inside a pinned allocation but
    runs past its end is never sent by direct DMA."""
    rng = np.random.default_rng(43)
    pinned = [ctx.host_array(n) for n in (5000, 64, 1 << 20)]
    for p in pinned:
        p[:] = rng.integers(0, 256, p.size, dtype=np.uint8)
    pageable = [rng.integers(0, 256, n, dtype=np.uint8) for n in (1, 99_999)]
    bufs = [pinned[0], pageable[0], pinned[1], pageable[1], pinned[2]]
    assert ctx.sha256(bufs) == [hashlib.sha256(b.tobytes()).digest() for b in bufs]
    # slices: inside one pinned allocation (direct) and the tail of one
    parts = [pinned[2][100:200_000], pinned[2][-7:], pinned[0][4999:]]
    assert ctx.sha256(parts) == [hashlib.sha256(b.tobytes()).digest() for b in parts]


def test_put_data_chunk_write_error_wins(ctx, tmp_path):
    """PUT whose data-chunk write fails (a directory squats on 000001): the
    I/O error is what the call reports — the reference writes the data chunks
    before compute_and_write_parity (filesystem.rs:729-750) — and the writer
    thread is joined (the context keeps working)."""
    ec = tmp_path / "w.ec"
    (ec / "000001").mkdir(parents=True)
    body = np.random.default_rng(44).integers(0, 256, 3 * 4096 + 5, dtype=np.uint8)
    with pytest.raises(maxio_amd.RSError) as ei:
        ctx.put_object_chunked(str(ec), 4096, 2, body)
    assert ei.value.code == -40 and "000001" in str(ei.value)
    assert not (ec / "manifest.json").exists()
    ok = tmp_path / "ok.ec"
    ctx.put_object_chunked(str(ok), 4096, 2, body)
    assert ctx.get_object_chunked(str(ok)) == body.tobytes()


def test_grid_tuner_decides_and_stays_exact():
    """The RS grid tuner (ops.cpp rs_grid_pick): launches 2-7 of a large
    uniform shape cycle through three grid sizes, the eighth keeps the fastest; every
    launch's parity is bit-exact (the grid never changes the bytes).  A fresh
    context so the shape's tuning starts here."""
    torch = _torch()
    import maxio_amd

    k, m, s, n = 4, 2, 1 << 20, 180  # 1.13 GB per launch (tuning starts at 1 GB)
    with maxio_amd.Context(device_mask=1, streams_per_device=1) as c:
        g = torch.Generator(device="cuda").manual_seed(9)
        obj = torch.randint(0, 256, (n, k + m, s), dtype=torch.uint8, device="cuda", generator=g)
        torch.cuda.synchronize()
        assert c.rs_grid(k, m, s) == 1024  # never launched: the default
        ref = None
        for it in range(10):
            obj[:, k:].zero_()
            torch.cuda.synchronize()
            c.encode_strided_device(k, m, s, n, obj.data_ptr(), (k + m) * s, s, obj[:, k:].data_ptr(), (k + m) * s, s)
            torch.cuda.synchronize()
            if ref is None:
                ref = obj[:, k:].clone()
                h = obj[0].cpu().numpy()
                want = oracle.encode(list(h[:k]), m, s)
                assert all(np.array_equal(h[k + i], want[i]) for i in range(m))
            else:
                assert torch.equal(obj[:, k:], ref), it
        assert c.rs_grid(k, m, s) in (1024, 512, 256)

"""Python host mirror of the reference's chunked-EC interface, over the C ABI.

Names follow the reference so the parity tests read like its own tests:

* ``ReedSolomon(k, m)`` mirrors ``reed_solomon_erasure::galois_8::ReedSolomon``
  (``new`` / ``encode`` / ``reconstruct`` / ``reconstruct_data`` / ``verify``)
  as called at filesystem.rs:1121-1124 and chunk_reader.rs:168,211; errors are
  ``RSError`` carrying the crate's variant name.
* ``Context.write_chunk`` / ``compute_and_write_parity`` /
  ``try_reconstruct_data_chunk`` / ``put_object_chunked`` /
  ``get_object_chunked`` mirror ``FilesystemStorage`` (filesystem.rs:686-1145)
  and ``VerifiedChunkReader`` (chunk_reader.rs:35-226).

Every byte of RS / SHA-256 work runs in the HIP kernels of libmaxio_ec.so;
this module only marshals buffers.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _native as N

ERROR_NAMES = {
    -1: "TooFewShards",
    -2: "TooManyShards",
    -3: "TooFewDataShards",
    -4: "TooManyDataShards",
    -5: "TooFewParityShards",
    -6: "TooManyParityShards",
    -7: "TooFewBufferShards",
    -8: "TooManyBufferShards",
    -9: "IncorrectShardSize",
    -10: "TooFewShardsPresent",
    -11: "EmptyShard",
    -12: "InvalidShardFlags",
    -13: "InvalidIndex",
    -14: "SingularMatrix",
    -20: "TooManyShards255",
    -21: "InvalidArgument",
    -30: "Device",
    -31: "OutOfMemory",
    -32: "NoDevice",
    -40: "Io",
    -41: "Integrity",
    -42: "Json",
}
DATA_ONLY = 0x1
# mxec_body_sums_batch flags (include/maxio_ec.h MXEC_SUM_*)
SUM_MD5, SUM_CRC32, SUM_CRC32C, SUM_SHA1, SUM_SHA256 = 0x01, 0x02, 0x04, 0x08, 0x10
FRAME_CHUNK_SIZE = 65536  # crypto.rs:46
_SUM_BY_ALGO = {"CRC32": SUM_CRC32, "CRC32C": SUM_CRC32C, "SHA1": SUM_SHA1, "SHA256": SUM_SHA256}


def _sums_dict(r: "N.BodySums", which: int) -> dict:
    d = {}
    if which & SUM_MD5:
        d["md5"] = bytes(r.md5)
    if which & SUM_CRC32:
        d["crc32"] = int(r.crc32)
    if which & SUM_CRC32C:
        d["crc32c"] = int(r.crc32c)
    if which & SUM_SHA1:
        d["sha1"] = bytes(r.sha1)
    if which & SUM_SHA256:
        d["sha256"] = bytes(r.sha256)
    return d


def put_result(sums: dict, algo: Optional[str]) -> dict:
    """PutResult's etag / checksum_value strings (filesystem.rs:775-777)."""
    import base64

    out = {"etag": '"%s"' % sums["md5"].hex()}
    if algo:
        raw = {"CRC32": lambda: sums["crc32"].to_bytes(4, "big"),
               "CRC32C": lambda: sums["crc32c"].to_bytes(4, "big"),
               "SHA1": lambda: sums["sha1"], "SHA256": lambda: sums["sha256"]}[algo]()
        out["checksum_value"] = base64.b64encode(raw).decode()
    return out


class RSError(Exception):
    def __init__(self, code: int, message: str = ""):
        self.code = code
        self.name = ERROR_NAMES.get(code, f"E{code}")
        super().__init__(f"{self.name} ({code}): {message}")


def _check(rc: int) -> None:
    if rc != 0:
        raise RSError(rc, N.lib().mxec_last_error().decode(errors="replace"))


def _u8(buf) -> np.ndarray:
    """A C-contiguous uint8 view (no copy for bytes/bytearray/np arrays)."""
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf.reshape(-1).view(np.uint8))
    return np.frombuffer(buf, dtype=np.uint8) if len(buf) else np.zeros(1, np.uint8)[:0]


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else _ptr.zero.ctypes.data


_ptr.zero = np.zeros(16, np.uint8)


def _pp(ptrs: Sequence[int]):
    return (ctypes.c_void_p * max(1, len(ptrs)))(*ptrs)


def _szp(vals: Sequence[int]):
    return (ctypes.c_size_t * max(1, len(vals)))(*vals)


def _u64p(vals: Sequence[int]):
    return (ctypes.c_uint64 * max(1, len(vals)))(*vals)


def rs_check(k: int, m: int) -> None:
    """ReedSolomon::new(k, m) argument checks (no GPU needed)."""
    _check(N.lib().mxec_rs_check(k, m))


def parity_matrix(k: int, m: int) -> np.ndarray:
    """The m x k parity rows of the crate's encoding matrix (host-side)."""
    out = np.zeros((m, k), np.uint8)
    _check(N.lib().mxec_rs_parity_matrix(k, m, out.ctypes.data_as(N.U8P)))
    return out


def device_count() -> int:
    return int(N.lib().mxec_device_count())


def version() -> str:
    """mxec_version(): '... (gfx950)', or '... (gfx950, lab build)' for `make lab`."""
    return N.lib().mxec_version().decode()


class Context:
    """An ``mxec_ctx``: every visible MI355X (or the ones in device_mask)."""

    def __init__(self, device_mask: int = 0, streams_per_device: int = 2, test: Optional[dict] = None):
        """``test`` (tests and bench rehearsals only) opens through
        mxec_open_test: ``logical_devices`` (open each GPU N times),
        ``rs_grid`` (cap every RS launch at N workgroups), ``coef_arena_kb``
        (KiB per half of the coefficient arena)."""
        self._lib = N.lib()
        self._host = {}  # mxec_host_alloc arrays: id(buffer) -> (pointer, finalizer)
        if test:
            unknown = set(test) - {"logical_devices", "rs_grid", "coef_arena_kb"}
            if unknown:
                raise ValueError(f"unknown test options {sorted(unknown)}")
            self._h = self._lib.mxec_open_test(
                device_mask, streams_per_device, int(test.get("logical_devices", 1)),
                int(test.get("rs_grid", 0)), int(test.get("coef_arena_kb", 0)) << 10)
        else:
            self._h = self._lib.mxec_open(device_mask, streams_per_device)
        if not self._h:
            raise RSError(-32, self._lib.mxec_last_error().decode())

    def close(self) -> None:
        if self._h:
            self._lib.mxec_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def combiner_stats(self, dev: int = 0) -> dict:
        """SHA-256 launches of device `dev`'s combiner and the messages they hashed."""
        b, m = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(self._lib.mxec_ctx_combiner_stats(self._h, dev, ctypes.byref(b), ctypes.byref(m)))
        return {"batches": b.value, "messages": m.value}

    def coef_stats(self, dev: int = 0) -> dict:
        """Coefficient-table arena of device `dev`: recycles of its halves,
        batches queued again after a recycle, recycles that waited for a
        fenced launch (mxec_ctx_coef_stats)."""
        r, q, w = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(self._lib.mxec_ctx_coef_stats(self._h, dev, ctypes.byref(r), ctypes.byref(q), ctypes.byref(w)))
        return {"recycles": r.value, "relaunches": q.value, "fence_waits": w.value}

    PIPE_STATS = ("copies_1d", "copies_2d", "rows_2d", "wave_blocks", "sdma_checks", "sdma_slow", "verify_waves",
                  "verify_groups", "sdma_last_mbps", "sdma_down_checks", "sdma_down_slow", "sdma_down_last_mbps",
                  "calls", "calls_shared", "spec_pieces", "spec_redos", "pace_waits")

    def pipe_stats(self, dev: int = 0) -> dict:
        """Host-batch pipeline counters of device `dev` since the context
        opened (mxec_ctx_pipe_stats): copies issued by engine, SDMA probes,
        verification groups."""
        v = (ctypes.c_uint64 * len(self.PIPE_STATS))()
        n = self._lib.mxec_ctx_pipe_stats(self._h, dev, v, len(self.PIPE_STATS))
        if n < 0:
            _check(n)
        return dict(zip(self.PIPE_STATS, list(v)[:n]))

    def rs_grid(self, k: int, m: int, shard_size: int, dev: int = 0) -> int:
        """Workgroups per CU large uniform RS launches of this shape run at on
        device `dev` (the grid tuner's pick; 0 while still tuning)."""
        rc = self._lib.mxec_ctx_rs_grid(self._h, dev, k, m, shard_size)
        if rc < 0:
            _check(rc)
        return rc

    def host_array(self, n: int, dev: Optional[int] = None) -> np.ndarray:
        """A uint8 array of n bytes in page-locked memory (mxec_host_alloc;
        with `dev`, mxec_host_alloc_device: on that context device's NUMA
        node): uploads from it and downloads into it skip the staging copy.
        Free it with host_free(); otherwise it is freed when the array is
        garbage collected -- but never from an interpreter-exit callback (the
        HIP runtime may be tearing down by then): memory still held at exit
        goes back with the process."""
        p = (self._lib.mxec_host_alloc(self._h, max(1, n)) if dev is None
             else self._lib.mxec_host_alloc_device(self._h, dev, max(1, n)))
        if not p:
            raise MemoryError("mxec_host_alloc failed")
        buf = (ctypes.c_uint8 * max(1, n)).from_address(p)
        a = np.frombuffer(buf, dtype=np.uint8, count=n)
        import weakref

        fin = weakref.finalize(buf, self._lib.mxec_host_free, None, p)
        fin.atexit = False
        self._host = {q: f for q, f in self._host.items() if f.alive}
        self._host[p] = fin
        return a

    def batch_alloc(self, k: int, m: int, shard_size: int, n_obj: int, dev: int = 0):
        """mxec_batch_alloc: HBM for a device-resident batch laid out
        [n_obj][k+m][shard_stride], placed by measurement.  Returns (device
        pointer, shard_stride, the candidates' probe times in ms).  Free with
        batch_free()."""
        stride = ctypes.c_uint64(0)
        ms = (ctypes.c_float * 4)()
        p = self._lib.mxec_batch_alloc(self._h, dev, k, m, shard_size, n_obj, ctypes.byref(stride), ms)
        if not p:
            raise RSError(-31, self._lib.mxec_last_error().decode(errors="replace"))
        return p, stride.value, [round(x, 4) for x in ms]

    def batch_free(self, p: int) -> None:
        _check(self._lib.mxec_batch_free(self._h, p))

    def host_free(self, a: np.ndarray) -> None:
        """Free a host_array now (the array must not be used afterwards)."""
        fin = self._host.pop(a.ctypes.data, None)
        if fin is None:
            raise ValueError("not a host_array of this context (or already freed)")
        fin()

    def device_ids(self) -> list[int]:
        n = self._lib.mxec_ctx_device_count(self._h)
        return [self._lib.mxec_ctx_device_id(self._h, i) for i in range(n)]

    # ---- host-pointer drop-ins --------------------------------------------
    def sha256(self, bufs: Sequence) -> list[bytes]:
        arrs = [_u8(b) for b in bufs]
        out = np.zeros((max(1, len(arrs)), 32), np.uint8)
        _check(self._lib.mxec_sha256_batch(
            self._h, _pp([_ptr(a) for a in arrs]), _szp([a.size for a in arrs]), len(arrs),
            out.ctypes.data_as(N.U8P)))
        return [bytes(out[i]) for i in range(len(arrs))]

    def encode(self, data: Sequence, m: int, shard_size: int, digests: bool = True):
        """compute_and_write_parity minus the files: returns (parity shards,
        k+m digests or None)."""
        arrs = [_u8(d) for d in data]
        k = len(arrs)
        parity = [np.zeros(shard_size, np.uint8) for _ in range(max(m, 0))]
        dig = np.zeros((max(1, k + m), 32), np.uint8)
        _check(self._lib.mxec_encode(
            self._h, k, m, shard_size, _pp([_ptr(a) for a in arrs]), _szp([a.size for a in arrs]),
            _pp([p.ctypes.data for p in parity]),
            dig.ctypes.data_as(N.U8P) if digests else None))
        return parity, ([bytes(dig[i]) for i in range(k + m)] if digests else None)

    def reconstruct(self, shards: Sequence[Optional[object]], k: int, m: int, shard_size: int,
                    shard_len: Optional[Sequence[int]] = None,
                    expected: Optional[Sequence[bytes]] = None, data_only: bool = False):
        """try_reconstruct_data_chunk minus the files.  Returns (shards as
        numpy arrays, present flags).  Missing shards are None."""
        total = k + m
        if shard_len is None:
            shard_len = [shard_size] * total
        bufs, present = [], np.zeros(total, np.uint8)
        for i in range(total):
            s = shards[i] if i < len(shards) else None
            if s is None:
                bufs.append(np.zeros(max(int(shard_len[i]), 1), np.uint8))
            else:
                a = np.array(_u8(s), dtype=np.uint8, copy=True)
                bufs.append(a if a.size else np.zeros(1, np.uint8))
                present[i] = 1
        exp = None
        if expected is not None:
            exp = np.frombuffer(b"".join(bytes(e) for e in expected), np.uint8).copy()
        npres = ctypes.c_int(0)
        _check(self._lib.mxec_reconstruct(
            self._h, k, m, shard_size, _pp([b.ctypes.data for b in bufs]), _szp(list(shard_len)),
            exp.ctypes.data_as(N.U8P) if exp is not None else None,
            present.ctypes.data_as(N.U8P), DATA_ONLY if data_only else 0, ctypes.byref(npres)))
        out = [bufs[i][: int(shard_len[i])] if present[i] else None for i in range(total)]
        return out, present

    # ---- completion-handle forms (mxec_*_async) -----------------------------
    def _submit(self, fn, args, keep, result) -> "Ticket":
        t = ctypes.c_void_p(0)
        _check(fn(*args, ctypes.byref(t)))
        return Ticket(self._lib, t, keep, result)

    def sha256_async(self, bufs: Sequence) -> "Ticket":
        arrs = [_u8(b) for b in bufs]
        out = np.zeros((max(1, len(arrs)), 32), np.uint8)
        ptrs, lens = _pp([_ptr(a) for a in arrs]), _szp([a.size for a in arrs])
        return self._submit(self._lib.mxec_sha256_batch_async,
                            (self._h, ptrs, lens, len(arrs), out.ctypes.data_as(N.U8P)), (arrs, out, ptrs, lens),
                            lambda: [bytes(out[i]) for i in range(len(arrs))])

    def encode_async(self, data: Sequence, m: int, shard_size: int) -> "Ticket":
        arrs = [_u8(d) for d in data]
        k = len(arrs)
        parity = [np.zeros(shard_size, np.uint8) for _ in range(max(m, 0))]
        dig = np.zeros((max(1, k + m), 32), np.uint8)
        args = (self._h, k, m, shard_size, _pp([_ptr(a) for a in arrs]), _szp([a.size for a in arrs]),
                _pp([p.ctypes.data for p in parity]), dig.ctypes.data_as(N.U8P))
        return self._submit(self._lib.mxec_encode_async, args, (arrs, parity, dig),
                            lambda: (parity, [bytes(dig[i]) for i in range(k + m)]))

    def reconstruct_async(self, shards: Sequence[Optional[object]], k: int, m: int, shard_size: int,
                          shard_len: Optional[Sequence[int]] = None,
                          expected: Optional[Sequence[bytes]] = None) -> "Ticket":
        total = k + m
        if shard_len is None:
            shard_len = [shard_size] * total
        bufs, present = [], np.zeros(total, np.uint8)
        for i in range(total):
            s = shards[i] if i < len(shards) else None
            if s is None:
                bufs.append(np.zeros(max(int(shard_len[i]), 1), np.uint8))
            else:
                a = np.array(_u8(s), dtype=np.uint8, copy=True)
                bufs.append(a if a.size else np.zeros(1, np.uint8))
                present[i] = 1
        exp = None
        if expected is not None:
            exp = np.frombuffer(b"".join(bytes(e) for e in expected), np.uint8).copy()
        npres = ctypes.c_int(0)
        args = (self._h, k, m, shard_size, _pp([b.ctypes.data for b in bufs]), _szp(list(shard_len)),
                exp.ctypes.data_as(N.U8P) if exp is not None else None, present.ctypes.data_as(N.U8P), 0,
                ctypes.byref(npres))
        return self._submit(self._lib.mxec_reconstruct_async, args, (bufs, present, exp, npres),
                            lambda: ([bufs[i][: int(shard_len[i])] if present[i] else None for i in range(total)],
                                     present))

    def put_object_chunked_async(self, ec_dir: str, chunk_size: int, parity_shards: int, body) -> "Ticket":
        b = _u8(body)
        return self._submit(self._lib.mxec_put_object_chunked_async,
                            (self._h, ec_dir.encode(), chunk_size, parity_shards, _ptr(b) if b.size else None,
                             b.size), (b,), None)

    def get_object_chunked_async(self, ec_dir: str, capacity: int, offset: int = 0,
                                 length: Optional[int] = None) -> "Ticket":
        out = np.zeros(max(1, capacity), np.uint8)
        n = ctypes.c_uint64(0)
        args = (self._h, ec_dir.encode(), offset, (1 << 64) - 1 if length is None else length, out.ctypes.data,
                capacity, ctypes.byref(n))
        return self._submit(self._lib.mxec_get_object_chunked_async, args, (out, n),
                            lambda: out[: n.value].tobytes())

    # ---- device-resident batches (integer device pointers) ------------------
    def encode_strided_device(self, k, m, shard_size, n_obj, data_ptr, data_obj_stride,
                              data_shard_stride, parity_ptr, parity_obj_stride, parity_shard_stride,
                              data_len=None, digests_ptr=None, dev=0, stream=None):
        _check(self._lib.mxec_encode_strided_device(
            self._h, dev, stream, k, m, shard_size, n_obj, data_ptr, data_obj_stride,
            data_shard_stride, _u64p(data_len) if data_len is not None else None, parity_ptr,
            parity_obj_stride, parity_shard_stride, digests_ptr))

    def encode_batch_device(self, objs: Sequence[tuple], data_ptrs, parity_ptrs, data_len=None,
                            digests_ptr=None, dev=0, stream=None):
        """Objects of mixed (k, m, shard_size); one launch per m (ctypes
        arrays for objs / pointers / lengths pass through as built)."""
        arr = objs if isinstance(objs, ctypes.Array) else (N.Object * len(objs))(*[N.Object(k, m, s) for (k, m, s) in objs])
        dp = data_ptrs if isinstance(data_ptrs, ctypes.Array) else _pp(data_ptrs)
        pp = parity_ptrs if isinstance(parity_ptrs, ctypes.Array) else _pp(parity_ptrs)
        dl = None if data_len is None else (data_len if isinstance(data_len, ctypes.Array) else _u64p(data_len))
        _check(self._lib.mxec_encode_batch_device(self._h, dev, stream, arr, len(objs), dp, dl, pp, digests_ptr))

    def encode_batch_host(self, objs: Sequence[tuple], data_ptrs, parity_ptrs, data_len=None,
                          digests: Optional[np.ndarray] = None, return_rc: bool = False):
        """mxec_encode_batch_host: host pointers in and out (ints), pipelined
        over every device.  digests: uint8 array of sum(k+m)*32 or None.
        Returns the per-object status array (with return_rc: (rc, status),
        no exception on a failing object)."""
        arr = (N.Object * len(objs))(*[N.Object(k, m, s) for (k, m, s) in objs])
        status = np.zeros(max(1, len(objs)), np.int32)
        rc = self._lib.mxec_encode_batch_host(
            self._h, arr, len(objs), _pp(data_ptrs),
            _u64p(data_len) if data_len is not None else None, _pp(parity_ptrs),
            digests.ctypes.data_as(N.U8P) if digests is not None else None,
            status.ctypes.data_as(N.I32P))
        if return_rc:
            return rc, status[: len(objs)]
        _check(rc)
        return status[: len(objs)]

    def reconstruct_batch_host(self, objs: Sequence[tuple], shard_ptrs, present: np.ndarray, shard_len=None,
                               expected: Optional[np.ndarray] = None, data_only: bool = False):
        """mxec_reconstruct_batch_host: host pointers (ints) for every shard,
        sum(k+m) object-major (a missing shard's pointer receives its rebuilt
        bytes); present (uint8, sum(k+m)) updated in place; expected: uint8
        array of sum(k+m)*32 digests or None.  Returns (rc, per-object
        status array)."""
        n = len(objs)
        arr = objs if isinstance(objs, ctypes.Array) else (N.Object * n)(*[N.Object(k, m, s) for (k, m, s) in objs])
        assert present.dtype == np.uint8
        status = np.zeros(max(1, n), np.int32)
        sp = shard_ptrs if isinstance(shard_ptrs, ctypes.Array) else _pp(shard_ptrs)
        sl = None if shard_len is None else (shard_len if isinstance(shard_len, ctypes.Array) else _u64p(shard_len))
        rc = self._lib.mxec_reconstruct_batch_host(
            self._h, arr, n, sp, sl, present.ctypes.data_as(N.U8P),
            expected.ctypes.data_as(N.U8P) if expected is not None else None,
            DATA_ONLY if data_only else 0, status.ctypes.data_as(N.I32P))
        return rc, status[:n]

    def reconstruct_strided_device(self, k, m, shard_size, n_obj, shards_ptr, obj_stride,
                                   shard_stride, present: np.ndarray, shard_len=None,
                                   expected_ptr=None, data_only=False, dev=0, stream=None):
        """present: uint8 array of n_obj*(k+m), updated in place.  Returns
        (rc, per-object status array)."""
        assert present.dtype == np.uint8 and present.size == n_obj * (k + m)
        status = np.zeros(max(1, n_obj), np.int32)
        rc = self._lib.mxec_reconstruct_strided_device(
            self._h, dev, stream, k, m, shard_size, n_obj, shards_ptr, obj_stride, shard_stride,
            _u64p(shard_len) if shard_len is not None else None, present.ctypes.data_as(N.U8P),
            expected_ptr, DATA_ONLY if data_only else 0, status.ctypes.data_as(N.I32P))
        return rc, status[:n_obj]

    def reconstruct_strided_device_async(self, k, m, shard_size, n_obj, shards_ptr, obj_stride,
                                         shard_stride, present: np.ndarray, shard_len=None,
                                         expected_ptr=None, data_only=False, dev=0,
                                         stream=None) -> "Ticket":
        """The completion-handle form: `present` is updated in place when the
        ticket completes; wait() returns the per-object status array."""
        assert present.dtype == np.uint8 and present.size == n_obj * (k + m)
        status = np.zeros(max(1, n_obj), np.int32)
        sl = _u64p(shard_len) if shard_len is not None else None
        args = (self._h, dev, stream, k, m, shard_size, n_obj, shards_ptr, obj_stride, shard_stride, sl,
                present.ctypes.data_as(N.U8P), expected_ptr, DATA_ONLY if data_only else 0,
                status.ctypes.data_as(N.I32P))
        return self._submit(self._lib.mxec_reconstruct_strided_device_async, args, (present, status, sl),
                            lambda: status[:n_obj])

    def reconstruct_batch_device(self, objs, shard_ptrs, present: np.ndarray, shard_len=None,
                                 expected_ptr=None, data_only=False, dev=0, stream=None):
        """mxec_reconstruct_batch_device: objects of mixed (k, m, shard_size);
        shard_ptrs / shard_len / present concatenated over objects (sum(k+m)
        each; ctypes arrays pass through as built).  present (uint8) is updated
        in place.  Returns (rc, per-object status array)."""
        n = len(objs)
        arr = objs if isinstance(objs, ctypes.Array) else (N.Object * n)(*[N.Object(k, m, s) for (k, m, s) in objs])
        assert present.dtype == np.uint8
        status = np.zeros(max(1, n), np.int32)
        sp = shard_ptrs if isinstance(shard_ptrs, ctypes.Array) else _pp(shard_ptrs)
        sl = None if shard_len is None else (shard_len if isinstance(shard_len, ctypes.Array) else _u64p(shard_len))
        rc = self._lib.mxec_reconstruct_batch_device(
            self._h, dev, stream, arr, n, sp, sl, present.ctypes.data_as(N.U8P), expected_ptr,
            DATA_ONLY if data_only else 0, status.ctypes.data_as(N.I32P))
        return rc, status[:n]

    def reconstruct_batch_device_async(self, objs, shard_ptrs, present: np.ndarray, shard_len=None,
                                       expected_ptr=None, data_only=False, dev=0, stream=None) -> "Ticket":
        """The completion-handle form of reconstruct_batch_device: `present`
        is updated in place when the ticket completes; wait() returns the
        per-object status array."""
        n = len(objs)
        arr = objs if isinstance(objs, ctypes.Array) else (N.Object * n)(*[N.Object(k, m, s) for (k, m, s) in objs])
        assert present.dtype == np.uint8
        status = np.zeros(max(1, n), np.int32)
        sp = shard_ptrs if isinstance(shard_ptrs, ctypes.Array) else _pp(shard_ptrs)
        sl = None if shard_len is None else (shard_len if isinstance(shard_len, ctypes.Array) else _u64p(shard_len))
        args = (self._h, dev, stream, arr, n, sp, sl, present.ctypes.data_as(N.U8P), expected_ptr,
                DATA_ONLY if data_only else 0, status.ctypes.data_as(N.I32P))
        return self._submit(self._lib.mxec_reconstruct_batch_device_async, args, (present, status),
                            lambda: status[:n])

    def sha256_batch_device(self, ptrs, lens, digests_ptr, dev=0, stream=None):
        _check(self._lib.mxec_sha256_batch_device(
            self._h, dev, stream, _pp(ptrs), _u64p(lens), len(ptrs), digests_ptr))

    # ---- file-level path (FilesystemStorage / VerifiedChunkReader) ---------
    @staticmethod
    def _info(ci: N.ChunkInfo) -> dict:
        d = {"index": int(ci.index), "size": int(ci.size), "sha256": ci.sha256.decode()}
        if ci.kind == 1:
            d["kind"] = "parity"
        return d

    def write_chunk(self, ec_dir: str, index: int, data) -> dict:
        a = _u8(data)
        ci = N.ChunkInfo()
        _check(self._lib.mxec_write_chunk(self._h, ec_dir.encode(), index, _ptr(a), a.size,
                                          ctypes.byref(ci)))
        return self._info(ci)

    def compute_and_write_parity(self, ec_dir: str, chunk_size: int, parity_shards: int,
                                 data_chunks: Sequence[dict]) -> list[dict]:
        k = len(data_chunks)
        ins = (N.ChunkInfo * max(1, k))()
        for i, c in enumerate(data_chunks):
            ins[i].index, ins[i].size = c["index"], c["size"]
            ins[i].sha256 = c["sha256"].encode()
        outs = (N.ChunkInfo * max(1, parity_shards))()
        _check(self._lib.mxec_compute_and_write_parity(self._h, ec_dir.encode(), chunk_size,
                                                       parity_shards, ins, k, outs))
        return [self._info(outs[i]) for i in range(parity_shards)]

    def put_object_chunked(self, ec_dir: str, chunk_size: int, parity_shards: int, body) -> None:
        a = _u8(body)
        _check(self._lib.mxec_put_object_chunked(self._h, ec_dir.encode(), chunk_size,
                                                 parity_shards, _ptr(a), a.size))

    def get_object_chunked(self, ec_dir: str, offset: int = 0, length: Optional[int] = None,
                           capacity: Optional[int] = None) -> bytes:
        import json
        import os

        if capacity is None:
            with open(os.path.join(ec_dir, "manifest.json")) as f:
                capacity = int(json.load(f)["total_size"])
        out = np.zeros(max(1, capacity), np.uint8)
        n = ctypes.c_uint64(0)
        _check(self._lib.mxec_get_object_chunked(
            self._h, ec_dir.encode(), offset, (1 << 64) - 1 if length is None else length,
            out.ctypes.data, capacity, ctypes.byref(n)))
        return out[: n.value].tobytes()

    def get_object_chunked_encrypted(self, ec_dir: str, key: bytes, aad_prefix: bytes, offset: int = 0,
                                     length: Optional[int] = None, plaintext_size: Optional[int] = None,
                                     frame_size: int = 65536) -> bytes:
        """GET / ranged GET of an encrypt-then-EC object (FrameDecryptor over
        VerifiedChunkReader, filesystem.rs:1618-1630, 1700-1725)."""
        import json
        import os

        if plaintext_size is None:
            with open(os.path.join(ec_dir, "manifest.json")) as f:
                cap = int(json.load(f).get("plaintext_size", 0))
        else:
            cap = plaintext_size
        out = np.zeros(max(1, cap), np.uint8)
        n = ctypes.c_uint64(0)
        k, ap = _u8(key), _u8(aad_prefix)
        _check(self._lib.mxec_get_object_chunked_encrypted(
            self._h, ec_dir.encode(), _ptr(k), _ptr(ap) if ap.size else None, ap.size, frame_size,
            (1 << 64) - 1 if plaintext_size is None else plaintext_size, offset,
            (1 << 64) - 1 if length is None else length, out.ctypes.data, cap, ctypes.byref(n)))
        return out[: n.value].tobytes()

    def open_reader(self, ec_dir: str, offset: int = 0, length: Optional[int] = None,
                    batch_bytes: int = 0) -> "ChunkReader":
        return ChunkReader(self, ec_dir, offset, length, batch_bytes)

    def body_sums(self, bodies: Sequence, which: int = 0x1F) -> list[dict]:
        """mxec_body_sums_batch: digests of host bodies (one dict each)."""
        arrs = [_u8(b) for b in bodies]
        n = len(arrs)
        if n == 0:
            return []
        out = (N.BodySums * n)()
        _check(self._lib.mxec_body_sums_batch(self._h, _pp([_ptr(a) for a in arrs]),
                                              _u64p([a.size for a in arrs]), n, which, out))
        return [_sums_dict(out[i], which) for i in range(n)]

    def body_sums_device(self, ptrs, lens, out_ptr: int, which: int = 0x1F, dev: int = 0, stream=None):
        """mxec_body_sums_batch_device: records (76 B each) written to out_ptr."""
        _check(self._lib.mxec_body_sums_batch_device(self._h, dev, stream, _pp(ptrs), _u64p(lens),
                                                     len(ptrs), which, out_ptr))

    def put_object_chunked_sums(self, ec_dir: str, chunk_size: int, parity_shards: int, body,
                                checksum_algo: Optional[str] = None) -> dict:
        """put_object_chunked + PutResult etag / checksum_value."""
        a = _u8(body)
        which = SUM_MD5 | (_SUM_BY_ALGO[checksum_algo] if checksum_algo else 0)
        r = N.BodySums()
        _check(self._lib.mxec_put_object_chunked_sums(self._h, ec_dir.encode(), chunk_size, parity_shards,
                                                      _ptr(a), a.size, which, ctypes.byref(r)))
        return put_result(_sums_dict(r, which), checksum_algo)

    def put_object_chunked_encrypted(self, ec_dir: str, chunk_size: int, parity_shards: int, key: bytes,
                                     nonce_prefix: bytes, aad_prefix: bytes, body,
                                     checksum_algo: Optional[str] = None) -> dict:
        """put_object_chunked_encrypted (filesystem.rs:835-1060): frames, chunks,
        parity, manifest with plaintext_size; returns the PutResult digests."""
        a, k, pre, ap = _u8(body), _u8(key), _u8(nonce_prefix), _u8(aad_prefix)
        which = SUM_MD5 | (_SUM_BY_ALGO[checksum_algo] if checksum_algo else 0)
        r = N.BodySums()
        _check(self._lib.mxec_put_object_chunked_encrypted(
            self._h, ec_dir.encode(), chunk_size, parity_shards, _ptr(k), _ptr(pre),
            _ptr(ap) if ap.size else None, ap.size, _ptr(a), a.size, which, ctypes.byref(r)))
        return put_result(_sums_dict(r, which), checksum_algo)

    @staticmethod
    def _parts(parts: Sequence[dict]):
        arr = (N.MultipartPart * max(1, len(parts)))()
        for i, p in enumerate(parts):
            arr[i].path = p["path"].encode()
            arr[i].size = p["size"]
            arr[i].md5[:] = list(bytes.fromhex(p["etag"].strip('"')))
            arr[i].part_number = p["part_number"]
            arr[i].encrypted = 1 if p.get("encrypted") else 0
        return arr

    def complete_multipart_chunked(self, ec_dir: str, chunk_size: int, parity_shards: int,
                                   parts: Sequence[dict]) -> str:
        """complete_multipart_chunked (filesystem.rs:1147-1310); parts: dicts of
        path, size, etag (hex), part_number.  Returns the quoted ETag."""
        etag = ctypes.create_string_buffer(48)
        _check(self._lib.mxec_complete_multipart_chunked(self._h, ec_dir.encode(), chunk_size, parity_shards,
                                                         self._parts(parts), len(parts), etag))
        return '"' + etag.value.decode() + '"'

    def complete_multipart_chunked_encrypted(self, ec_dir: str, chunk_size: int, parity_shards: int,
                                             parts: Sequence[dict], upload_key: bytes, upload_id: str,
                                             key: bytes, nonce_prefix: bytes, aad_prefix: bytes) -> str:
        """complete_multipart_chunked_encrypted (filesystem.rs:1315-1560)."""
        etag = ctypes.create_string_buffer(48)
        uk, k, pre, ap = _u8(upload_key), _u8(key), _u8(nonce_prefix), _u8(aad_prefix)
        _check(self._lib.mxec_complete_multipart_chunked_encrypted(
            self._h, ec_dir.encode(), chunk_size, parity_shards, self._parts(parts), len(parts), _ptr(uk),
            upload_id.encode(), _ptr(k), _ptr(pre), _ptr(ap) if ap.size else None, ap.size, etag))
        return '"' + etag.value.decode() + '"'

    # ---- encrypt-then-EC frames (storage/crypto.rs) ----------------------------
    def frames_encrypt(self, key: bytes, nonce_prefix: bytes, pt, aads: Optional[Sequence[bytes]] = None,
                       first_index: int = 0, frame_size: int = FRAME_CHUNK_SIZE) -> bytes:
        """FrameEncryptor over a whole buffer (aads[i] = frame i's AAD)."""
        p = _u8(pt)
        total = int(self._lib.mxec_frames_len(p.size, frame_size))
        out = np.zeros(max(1, total), np.uint8)
        a = _u8(b"".join(aads)) if aads else np.zeros(0, np.uint8)
        alen = len(aads[0]) if aads else 0
        n = ctypes.c_uint64(0)
        k, pre = _u8(key), _u8(nonce_prefix)
        _check(self._lib.mxec_frames_encrypt(self._h, _ptr(k), _ptr(pre), first_index, _ptr(a) if alen else None,
                                             alen, frame_size, _ptr(p), p.size, out.ctypes.data, total,
                                             ctypes.byref(n)))
        return out[: n.value].tobytes()

    def frames_decrypt(self, key: bytes, frames, plaintext_size: int, aads: Optional[Sequence[bytes]] = None,
                       first_index: int = 0, frame_size: int = FRAME_CHUNK_SIZE) -> bytes:
        """FrameDecryptor over a whole buffer; RSError(Integrity) on a bad frame."""
        f = _u8(frames)
        out = np.zeros(max(1, plaintext_size), np.uint8)
        a = _u8(b"".join(aads)) if aads else np.zeros(0, np.uint8)
        alen = len(aads[0]) if aads else 0
        n = ctypes.c_uint64(0)
        k = _u8(key)
        _check(self._lib.mxec_frames_decrypt(self._h, _ptr(k), first_index, _ptr(a) if alen else None, alen,
                                             frame_size, _ptr(f), f.size, plaintext_size, out.ctypes.data,
                                             plaintext_size, ctypes.byref(n)))
        return out[: n.value].tobytes()

    def frames_device(self, jobs: Sequence[dict], decrypt: bool = False, dev: int = 0, stream=None):
        """mxec_frames_{en,de}crypt_device; jobs: dicts with key, nonce_prefix,
        frame_size, first_index, aad_dev, aad_len, in_dev, len, out_dev.
        Decrypt returns the per-job status list."""
        arr = (N.FramesJob * max(1, len(jobs)))()
        keep = []
        for i, j in enumerate(jobs):
            k = _u8(j["key"])
            keep.append(k)
            arr[i].key = _ptr(k)
            for b, v in enumerate(j.get("nonce_prefix", b"\0\0\0\0")):
                arr[i].nonce_prefix[b] = v
            arr[i].frame_size = j.get("frame_size", FRAME_CHUNK_SIZE)
            arr[i].first_index = j.get("first_index", 0)
            arr[i].aad_dev = j.get("aad_dev") or None
            arr[i].aad_len = j.get("aad_len", 0)
            arr[i].in_dev = j["in_dev"]
            arr[i].len = j["len"]
            arr[i].out_dev = j["out_dev"]
        if not decrypt:
            _check(self._lib.mxec_frames_encrypt_device(self._h, dev, stream, arr, len(jobs)))
            return None
        st = (ctypes.c_int32 * max(1, len(jobs)))()
        self._lib.mxec_frames_decrypt_device(self._h, dev, stream, arr, len(jobs), st)
        return [int(st[i]) for i in range(len(jobs))]

    def frame_aads(self, prefix: bytes, first_index: int, n: int) -> list[bytes]:
        """build_frame_aad for frames first_index .. first_index + n - 1."""
        if n == 0:
            return []
        p = _u8(prefix)
        out = np.zeros((n, 32), np.uint8)
        _check(self._lib.mxec_frame_aads(self._h, _ptr(p), p.size, first_index, n, out.ctypes.data))
        return [out[i].tobytes() for i in range(n)]

    def try_reconstruct_data_chunk(self, ec_dir: str, target: int, capacity: int = 1 << 26) -> bytes:
        out = np.zeros(max(1, capacity), np.uint8)
        n = ctypes.c_uint64(0)
        _check(self._lib.mxec_try_reconstruct_data_chunk(self._h, ec_dir.encode(), target,
                                                         out.ctypes.data, capacity, ctypes.byref(n)))
        return out[: n.value].tobytes()


class Ticket:
    """An mxec_ticket (completion handle of an *_async call).  `fd` is an
    eventfd that becomes readable when the call is done (select / asyncio
    add_reader); `wait()` returns the result or raises RSError.  Keeps the
    call's buffers alive until it completes."""

    def __init__(self, lib, handle, keep, result):
        self._lib, self._h, self._keep, self._result = lib, handle, keep, result

    @property
    def fd(self) -> int:
        return self._lib.mxec_ticket_fd(self._h)

    def done(self) -> bool:
        return self._lib.mxec_ticket_poll(self._h) == 1

    def wait(self):
        rc = self._lib.mxec_ticket_wait(self._h)
        msg = self._lib.mxec_ticket_error(self._h).decode()
        self.close()
        if rc != 0:
            raise RSError(rc, msg)
        return self._result() if self._result else None

    def close(self) -> None:
        if self._h:
            self._lib.mxec_ticket_free(self._h)
            self._h = None
            self._keep = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class ChunkReader:
    """Mirror of VerifiedChunkReader (chunk_reader.rs:12-276): ``read(n)``
    returns up to n bytes, b"" at the end of the range, and raises RSError
    when it reaches a chunk that is corrupt and cannot be rebuilt -- after the
    bytes before that chunk have been returned by earlier reads."""

    def __init__(self, ctx: "Context", ec_dir: str, offset: int = 0, length: Optional[int] = None,
                 batch_bytes: int = 0):
        self._lib = ctx._lib
        self._ctx = ctx  # keeps the device context alive while the reader is open
        h = ctypes.c_void_p()
        _check(self._lib.mxec_reader_open(ctx._h, ec_dir.encode(), offset,
                                          (1 << 64) - 1 if length is None else length,
                                          batch_bytes, ctypes.byref(h)))
        self._r = h

    def read(self, n: int = 1 << 20) -> bytes:
        buf = np.empty(max(1, n), np.uint8)
        got = self._lib.mxec_reader_read(self._r, buf.ctypes.data, n)
        if got < 0:
            _check(int(got))
        return buf[:got].tobytes()

    def close(self) -> None:
        if self._r:
            self._lib.mxec_reader_close(self._r)
            self._r = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()


class ReedSolomon:
    """Mirror of reed_solomon_erasure::galois_8::ReedSolomon (crate 6.0.0)."""

    def __init__(self, data_shards: int, parity_shards: int, ctx: Optional[Context] = None):
        rs_check(data_shards, parity_shards)
        self.k, self.m = data_shards, parity_shards
        self.ctx = ctx or _default_ctx()

    def data_shard_count(self) -> int:
        return self.k

    def parity_shard_count(self) -> int:
        return self.m

    def total_shard_count(self) -> int:
        return self.k + self.m

    def _check_shards(self, shards, allow_none=False):
        if len(shards) < self.k + self.m:
            raise RSError(-1, "too few shards")
        if len(shards) > self.k + self.m:
            raise RSError(-2, "too many shards")
        sizes = {len(s) for s in shards if s is not None}
        if not sizes:
            raise RSError(-10, "no shard present")
        if len(sizes) != 1:
            raise RSError(-9, "shard sizes differ")
        size = sizes.pop()
        if size == 0:
            raise RSError(-11, "empty shard")
        return size

    def encode(self, shards: list) -> None:
        """Fill shards[k:] with parity (in place), like the crate's encode."""
        size = self._check_shards(shards)
        parity, _ = self.ctx.encode(shards[: self.k], self.m, size, digests=False)
        for i in range(self.m):
            target = shards[self.k + i]
            if isinstance(target, np.ndarray):
                target.reshape(-1).view(np.uint8)[:] = parity[i]
            else:
                target[:] = parity[i].tobytes()

    def verify(self, shards: list) -> bool:
        size = self._check_shards(shards)
        parity, _ = self.ctx.encode(shards[: self.k], self.m, size, digests=False)
        return all(bytes(_u8(shards[self.k + i])) == parity[i].tobytes() for i in range(self.m))

    def _reconstruct(self, shards: list, data_only: bool) -> None:
        size = self._check_shards(shards, allow_none=True)
        present = sum(s is not None for s in shards)
        if present == self.k + self.m:
            return
        if present < self.k:
            raise RSError(-10, "too few shards present")
        out, _ = self.ctx.reconstruct(shards, self.k, self.m, size, data_only=data_only)
        for i in range(self.k + self.m):
            if shards[i] is None and out[i] is not None:
                shards[i] = bytearray(out[i].tobytes())

    def reconstruct(self, shards: list) -> None:
        self._reconstruct(shards, False)

    def reconstruct_data(self, shards: list) -> None:
        self._reconstruct(shards, True)


_ctx_singleton: Optional[Context] = None


def _default_ctx() -> Context:
    global _ctx_singleton
    if _ctx_singleton is None:
        _ctx_singleton = Context()
    return _ctx_singleton

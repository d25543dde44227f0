#!/usr/bin/env python3
"""bench.py — device-resident RS encode / reconstruct throughput on MI355X.

Default step (BASELINE configs[1], the metric's configuration): Reed–Solomon
encode of 1024 objects per GPU, k=4 data + m=2 parity shards of chunk_size =
10 MiB each (MaxIO `--chunk-size 10485760 --parity-shards 2`, 40 MiB objects),
inputs resident in HBM, parity written to HBM, through the C ABI
(mxec_encode_strided_device) on a dedicated HIP stream.

  python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4a|4b|5] [--no-extra] [--no-e2e]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

--gpus N in one process opens ONE mxec_ctx over GPUs 0..N-1 (MaxIO's
production shape): each GPU gets its own objects (object i -> GPU i mod N,
seeded per GPU), stream, HIP events and host thread; the step is timed over
all of them (wall clock, after a sync of every device) and the roofline is
the slowest GPU's kernel, with a per-GPU list.  Under torch.distributed.run
each rank drives GPU LOCAL_RANK and --gpus must equal WORLD_SIZE.  Fewer
visible GPUs than --gpus: exit 2 with a message and no JSON line
(BENCH_REHEARSE_LOGICAL=1: a labelled rehearsal on logical devices of one
card instead).  The default config-2 run also reports extra.e2e_host: the
same encode from page-locked host memory through mxec_encode_batch_host
(PCIe included) over every GPU of the run.

Other BASELINE configs (same JSON line, for DESIGN.md / profiles):
  3   reconstruct k=8 m=4, 2 data erasures + SHA-256 verify of the 10 present
      shards, 1 MiB chunks, 1024 objects (8192 data chunks) per GPU
  3c  the same batches as a continuous GET stream: --workers host threads
      (default 8) each reconstructing its own batch on its own HIP stream
  ns  encode k=8 m=4, 1 MiB chunks, 4096 objects per GPU (north_star's
      target shape)
  4a  encode k=10 m=4, 1 MiB chunks (10 MiB objects), 4096 objects per GPU
  4b  encode k=64 m=4, 1 MiB chunks (literal 64 MiB objects), 640 per GPU
  5   mixed 4+2 / 8+4 / 10+4 at 64 KiB..10 MiB chunks with short last chunks:
      encode the batch, then reconstruct it with seeded erasures, per step
      (one mixed-shape batch call each way; BENCH_MIXED_MODE=streams: the
      classes as separate calls on four streams)

Objects are partitioned per GPU (weak scaling, no collective on the data
path; only the timing barrier / max-reduce between ranks).  Rank 0 prints
ONE JSON line.  value = payload GiB/s (k * chunk_size bytes per object)
over all GPUs; roofline = the dominant kernel's algorithmic bytes / its
HIP-event-timed duration vs 8 TB/s; cpu_baseline = oracle/ (C restatement of
the crate's pure-Rust path) on one host core over a bounded sample, plus the
same on every host core as cpu_baseline_all_cores.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident RS encode+reconstruct GiB/s (k+m, chunk_size); % HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GIB = float(1 << 30)
# INT32-VALU roofline of the SHA-256 kernels (configs 3 / 3c):
# lane-ops per 64-byte block = the wave-instructions each form issues per
# block (one wave instruction serves 64 messages, one block each), counted in
# the gfx950 ISA of the loop bodies (tools/isa_count.py): split form =
# consumer 905 (64 rounds x 14 + 9) + producer 565 (2261 per 4-block step);
# one-wave form 1410 (64 x 14 rounds + 48 x 10 schedule + 16 byte swaps + 18);
# stream form 1415 (the one-wave rounds plus the clamped prefetch).
# Quad form (the lag variant with two messages per quad, 64 messages per
# workgroup): since round 5 two producer waves (two lanes per message, 367
# wave-instructions per block each) + 2 consumers x 607 over 64 messages =
# 1948 lane-ops per message-block (round 4's one producer wave: 566, 1780);
# it spends more lane-ops per hash to cut the serial wave's count, so config 3
# keeps the one-lane split form's 1470 as its chip-wide denominator
# (comparable across rounds).
SHA_VALU_PER_BLOCK = {"split": 1470, "one": 1410, "stream": 1415, "quad": 1948}
# The serial wave (the consumer) of each latency form issues this many VALU
# per block (split: 64 rounds x 14 + 9; quad, lag variant: 66 steps x 9 + 13); a wave issues at
# most one VALU every 4 cycles, so a lone message's chain cannot beat that
# x 4 cycles per block at the clock the chip holds.
SHA_CONSUMER_VALU_PER_BLOCK = {"split": 905, "quad": 607}
SHA_QUAD_MSGS_PER_CU = 64  # the lag form, two messages per quad
# The hardware floor of ONE message's chain, whatever the form: a round's
# e' (and a') depends on the previous one through Σ's rotates, their XOR3 and
# one three-way add (Ch / Maj and the h + d + K + W sums run beside it), so a
# round cannot take less than the dependent latencies of v_alignbit_b32 ->
# v_bitop3_b32 -> v_add3_u32 measured for one wave alone on its SIMD
# (tools/valu_lab.cpp, profiles/r1_lab_valu_issue.jsonl, chains = 1).
SHA_ROUND_DEP_CYCLES = 10.77 + 8.63 + 8.63
# Chip INT32 issue ceiling for those instructions (v_alignbit / v_bitop3 /
# v_add3 / v_add / v_perm): CUs x 4 SIMDs x lanes per cycle x 2.4 GHz, lanes
# per cycle measured with tools/valu_lab chip (profiles/r2_lab_valu_chip.jsonl).
VALU_LANES_PER_SIMD_CYCLE = 16
CLOCK_GHZ = 2.4
SEED = 0x6D6178696F  # "maxio"


def shard_objects(n_total: int, rank: int, world: int) -> range:
    """Objects of the global batch owned by `rank`: object i -> GPU i mod G
    (DESIGN §6)."""
    return range(rank, n_total, world)


def reduce_max(value: float) -> float:
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return value
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/baseline infrastructure only

    return oracle


def cpu_leg(work, payload_per_call: int, seconds: float, threads: int):
    """Run `work(i)` (an oracle call; ctypes drops the GIL) on `threads`
    threads for about `seconds`; returns (GiB/s, calls, elapsed)."""
    work(0)  # warm tables / page in
    stop = time.perf_counter() + seconds
    counts = [0] * threads

    def run(t):
        while time.perf_counter() < stop:
            work(t)
            counts[t] += 1

    t0 = time.perf_counter()
    ths = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    n = sum(counts)
    return n * payload_per_call / GIB / el, n, el


# ---- workloads ------------------------------------------------------------------


class _DevMem:
    """Device memory the library allocated, viewed by torch without a copy
    (__cuda_array_interface__; torch.as_tensor wraps it)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 2, "strides": None}


class Encode:
    """RS encode of n uniform objects (data [n][k][S] -> parity [n][m][S])."""

    bound = "hbm"

    def __init__(self, torch, ctx, dev, sh, k, m, S, n, label, seed, streams=1, separate=False):
        self.torch, self.ctx, self.sh = torch, ctx, sh
        self.separate = separate
        self.k, self.m, self.S, self.n = k, m, S, n
        # streams > 1 (BENCH_ENCODE_STREAMS, lab): the batch as that many
        # launches over consecutive object ranges on their own streams,
        # joined on the bench's stream.
        self.main = torch.cuda.ExternalStream(sh, device=dev)
        self.streams = [self.main] if streams <= 1 else [torch.cuda.Stream(device=dev) for _ in range(streams)]
        g = torch.Generator(device=dev).manual_seed(seed)
        # Object-major [n][k+m][S]: each object's parity right after its data
        # (an object's shards staged together, the layout the reconstruct
        # configs use).  With data [n][k][S] and parity [n][m][S] as two
        # allocations the rate followed the parity buffer's physical
        # placement (5.25-6.29 TB/s from one allocation to the next); parity
        # interleaved with data measured 5.85-6.08 (tools/alloc_lab.py,
        # profiles/r2_cfg2_allocation_spread.txt).
        # Multi-MiB shard slots are padded by 2 MiB + 64 KiB, so an object's
        # slots start at different offsets modulo 2 MiB: on one box the
        # unpadded layout fell to 5.2 TB/s on 2 of 8 allocations and the
        # padded one on none; elsewhere the pad measured +1 %
        # (profiles/r2_shard_pad_spread.txt).
        self.pad = (2 << 20) + (64 << 10) if S >= (4 << 20) and not separate else 0
        self.sstride = S + self.pad
        # The batch's HBM from the library's batch allocator (mxec_batch_alloc,
        # placement.cpp): of two allocations x two shard strides, the one its
        # own encode ran fastest on (where a batch lies moves the encode by up
        # to ~8 %).  BENCH_TORCH_ALLOC=1: torch's allocator at the
        # round-2 pad instead (the A/B).
        self.batch_ptr = None
        self.placement = None
        lib_alloc = not separate and os.environ.get("BENCH_TORCH_ALLOC") != "1"
        if separate:
            # What a caller with its own buffers hands the *_device API: data
            # [n][k][S] and parity [n][m][S] as two allocations, no pad
            # (extra.config2_separate_buffers).
            self.obj = torch.empty((n, k, S), dtype=torch.uint8, device=dev)
            for o in range(n):
                self.obj[o].copy_(torch.randint(0, 256, (k, S), dtype=torch.uint8, device=dev, generator=g))
            self.par_buf = torch.zeros((n, m, S), dtype=torch.uint8, device=dev)
            self.data, self.parity = self.obj, self.par_buf
            self.stride, self.pstride = k * S, m * S
        else:
            if lib_alloc:
                ptr, stride, probe = ctx.batch_alloc(k, m, S, n)
                self.batch_ptr, self.sstride, self.pad = ptr, stride, stride - S
                self.placement = {"allocator": "mxec_batch_alloc", "shard_stride": stride, "pad": stride - S,
                                  "probe_ms": probe}
                self.obj = torch.as_tensor(_DevMem(ptr, n * (k + m) * stride), device=dev).view(n, k + m, stride)
            else:
                self.obj = torch.empty((n, k + m, self.sstride), dtype=torch.uint8, device=dev)
                self.placement = {"allocator": "torch", "shard_stride": self.sstride, "pad": self.pad}
            for o in range(n):  # per object keeps the randint temporary small
                self.obj[o, :k, :S].copy_(torch.randint(0, 256, (k, S), dtype=torch.uint8, device=dev, generator=g))
            self.obj[:, k:].zero_()
            self.data, self.parity = self.obj[:, :k, :S], self.obj[:, k:, :S]
            self.stride = self.pstride = (k + m) * self.sstride
        self.payload = n * k * S
        self.alg_bytes = n * (k + m) * S
        r = min(m, 8)
        self.kernel = f"rs_apply_fast<R={r},V={4 if r <= 4 else 2},NT=1>"
        self.name = label

    def step(self):
        k, m, S = self.k, self.m, self.S
        if len(self.streams) == 1:
            self.ctx.encode_strided_device(k, m, S, self.n, self.data.data_ptr(), self.stride, self.sstride,
                                           self.parity.data_ptr(), self.pstride, self.sstride, stream=self.sh)
            return
        ns = len(self.streams)
        for st in self.streams:
            st.wait_stream(self.main)
        for i, st in enumerate(self.streams):
            a, b = self.n * i // ns, self.n * (i + 1) // ns
            self.ctx.encode_strided_device(k, m, S, b - a, self.data[a].data_ptr(), self.stride, self.sstride,
                                           self.parity[a].data_ptr(), self.pstride, self.sstride,
                                           stream=st.cuda_stream)
        for st in self.streams:
            self.main.wait_stream(st)

    def spot_check(self):
        """First, middle and last object, and the objects either side of
        every grid-stride iteration boundary of the grid in use, against the
        oracle (most of a full batch's tiles run in iterations >= 2)."""
        import numpy as np

        oracle = _oracle()
        r = min(self.m, 8)
        tile = 16384 if self.m <= 4 else 8192
        n_cus = self.torch.cuda.get_device_properties(self.data.device).multi_processor_count
        bpc = self.ctx.rs_grid(self.k, self.m, self.S) or rs_blocks_per_cu(r)
        for o in spot_objects(self.n, -(-self.S // tile), bpc * n_cus):
            want = oracle.encode(list(self.data[o].cpu().numpy()), self.m, self.S)
            got = self.parity[o].cpu().numpy()
            if not all(np.array_equal(got[i], want[i]) for i in range(self.m)):
                return False
        return True

    def cpu_work(self):
        import numpy as np

        oracle = _oracle()
        rng = np.random.default_rng(SEED)
        objs = [[rng.integers(0, 256, self.S, dtype=np.uint8) for _ in range(self.k)] for _ in range(2)]
        return (lambda i: oracle.encode(objs[i % 2], self.m, self.S)), self.k * self.S, (
            f"encode k={self.k} m={self.m} chunk_size={self.S}: oracle/rs_oracle.c "
            "(crate 6.0.0 pure-Rust mul_slice restated: 64 KiB MUL_TABLE, input-major)")

    def drop(self):
        del self.data, self.parity, self.obj
        if self.separate:
            del self.par_buf
        if self.batch_ptr:
            self.torch.cuda.synchronize()
            self.ctx.batch_free(self.batch_ptr)
            self.batch_ptr = None


class Reconstruct:
    """configs[2]: k=8 m=4, 2 seeded data erasures per object, SHA-256 verify
    of the present shards (chunk_reader.rs:176-196), rebuild, 1 MiB chunks."""

    bound = "valu"

    def __init__(self, torch, ctx, dev, sh, n, seed):
        import numpy as np

        self.torch, self.ctx, self.sh = torch, ctx, sh
        self.k, self.m, self.S, self.n = 8, 4, 1 << 20, n
        k, m, S = self.k, self.m, self.S
        g = torch.Generator(device=dev).manual_seed(seed)
        self.obj = torch.randint(0, 256, (n, k + m, S), dtype=torch.uint8, device=dev, generator=g)
        self.dig = torch.empty((n, k + m, 32), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()  # randint ran on the current stream; encode runs on sh
        ctx.encode_strided_device(k, m, S, n, self.obj.data_ptr(), (k + m) * S, S,
                                  self.obj[:, k:].data_ptr(), (k + m) * S, S,
                                  digests_ptr=self.dig.data_ptr(), stream=sh)
        torch.cuda.synchronize()
        # first / middle / last object and both sides of each grid-stride
        # iteration boundary of the R = 2 decode (64 tiles per object)
        n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
        self.spot = spot_objects(n, 64, rs_blocks_per_cu(2) * n_cus)
        self.ref = self.obj[self.spot].clone()
        rng = np.random.default_rng(seed)
        self.present0 = np.ones(n * (k + m), np.uint8)
        for o in range(n):
            for i in rng.choice(k, 2, replace=False):
                self.present0[o * (k + m) + i] = 0
        self.payload = n * k * S
        self.alg_bytes = n * (k + m) * S  # hash 10 present + write 2 rebuilt
        self.kernel = "sha256_quad_kernel + rs_apply_fast<R=2>"
        self.name = ("RS reconstruct k=8 m=4, 2 data erasures + SHA-256 verify of the 10 present "
                     f"shards, chunk_size=1 MiB, {n} objects per GPU (BASELINE configs[2])")

    def step(self):
        pr = self.present0.copy()
        rc, _ = self.ctx.reconstruct_strided_device(
            self.k, self.m, self.S, self.n, self.obj.data_ptr(), (self.k + self.m) * self.S, self.S,
            pr, expected_ptr=self.dig.data_ptr(), stream=self.sh)
        assert rc == 0, f"reconstruct rc={rc}: {self.ctx.last_error() if hasattr(self.ctx, 'last_error') else ''}"

    def spot_check(self):
        return bool(self.torch.equal(self.obj[self.spot], self.ref))

    def cpu_work(self):
        import numpy as np

        oracle = _oracle()
        k, m, S = self.k, self.m, self.S
        rng = np.random.default_rng(SEED)
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        parity, dig, _ = oracle.compute_parity(data, m, S)
        shards = [d.tobytes() for d in data] + [p.tobytes() for p in parity]
        shards[1] = shards[5] = None
        sizes = [S] * (k + m)
        ni = oracle.have_sha_ni()
        self.cpu_sha_ni = ni
        return (lambda i: oracle.try_reconstruct_data_chunk(shards, k, m, S, dig, sizes, 1, sha_ni=True)), k * S, (
            f"try_reconstruct_data_chunk restated (oracle): SHA-256 ({'SHA-NI, as sha2 0.10.9 selects' if ni else 'scalar: no SHA-NI on this host'}) "
            "of the 10 present 1 MiB shards + crate reconstruct (64 KiB MUL_TABLE) of 2, per object")

    def drop(self):
        del self.obj, self.dig, self.ref


class ReconstructStream:
    """configs[2] as a continuous GET stream: W workers (host threads, as
    MaxIO's tokio workers) each own an 8192-chunk batch and a HIP stream and
    call mxec_reconstruct_strided_device concurrently through the one
    context; a step is one batch per worker.  The SHA-256 verify of a batch
    is a per-message latency chain (~1.2 us per 64-byte block in the quad
    form: ~20 ms per 1 MiB shard) that leaves most SIMDs' issue slots idle, so
    batches in flight side by side are what fills the chip."""

    bound = "valu"
    wall_timed = True

    def __init__(self, torch, ctx, dev, sh, n, workers, seed):
        from concurrent.futures import ThreadPoolExecutor

        self.torch = torch
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(workers)]
        self.parts = [Reconstruct(torch, ctx, dev, st.cuda_stream, n, seed + 97 * i)
                      for i, st in enumerate(self.streams)]
        self.pool = ThreadPoolExecutor(workers)
        self.k, self.m, self.S, self.n = 8, 4, 1 << 20, n * workers
        self.payload = sum(p.payload for p in self.parts)
        self.alg_bytes = sum(p.alg_bytes for p in self.parts)
        self.kernel = "sha256_stream_kernel (combined) / sha256_quad_kernel + rs_apply_fast<R=2>, W streams"
        self.lat = []
        self.name = (f"RS reconstruct k=8 m=4, 2 data erasures + SHA-256 verify, chunk_size=1 MiB: "
                     f"{workers} concurrent batches of {n} objects (8192-chunk batches, BASELINE "
                     "configs[2]) per GPU, one host thread + HIP stream each")

    def _one(self, part):
        t = time.perf_counter()
        part.step()
        self.lat.append(time.perf_counter() - t)

    def step(self):
        for f in [self.pool.submit(self._one, p) for p in self.parts]:
            f.result()

    def breakdown(self):
        lat = sorted(self.lat)
        st = self.parts[0].ctx.combiner_stats()
        return {"workers": len(self.parts),
                "batch_call_ms_median": round(1e3 * lat[len(lat) // 2], 2) if lat else None,
                "combiner_launches": st["batches"], "combiner_messages": st["messages"],
                "messages_per_launch": round(st["messages"] / max(1, st["batches"]), 1),
                "what": "host-side duration of one worker's reconstruct call (verify kernel + "
                        "readback + decode enqueue); SHA-256 launches of the device's combiner since "
                        "the context opened"}

    def spot_check(self):
        return all(p.spot_check() for p in self.parts)

    def cpu_work(self):
        spec = self.parts[0].cpu_work()
        self.cpu_sha_ni = self.parts[0].cpu_sha_ni
        return spec

    def drop(self):
        self.pool.shutdown()
        for p in self.parts:
            p.drop()


class Mixed:
    """configs[4]: mixed (k, m) and chunk sizes with short last chunks;
    a step encodes the batch and reconstructs it with seeded erasures.

    The 15 (k, m, S) classes are independent, as concurrent requests of a
    server are: class i runs on stream i mod `streams` (encode then
    reconstruct, in order on that stream), and the bench's stream waits for
    all of them, so its HIP events still bracket the whole step.  One stream
    serialises ~65 launches per step with an idle gap and a drain tail each
    (the smallest run 40-100 us)."""

    bound = "hbm"

    def __init__(self, torch, ctx, dev, sh, budget, seed, streams=4, mode="streams"):
        import ctypes

        import numpy as np

        self.torch, self.ctx, self.sh = torch, ctx, sh
        self.mode = mode
        self.main = torch.cuda.ExternalStream(sh, device=dev)
        self.streams = [self.main] if streams <= 1 or mode == "batch" else \
            [torch.cuda.Stream(device=dev) for _ in range(streams)]
        rng = np.random.default_rng(seed)
        kms = [(4, 2), (8, 4), (10, 4)]
        sizes = [64 << 10, 256 << 10, 1 << 20, 4 << 20, 10 << 20]
        self.classes = []  # (k, m, S, n, tensor, data_len, present0)
        per = budget // (len(kms) * len(sizes))
        payload = alg = 0
        for (k, m) in kms:
            for S in sizes:
                n = max(1, per // ((k + m) * S))
                t = torch.randint(0, 256, (n, k + m, S), dtype=torch.uint8, device=dev)
                last = int(rng.integers(1, S))  # short last chunk, zero padded
                dl = [S] * (k - 1) + [last]
                pres = np.ones(n * (k + m), np.uint8)
                lens = dl + [S] * m
                # Algorithmic bytes, exactly: the encode reads the k data
                # chunks (the last one short) and writes m parity; the
                # reconstruct reads the first k present shards and writes the
                # e missing ones (1 <= e <= m).
                alg += n * (sum(dl) + m * S)
                for o in range(n):
                    miss = rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False)
                    for i in miss:
                        pres[o * (k + m) + i] = 0
                    row = pres[o * (k + m): (o + 1) * (k + m)]
                    used = [i for i in range(k + m) if row[i]][:k]
                    alg += sum(lens[i] for i in used) + sum(lens[i] for i in miss)
                self.classes.append((k, m, S, n, t, dl, pres))
                payload += n * ((k - 1) * S + last) * 2  # encoded + decoded
        self.payload, self.alg_bytes = payload, alg
        self.kernel = "rs_apply_fast (mixed R) + edge tiles"
        self.name = ("mixed 4+2 / 8+4 / 10+4 at 64 KiB-10 MiB chunks, short last chunks: encode then "
                     f"reconstruct (1..m erasures), {sum(c[3] for c in self.classes)} objects per GPU "
                     "(BASELINE configs[4], per GPU)")
        if mode == "batch":
            # Every object of every class in ONE mxec_encode_batch_device and
            # ONE mxec_reconstruct_batch_device call per step (grouped launches:
            # one per m, one per erasure count), arrays built once.
            from maxio_amd import _native as N

            objs, dptr, pptr, dlen, sptr, slen, pres = [], [], [], [], [], [], []
            for (k, m, S, n, t, dl, pr) in self.classes:
                base, ss, os_ = t.data_ptr(), S, (k + m) * S
                for o in range(n):
                    objs.append(N.Object(k, m, S))
                    dptr += [base + o * os_ + j * ss for j in range(k)]
                    pptr += [base + o * os_ + (k + i) * ss for i in range(m)]
                    dlen += dl
                    sptr += [base + o * os_ + i * ss for i in range(k + m)]
                    slen += dl + [S] * m
                pres.append(pr)
            self.b_objs = (N.Object * len(objs))(*objs)
            self.b_dptr = (ctypes.c_void_p * len(dptr))(*dptr)
            self.b_pptr = (ctypes.c_void_p * len(pptr))(*pptr)
            self.b_dlen = (ctypes.c_uint64 * len(dlen))(*dlen)
            self.b_sptr = (ctypes.c_void_p * len(sptr))(*sptr)
            self.b_slen = (ctypes.c_uint64 * len(slen))(*slen)
            self.b_pres = np.concatenate(pres)
            self.kernel = "rs_apply_fast grouped (one launch per m, one per erasure count)"
            self.name += "; one encode + one reconstruct call per step (mixed-shape batches)"

    def step(self):
        if self.mode == "batch":
            self.ctx.encode_batch_device(self.b_objs, self.b_dptr, self.b_pptr, data_len=self.b_dlen,
                                         stream=self.sh)
            pr = self.b_pres.copy()
            rc, _ = self.ctx.reconstruct_batch_device(self.b_objs, self.b_sptr, pr, shard_len=self.b_slen,
                                                      stream=self.sh)
            assert rc == 0
            return
        ns = len(self.streams)
        for st in self.streams:
            if st is not self.main:
                st.wait_stream(self.main)
        for c, (k, m, S, n, t, dl, pres) in enumerate(self.classes):
            self.ctx.encode_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, t[:, k:].data_ptr(),
                                           (k + m) * S, S, data_len=dl, stream=self.streams[c % ns].cuda_stream)
        for c, (k, m, S, n, t, dl, pres) in enumerate(self.classes):
            pr = pres.copy()
            rc, _ = self.ctx.reconstruct_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, pr,
                                                        shard_len=dl + [S] * m,
                                                        stream=self.streams[c % ns].cuda_stream)
            assert rc == 0
        for st in self.streams:
            if st is not self.main:
                self.main.wait_stream(st)

    def spot_check(self):
        """The last object of every class after the steps: its parity equals
        the oracle's encode of its (short-last-chunk) data."""
        import numpy as np

        oracle = _oracle()
        for (k, m, S, n, t, dl, pres) in self.classes:
            h = t[n - 1].cpu().numpy()
            want = oracle.encode([h[j][:dl[j]] for j in range(k)], m, S)
            if not all(np.array_equal(h[k + i], want[i]) for i in range(m)):
                return False
        return True

    def cpu_work(self):
        return None

    def drop(self):
        del self.classes


class BodySums:
    """the PUT body digests of a batch of device-resident
    bodies — MD5 (the ETag, every PUT) + CRC32C (x-amz-checksum-crc32c) —
    in one call (filesystem.rs:700-725, 775-777)."""

    bound = "hbm"

    def __init__(self, torch, ctx, dev, sh, n, size, seed):
        self.torch, self.ctx, self.sh = torch, ctx, sh
        self.n, self.size = n, size
        g = torch.Generator(device=dev).manual_seed(seed)
        self.buf = torch.empty((n, size), dtype=torch.uint8, device=dev)
        for o in range(n):
            self.buf[o].copy_(torch.randint(0, 256, (size,), dtype=torch.uint8, device=dev, generator=g))
        self.out = torch.zeros((n, 76), dtype=torch.uint8, device=dev)
        self.ptrs = [self.buf[o].data_ptr() for o in range(n)]
        self.lens = [size] * n
        self.payload = n * size
        self.alg_bytes = n * size  # the CRC pass reads every body byte once
        self.which = 0x01 | 0x04
        self.kernel = "crc_tiles_kernel (CRC32C) + body_hash_kernel (MD5, lane per body)"
        self.name = (f"PUT body digests MD5 + CRC32C of {n} device-resident bodies x {size} B "
                     "(SURVEY 8f rank 3)")

    def step(self):
        self.ctx.body_sums_device(self.ptrs, self.lens, self.out.data_ptr(), self.which, stream=self.sh)

    def breakdown(self):
        """Each half alone, HIP-event timed on the same stream."""
        torch = self.torch
        res = {}
        for name, which in (("crc32c", 0x04), ("md5", 0x01), ("crc32", 0x02), ("sha1", 0x08)):
            self.ctx.body_sums_device(self.ptrs, self.lens, self.out.data_ptr(), which, stream=self.sh)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st = torch.cuda.ExternalStream(self.sh)
            a.record(st)
            self.ctx.body_sums_device(self.ptrs, self.lens, self.out.data_ptr(), which, stream=self.sh)
            b.record(st)
            torch.cuda.synchronize()
            ms = a.elapsed_time(b)
            d = {"ms": round(ms, 3)}
            if name.startswith("crc"):
                d["GBps"] = round(self.payload / (ms * 1e-3) / 1e9, 1)
                d["frac_of_8TBps"] = round(self.payload / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
            else:
                d["us_per_block"] = round(ms * 1e3 / (self.size / 64), 4)
            res[name] = d
        return res

    def spot_check(self):
        import hashlib

        oracle = _oracle()
        body = self.buf[0].cpu().numpy().tobytes()
        rec = self.out[0].cpu().numpy()
        return (rec[0:16].tobytes() == hashlib.md5(body).digest()
                and int.from_bytes(rec[20:24].tobytes(), "little") == oracle.crc32c(body, fast=True))

    def cpu_work(self):
        import hashlib

        import numpy as np

        oracle = _oracle()
        body = np.random.default_rng(SEED).integers(0, 256, self.size, dtype=np.uint8).tobytes()

        def work(i):
            hashlib.md5(body).digest()
            oracle.crc32c(body, fast=True)

        return work, self.size, ("hashlib.md5 (OpenSSL, as the md-5 crate) + CRC32C with SSE4.2 "
                                 "(the crc32c crate's hardware path) over one body per call")

    def drop(self):
        del self.buf, self.out


class Frames:
    """encrypt-then-EC — AES-256-GCM frame encryption
    (crypto.rs FrameEncryptor, 64 KiB frames, 32-byte per-frame AADs) of a
    batch of device-resident object bodies, one launch per step."""

    bound = "valu"

    def __init__(self, torch, ctx, dev, sh, n, size, seed):
        import numpy as np

        self.torch, self.ctx, self.sh = torch, ctx, sh
        self.n, self.size = n, size
        g = torch.Generator(device=dev).manual_seed(seed)
        self.pt = torch.randint(0, 256, (n, size), dtype=torch.uint8, device=dev, generator=g)
        fl = size + 28 * ((size + 65535) // 65536)
        self.fr = torch.zeros((n, fl), dtype=torch.uint8, device=dev)
        self.back = torch.zeros((n, size), dtype=torch.uint8, device=dev)
        nfr = (size + 65535) // 65536
        rng = np.random.default_rng(seed)
        self.keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(n)]
        aad = rng.integers(0, 256, (n, nfr, 32), dtype=np.uint8)
        self.aad = torch.from_numpy(aad).to(dev)
        self.jobs = [{"key": self.keys[o], "nonce_prefix": bytes([o & 255, 1, 2, 3]),
                      "aad_dev": self.aad[o].data_ptr(), "aad_len": 32,
                      "in_dev": self.pt[o].data_ptr(), "len": size, "out_dev": self.fr[o].data_ptr()}
                     for o in range(n)]
        self.djobs = [dict(j, in_dev=self.fr[o].data_ptr(), out_dev=self.back[o].data_ptr())
                      for o, j in enumerate(self.jobs)]
        self.payload = n * size
        self.alg_bytes = n * (size + fl)  # read plaintext, write frames
        self.kernel = "gcm_frames_kernel<encrypt> (T-table AES-256 + GHASH)"
        self.name = (f"encrypt-then-EC: AES-256-GCM 64 KiB frames of {n} device-resident bodies x {size} B, "
                     "32-byte AAD per frame (SURVEY 8f rank 4)")

    def step(self):
        self.ctx.frames_device(self.jobs, stream=self.sh)

    def breakdown(self):
        torch = self.torch
        st = torch.cuda.ExternalStream(self.sh)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        self.ctx.frames_device(self.djobs, decrypt=True, stream=self.sh)  # warm (first-call setup)
        a.record(st)
        status = self.ctx.frames_device(self.djobs, decrypt=True, stream=self.sh)
        b.record(st)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b)
        ok = all(s == 0 for s in status) and bool(torch.equal(self.back[0], self.pt[0]))
        return {"decrypt": {"ms_incl_status_readback": round(ms, 3),
                            "GiBps": round(self.payload / (ms * 1e-3) / GIB, 2), "round_trip_ok": ok}}

    def spot_check(self):
        oracle = _oracle()
        o = 1 if self.n > 1 else 0
        want = oracle.frames_encrypt(self.keys[o], self.jobs[o]["nonce_prefix"], self.pt[o].cpu().numpy(),
                                     [bytes(x) for x in self.aad[o].cpu().numpy()])
        return self.fr[o].cpu().numpy().tobytes() == want

    def cpu_work(self):
        import numpy as np

        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import openssl_gcm  # baseline only: OpenSSL EVP (AES-NI + PCLMUL), as the aes-gcm crate

        fn = openssl_gcm.frames_encrypt_fn()
        if fn is None:
            return None
        body = np.random.default_rng(SEED).integers(0, 256, self.size, dtype=np.uint8)
        key, pre, aad = np.zeros(32, np.uint8), np.frombuffer(b"abcd", np.uint8), np.full(32, 65, np.uint8)
        fl = self.size + 28 * ((self.size + 65535) // 65536)
        outs = {}

        def work(i):
            out = outs.setdefault(i, np.zeros(fl, np.uint8))  # one output buffer per thread
            fn(key.ctypes.data, pre.ctypes.data, aad.ctypes.data, 32, 65536, body.ctypes.data, body.size,
               out.ctypes.data)

        return work, self.size, ("OpenSSL EVP_aes_256_gcm over 64 KiB frames with 32-byte AADs (AES-NI/PCLMUL, "
                                 "as the aes-gcm crate), C loop, one body per call")

    def drop(self):
        del self.pt, self.fr, self.back, self.aad


def make_workload(cfg, torch, ctx, dev, sh, n_objects, rank, workers=8):
    seed = SEED + rank
    if cfg == "2":
        n = n_objects or 1024
        return Encode(torch, ctx, dev, sh, 4, 2, 10 << 20, n,
                      f"RS encode k=4 m=2, chunk_size=10485760 B, {n} objects per GPU, device-resident "
                      "(BASELINE configs[1])", seed, int(os.environ.get("BENCH_ENCODE_STREAMS", "1")))
    if cfg == "3":
        return Reconstruct(torch, ctx, dev, sh, n_objects or 1024, seed)
    if cfg == "3c":
        return ReconstructStream(torch, ctx, dev, sh, n_objects or 1024, workers, seed)
    if cfg == "ns":
        n = n_objects or 4096
        return Encode(torch, ctx, dev, sh, 8, 4, 1 << 20, n,
                      f"RS encode k=8 m=4, chunk_size=1 MiB (8 MiB objects), {n} objects per GPU "
                      "(north_star target shape)", seed)
    if cfg == "4a":
        n = n_objects or 4096
        return Encode(torch, ctx, dev, sh, 10, 4, 1 << 20, n,
                      f"RS encode k=10 m=4, chunk_size=1 MiB (10 MiB objects), {n} objects per GPU "
                      "(BASELINE configs[3], primary reading)", seed)
    if cfg == "4b":
        n = n_objects or 640
        return Encode(torch, ctx, dev, sh, 64, 4, 1 << 20, n,
                      f"RS encode k=64 m=4, chunk_size=1 MiB (literal 64 MiB objects), {n} objects per "
                      "GPU (BASELINE configs[3], literal reading)", seed)
    if cfg == "5":
        return Mixed(torch, ctx, dev, sh, 24 << 30, seed, int(os.environ.get("BENCH_MIXED_STREAMS", "4")),
                     os.environ.get("BENCH_MIXED_MODE", "batch"))
    if cfg == "sums":
        return BodySums(torch, ctx, dev, sh, n_objects or 1024, 40 << 20, seed)
    if cfg == "frames":
        return Frames(torch, ctx, dev, sh, n_objects or 256, 40 << 20, seed)
    raise SystemExit(f"unknown --config {cfg}")


def spot_objects(n: int, tiles_per_obj: int, grid: int) -> list:
    """Objects a spot check compares: the first, middle and last, and those
    either side of every grid-stride iteration boundary (tile = grid * i)."""
    s = {0, n // 2, n - 1}
    b = grid
    while b < tiles_per_obj * n:
        o = b // tiles_per_obj
        s.update({max(o - 1, 0), o, min(o + 1, n - 1)})
        b += grid
    return sorted(s)


def rs_blocks_per_cu(r_total: int) -> int:
    """Workgroups per CU of a uniform RS launch with r_total output rows --
    mirrors rs_default_variant (maxio_amd/csrc/rs_kernel.hip; a CPU test
    keeps the two in step)."""
    return 1024 if r_total <= 2 else 512


# Grouped (mixed-batch) launches: rs_group_variant's workgroups per CU.
RS_GROUP_BLOCKS_PER_CU = 512


def pmc_traffic(tag: str, alg_bytes: float, bpc=None):
    """Per-launch HBM bytes of the dominant kernel from the committed rocprofv3
    PMC summary (profiles/*pmc*<tag>*.json, FETCH_SIZE x2 per the gfx950
    correction + WRITE_SIZE; tools/pmc_summary.py): the measured
    traffic / algorithmic ratio applied to this launch's algorithmic bytes
    (the summary may come from a smaller batch of the same kernel).  With
    `bpc` (an RS launch's workgroups per CU) only a summary measured at the
    timed kernel's grid counts: its blocks_per_cu must equal it, else (older
    summaries without the field included) traffic is null."""
    want = bpc
    # newest round first (profiles/rNN_…)
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc*{tag}*.json")), reverse=True):
        try:
            with open(p) as f:
                d = json.load(f)
            if want is not None and d.get("blocks_per_cu") != want:
                continue
            ratio = d["hbm_bytes_per_launch"] / d["algorithmic_bytes_per_launch"]
            return round(ratio * alg_bytes, 0), os.path.relpath(p, ROOT)
        except Exception:
            continue
    return None, None


def probe_lib():
    """libmaxio_probe.so: HBM calibration streams (same load/store forms as
    the RS kernel), bench-only."""
    import ctypes

    p = os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_probe.so")
    lib = ctypes.CDLL(p)
    for fn, args in (("mxprobe_copy", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
                     ("mxprobe_copy_float4", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
                     ("mxprobe_read2_write1", [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]),
                     ("mxprobe_read", [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
                     ("mxprobe_write", [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]),
                     ("mxprobe_rs_pattern", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]),
                     ("mxprobe_set_stream_wpc", [ctypes.c_int]),
                     ("mxprobe_rs_pattern_strided", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                     ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                                     ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                     ctypes.c_void_p]),
                     ("mxprobe_rs_float4_strided", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                    ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                    ctypes.c_void_p])):
        getattr(lib, fn).argtypes = args
        getattr(lib, fn).restype = ctypes.c_int
    return lib


def event_ms(torch, stream, fn, reps: int, warm: int = 1) -> float:
    """Average HIP-event time of fn() on `stream` after `warm` untimed calls
    (7 for RS launches: the grid tuner times launches 2-7 of a shape)."""
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    torch.cuda.synchronize()
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / reps


def calibrate(torch, dev, stream) -> dict:
    """This box's HBM rates for plain streams of the RS kernel's load/store
    forms (nt dwordx4, 4 loads in flight per lane, 16 WG/CU; the read also at
    the RS kernel's 512): the second
    denominator of SURVEY §8(d)."""
    lib = probe_lib()
    sh = stream.cuda_stream
    n = 2 << 30
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    c = torch.empty(n, dtype=torch.uint8, device=dev)
    a.random_(0, 256)
    b.random_(0, 256)
    sink = torch.zeros(16, dtype=torch.uint8, device=dev)
    out = {}

    def run(rc):
        assert rc == 0, rc

    ms = event_ms(torch, stream, lambda: run(lib.mxprobe_copy(c.data_ptr(), a.data_ptr(), n, sh)), 5)
    out["copy_GBps"] = round(2 * n / (ms * 1e-3) / 1e9, 1)
    # the guide's float4 copy (MI355X_MICROARCH.md: 6.29 TB/s), same buffers
    ms = event_ms(torch, stream, lambda: run(lib.mxprobe_copy_float4(c.data_ptr(), a.data_ptr(), n, sh)), 5)
    out["copy_float4_GBps"] = round(2 * n / (ms * 1e-3) / 1e9, 1)
    ms = event_ms(torch, stream, lambda: run(lib.mxprobe_read2_write1(c.data_ptr(), a.data_ptr(), b.data_ptr(), n, sh)), 5)
    out["read2_write1_GBps"] = round(3 * n / (ms * 1e-3) / 1e9, 1)
    ms = event_ms(torch, stream, lambda: run(lib.mxprobe_read(a.data_ptr(), n, sink.data_ptr(), sh)), 5)
    out["read_GBps"] = round(n / (ms * 1e-3) / 1e9, 1)
    # the read stream at the RS kernel's 512 WG per CU: the box's read
    # bandwidth that north_star's ">= 80 % of HBM read bandwidth" refers to
    run(lib.mxprobe_set_stream_wpc(512))
    ms = event_ms(torch, stream, lambda: run(lib.mxprobe_read(a.data_ptr(), n, sink.data_ptr(), sh)), 5)
    run(lib.mxprobe_set_stream_wpc(16))
    out["read_wpc512_GBps"] = round(n / (ms * 1e-3) / 1e9, 1)
    del a, b, c, sink
    torch.cuda.empty_cache()
    # The RS kernel's own access pattern (same tile, same loads in flight,
    # 512 WG per CU) with XOR for the GF math, at the two encode shapes.
    # In the bench's object-major layout ([n][k+m][S], Encode), 15 / 24 GiB:
    # a few GiB measured low (launch ramp and tail on a ~1 ms launch).
    for k, m, S, n in ((4, 2, 10 << 20, 256), (8, 4, 1 << 20, 2048)):
        whole = torch.empty((n, k + m, S), dtype=torch.uint8, device=dev)
        whole.random_(0, 256)
        st = (k + m) * S
        ms = event_ms(torch, stream, lambda: run(lib.mxprobe_rs_pattern_strided(
            whole.data_ptr(), whole[:, k:].data_ptr(), k, m, S, n, st, st, S, sh)), 5)
        out[f"rs_pattern_k{k}m{m}_GBps"] = round(n * (k + m) * S / (ms * 1e-3) / 1e9, 1)
        del whole
    out["what"] = ("libmaxio_probe.so streams, HIP-event timed, 5 launches each: copy / copy_float4 (the guide's "
                   "float4 copy: plain loads and stores, one element per lane) / read2_write1 / read over 2 GiB "
                   "buffers (nontemporal global_load_dwordx4, 4 loads in flight per lane, nontemporal stores, 16 WG "
                   "x 256 lanes per CU; read_wpc512: the read at 512); rs_pattern_kXmY = the RS kernel's tile and load "
                   "schedule with XOR for the GF math, 512 WG per CU, over 15 GiB (k=4 m=2, 10 MiB) / 24 GiB (k=8 m=4, 1 MiB) in the "
                   "object-major [n][k+m][S] layout the Encode workloads use")
    torch.cuda.empty_cache()
    return out


def pattern_on_buffers(torch, stream, w) -> float:
    """The RS-pattern probe (the kernel's tile and load schedule, XOR for the
    GF math) over an Encode workload's own data / parity buffers: the same
    physical placement, so the ratio to it is the kernel's, not the
    allocation's.  Overwrites the parity (after the timed steps
    and the spot check)."""
    lib = probe_lib()
    k, m, S, n = w.k, w.m, w.S, w.n
    if k % 4 or m not in (1, 2, 4) or S % 16384:
        return None
    ms = event_ms(torch, stream, lambda: lib.mxprobe_rs_pattern_strided(
        w.data.data_ptr(), w.parity.data_ptr(), k, m, S, n, w.stride, w.pstride, w.sstride, stream.cuda_stream), 5)
    return round(n * (k + m) * S / (ms * 1e-3) / 1e9, 1)


def float4_copy_on_buffers(torch, stream, w):
    """The guide's float4 copy (plain loads and stores, one 16-byte element
    per lane, MI355X_MICROARCH.md's 6.29 TB/s recipe) over an Encode
    workload's own allocation: the first half of its object-major buffer
    copied onto the second half.  A denominator that shares nothing with the
    RS kernel's schedule.  Overwrites the objects (after the timed steps and
    the spot check)."""
    lib = probe_lib()
    half = (w.obj.numel() // 2) & ~15
    if half < (1 << 20):
        return None
    src = w.obj.data_ptr()
    dst = src + half
    ms = event_ms(torch, stream, lambda: lib.mxprobe_copy_float4(dst, src, half, stream.cuda_stream), 5)
    return round(2 * half / (ms * 1e-3) / 1e9, 1)


def measured_clock(kernel: str, cfg: str):
    """The shader clock a kernel ran at, from the committed GRBM_GUI_ACTIVE
    pass (profiles/r*/clock/clock_<cfg>.json, tools/clock_summary.py; newest
    round first), or (None, None)."""
    # clock_<cfg>.json and clock_<cfg>_<what>.json (an earlier pass kept
    # for the kernels that no longer run in it), newest round first
    paths = glob.glob(os.path.join(ROOT, "profiles", "r*", "clock", f"clock_{cfg}.json")) + \
        glob.glob(os.path.join(ROOT, "profiles", "r*", "clock", f"clock_{cfg}_*.json"))
    for p in sorted(paths, reverse=True):
        try:
            with open(p) as f:
                ks = json.load(f)["kernels"]
            # template arguments aside (sha256_quad_kernel<true> is the quad form's)
            k = ks.get(kernel) or next(v for n, v in ks.items() if n.split("<")[0] == kernel)
            return float(k["clock_GHz_median"]), os.path.relpath(p, ROOT)
        except Exception:
            continue
    return None, None


def valu_bound_GBps(form: str, n_cus: int) -> float:
    """Hashed-bytes ceiling of the SHA-256 form when every SIMD issues INT32
    VALU at its measured rate: 64 B per block / lane-ops per block."""
    lane_ops = n_cus * 4 * VALU_LANES_PER_SIMD_CYCLE * CLOCK_GHZ * 1e9
    return lane_ops / SHA_VALU_PER_BLOCK[form] * 64 / 1e9


# RS decode (R = 2) VALU lane-ops per input byte, from PMC: config 2's
# rs_apply_fast<2,4,true> retires 2.84e9 wave-instructions x 64 lanes per
# launch over 42.9 GB of input (profiles/r2_pmc_valu.json).
RS_R2_VALU_PER_INPUT_BYTE = 4.24


def sha_chain_block(form: str, us_per_block: float):
    """Config 3's binding roofline: the serial chain of one message.  The
    form's consumer wave issues SHA_CONSUMER_VALU_PER_BLOCK VALU per block,
    one per 4 cycles, at the clock the chip held for this kernel
    (GRBM_GUI_ACTIVE pass) and at the 2.4 GHz maximum."""
    if form not in SHA_CONSUMER_VALU_PER_BLOCK:
        return None
    clk, src = measured_clock(f"sha256_{form}_kernel", "3")
    cyc = SHA_CONSUMER_VALU_PER_BLOCK[form] * 4
    d = {"bound": "valu-chain", "form": form, "consumer_valu_per_block": SHA_CONSUMER_VALU_PER_BLOCK[form],
         "cycles_per_valu": 4, "us_per_block": round(us_per_block, 4),
         "floor_us_per_block_at_2.4GHz": round(cyc / (CLOCK_GHZ * 1e3), 4),
         "frac_at_2.4GHz": round(cyc / (CLOCK_GHZ * 1e3) / us_per_block, 4)}
    if clk:
        d.update({"clock_GHz_measured": clk, "clock_source": src,
                  "floor_us_per_block": round(cyc / (clk * 1e3), 4),
                  "frac": round(cyc / (clk * 1e3) / us_per_block, 4)})
    # against the hardware rather than the form's own instruction count
    hz = (clk or CLOCK_GHZ) * 1e3
    hw = 64 * SHA_ROUND_DEP_CYCLES / hz
    d["hw_chain_floor"] = {
        "path": "per round: v_alignbit_b32 -> v_bitop3_b32 (XOR3) -> v_add3_u32, one wave's dependent latencies "
                "10.77 + 8.63 + 8.63 cycles (profiles/r1_lab_valu_issue.jsonl); 64 rounds per block",
        "cycles_per_block": round(64 * SHA_ROUND_DEP_CYCLES, 1), "clock_GHz": clk or CLOCK_GHZ,
        "floor_us_per_block": round(hw, 4), "frac": round(hw / us_per_block, 4)}
    return d


def config3_roofline(form: str, nmsg: int, sha_GBps: float, ms_sha: float, S: int, vb: float, vform: str,
                     n_cus: int) -> dict:
    """Config 3's hash launch against the bound that binds it.  A batch of
    up to 48 messages per CU (10 240 here) is one serial chain per message,
    so the floor is the chain: the form's consumer VALU per block at 4 cycles
    each, at the clock the chip held for this kernel (GRBM pass) when one is
    committed, else 2.4 GHz.  The chip-wide INT32-VALU bound of the one-lane
    SHA-256 (1470 lane-ops per block) stays beside it as `chip_valu`: it
    would bind only with enough messages to fill every SIMD."""
    us_block = ms_sha * 1e3 / (S / 64)
    chain = sha_chain_block(form, us_block)
    d = {"kernel": f"sha256_{form}_kernel (alone, {nmsg} x 1 MiB)", "unit": "GB/s hashed",
         "achieved": round(sha_GBps, 1), "ms_per_launch": round(ms_sha, 3), "us_per_block": round(us_block, 4),
         "frac_of_hbm": round(sha_GBps / HBM_PEAK_GBPS, 4),
         "chip_valu": {"bound": "valu", "peak": round(vb, 1), "frac": round(sha_GBps / vb, 4),
                       "valu_lane_ops_per_block": SHA_VALU_PER_BLOCK[vform],
                       "form_lane_ops_per_block": SHA_VALU_PER_BLOCK[form],
                       "valu_peak_lane_ops_per_s": n_cus * 4 * VALU_LANES_PER_SIMD_CYCLE * CLOCK_GHZ * 1e9}}
    if chain:
        # `frac` is against the hardware's chain floor (hw_chain_floor); the
        # form's own 4-cycle issue floor stays in chain.frac
        f = chain["hw_chain_floor"]["frac"]
        d.update({"bound": "valu-chain", "peak": round(sha_GBps / f, 1), "frac": f, "chain": chain})
    else:
        d.update({"bound": "valu", "peak": round(vb, 1), "frac": round(sha_GBps / vb, 4)})
    return d


def stream_step_roofline(ms: float, workers: int, n: int, n_cus: int) -> dict:
    """Config 3c's step against its bound.  The step hashes every present
    shard (one combined stream-form launch) and rebuilds 2 of 12 shards per
    object; the rebuild runs speculatively beside the hash (capi.cpp), so the
    two share the SIMDs: the bound is the larger of the step's INT32-VALU
    work (hash lane-ops per block x blocks + decode lane-ops per input byte x
    input bytes) at the chip's issue rate and its HBM traffic at 8 TB/s.
    frac_hash_only sets the step against the hash's VALU time alone."""
    S = float(1 << 20)
    hashed = workers * n * 10 * S
    dec_in = workers * n * 8 * S  # the decode reads 8 shards, writes 2
    traffic = hashed + workers * n * 10 * S
    lane_ops_s = n_cus * 4 * VALU_LANES_PER_SIMD_CYCLE * CLOCK_GHZ * 1e9
    hash_ms = hashed / 64 * SHA_VALU_PER_BLOCK["stream"] / lane_ops_s * 1e3
    dec_ms = dec_in * RS_R2_VALU_PER_INPUT_BYTE / lane_ops_s * 1e3
    hbm_ms = traffic / (HBM_PEAK_GBPS * 1e9) * 1e3
    bound_ms = max(hash_ms + dec_ms, hbm_ms)
    return {"bound": "valu", "kernel": "sha256_stream_kernel (combined) + rs_apply_fast<R=2> x workers beside it",
            "achieved_ms_per_step": round(ms, 2), "bound_ms_per_step": round(bound_ms, 2),
            "frac": round(bound_ms / ms, 4),
            "hash_valu_ms": round(hash_ms, 2), "decode_valu_ms": round(dec_ms, 2), "hbm_ms": round(hbm_ms, 2),
            "frac_hash_only": round(hash_ms / ms, 4),
            "hash_GBps_over_step": round(hashed / (ms * 1e-3) / 1e9, 1),
            "valu_lane_ops_per_block": SHA_VALU_PER_BLOCK["stream"],
            "decode_valu_lane_ops_per_input_byte": RS_R2_VALU_PER_INPUT_BYTE,
            "valu_peak_lane_ops_per_s": lane_ops_s,
            "what": (f"{workers} x {n} objects 8+4 x 1 MiB per step: {hashed / 1e9:.1f} GB hashed + "
                     f"{dec_in / 1e9:.1f} GB decoded on the INT32 VALU (the decode runs beside the hash), "
                     f"{traffic / 1e9:.1f} GB of HBM traffic")}


def hbm_block(alg_bytes: float, ms: float, kernel: str, cal: dict, ratio_key: str) -> dict:
    ach = alg_bytes / (ms * 1e-3) / 1e9
    d = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
         "frac": round(ach / HBM_PEAK_GBPS, 4), "kernel": kernel, "bytes_per_launch": float(alg_bytes),
         "ms_per_launch": round(ms, 4)}
    if cal and cal.get(ratio_key):
        d["box_stream_GBps"] = cal[ratio_key]
        d["frac_of_box_stream"] = round(ach / cal[ratio_key], 4)
        d["box_stream"] = ratio_key
    return d


def extras(ctx, torch, dev, stream, steps: int, cal: dict) -> dict:
    """Driver-timed secondary measurements beside the headline (VERDICT r1
    item 1), each with its own roofline block: the north-star shape (encode
    k=8 m=4, 1 MiB chunks), config 3 (verify + rebuild) with the SHA kernel
    timed alone against the INT32-VALU bound, config 5 (the mixed
    encode + reconstruct stream), config 3c (8 concurrent batches), and the
    reference-equivalent PUT compute (encode + SHA-256 of all k+m chunks)."""
    sh = stream.cuda_stream
    n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    out = {}
    # -- north star: encode k=8 m=4, 1 MiB, 4096 objects -------------------
    w = make_workload("ns", torch, ctx, dev, sh, 0, 0)
    torch.cuda.synchronize()
    ms = event_ms(torch, stream, w.step, max(5, steps // 2), warm=7)
    ok = w.spot_check()
    same = pattern_on_buffers(torch, stream, w)
    f4_ns = float4_copy_on_buffers(torch, stream, w)
    cal_ns = dict(cal or {}, rs_pattern_same_buffers_GBps=same)
    out["ns"] = {"workload": w.name, "GiBps_payload": round(w.payload / GIB / (ms * 1e-3), 3),
                 "spot_check_vs_oracle": ok,
                 "roofline": hbm_block(w.alg_bytes, ms, w.kernel, cal_ns,
                                       "rs_pattern_same_buffers_GBps" if same else "rs_pattern_k8m4_GBps")}
    ns_bpc = ctx.rs_grid(8, 4, 1 << 20)
    tr, src = pmc_traffic("k8m4", w.alg_bytes, ns_bpc)
    out["ns"]["roofline"]["blocks_per_cu"] = ns_bpc
    out["ns"]["roofline"]["traffic"], out["ns"]["roofline"]["traffic_source"] = tr, src
    if f4_ns:
        out["ns"]["roofline"]["float4_copy_GBps"] = f4_ns
        out["ns"]["roofline"]["frac_of_float4_copy"] = round(out["ns"]["roofline"]["achieved"] / f4_ns, 4)
    if cal and cal.get("read_wpc512_GBps"):  # north_star: >= 80 % of per-GPU HBM read bandwidth
        rd = max(cal["read_wpc512_GBps"], cal.get("read_GBps") or 0)
        out["ns"]["roofline"]["box_read_GBps"] = rd
        out["ns"]["roofline"]["frac_of_box_read"] = round(out["ns"]["roofline"]["achieved"] / rd, 4)
    w.drop()
    del w
    torch.cuda.empty_cache()
    # -- config 3: reconstruct 8+4, 2 erasures + verify, 1024 objects --------
    r = Reconstruct(torch, ctx, dev, sh, 1024, SEED)
    ms_call = event_ms(torch, stream, r.step, 5, warm=7)
    ok = r.spot_check()
    k, m, S, n = r.k, r.m, r.S, r.n
    present_ptrs, present_lens = [], []
    for o in range(n):
        for i in range(k + m):
            if r.present0[o * (k + m) + i]:
                present_ptrs.append(r.obj[o, i].data_ptr())
                present_lens.append(S)
    dig = torch.empty((len(present_ptrs), 32), dtype=torch.uint8, device=dev)
    ms_sha = event_ms(torch, stream, lambda: ctx.sha256_batch_device(present_ptrs, present_lens, dig.data_ptr(),
                                                                     stream=sh), 3)
    hashed = float(len(present_ptrs)) * S
    nmsg = len(present_ptrs)
    form = "quad" if nmsg <= SHA_QUAD_MSGS_PER_CU * n_cus else "split" if nmsg <= 49152 else "stream"
    sha_GBps = hashed / (ms_sha * 1e-3) / 1e9
    # chip-wide INT32 bound of the one-lane SHA-256 (the split form's count
    # for the latency forms): the same denominator whatever form ran
    vform = "split" if form == "quad" else form
    vb = valu_bound_GBps(vform, n_cus)
    # decode alone: the same erasures, no digests (RS over the 8 survivors -> 2)
    def decode_only():
        pr = r.present0.copy()
        rc, _ = ctx.reconstruct_strided_device(k, m, S, n, r.obj.data_ptr(), (k + m) * S, S, pr, stream=sh)
        assert rc == 0
    ms_rs = event_ms(torch, stream, decode_only, 3, warm=2)
    # its denominator: the RS pattern on the same buffers, 8 shards read and
    # 2 written per object (shards 0-7 -> 10-11; after the spot check)
    lib = probe_lib()
    ms_pat = event_ms(torch, stream, lambda: lib.mxprobe_rs_pattern_strided(
        r.obj.data_ptr(), r.obj[:, k + 2:].data_ptr(), k, 2, S, n, (k + m) * S, (k + m) * S, S, sh), 3)
    cal3 = dict(cal or {}, rs_pattern_same_buffers_GBps=round(n * (k + 2) * S / (ms_pat * 1e-3) / 1e9, 1))
    out["config3"] = {
        "workload": r.name, "GiBps_payload": round(r.payload / GIB / (ms_call * 1e-3), 3),
        "ms_per_call": round(ms_call, 3), "spot_check_vs_original": ok,
        "roofline": config3_roofline(form, len(present_ptrs), sha_GBps, ms_sha, S, vb, vform, n_cus),
        "rs_decode": hbm_block(float(n) * (k + 2) * S, ms_rs, "rs_apply_fast<R=2> (decode 8 -> 2, no verify)",
                               cal3, "rs_pattern_same_buffers_GBps"),
    }
    # the reference's CPU path for the same work, 1 core and all cores
    # (SHA-NI as sha2 0.10.9 selects it on x86-64)
    work, per_call, what = r.cpu_work()
    v1, n1, el1 = cpu_leg(work, per_call, 4.0, 1)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 64)
    va, na, ela = cpu_leg(work, per_call, 3.0, threads)
    out["config3"]["cpu_baseline"] = {"value": round(v1, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                                      "sha_ni": r.cpu_sha_ni, "sample": f"{n1} calls in {el1:.1f}s: {what}"}
    out["config3"]["cpu_baseline_all_cores"] = {"value": round(va, 4), "unit": "GiB/s", "cores": threads,
                                                "kind": "port", "sha_ni": r.cpu_sha_ni,
                                                "sample": f"{na} calls in {ela:.1f}s on {threads} threads"}
    del dig
    r.drop()
    del r
    torch.cuda.empty_cache()
    # -- config 5: the mixed 4+2 / 8+4 / 10+4 stream, encode + reconstruct --
    w5 = make_workload("5", torch, ctx, dev, sh, 0, 0)
    torch.cuda.synchronize()
    ms5 = event_ms(torch, stream, w5.step, max(5, steps // 6))
    ok5 = w5.spot_check()
    out["config5"] = {"workload": w5.name, "GiBps_payload": round(w5.payload / GIB / (ms5 * 1e-3), 3),
                      "ms_per_step": round(ms5, 3), "spot_check_vs_oracle": ok5,
                      "roofline": hbm_block(w5.alg_bytes, ms5, w5.kernel + ", whole step", cal,
                                            "rs_pattern_k4m2_GBps")}
    tr, src = pmc_traffic("cfg5_grouped", w5.alg_bytes, RS_GROUP_BLOCKS_PER_CU)
    out["config5"]["roofline"]["traffic"], out["config5"]["roofline"]["traffic_source"] = tr, src
    w5.drop()
    del w5
    torch.cuda.empty_cache()
    # -- config 3c: 8 concurrent batches -----------------------------------
    rs = ReconstructStream(torch, ctx, dev, sh, 1024, 8, SEED)
    torch.cuda.synchronize()
    for _ in range(4):  # the first steps gather and place unevenly (the combiner adapts to 8 callers)
        rs.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 6
    for _ in range(reps):
        rs.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    out["config3c"] = {"workload": rs.name, "GiBps_payload": round(rs.payload / GIB / (ms * 1e-3), 3),
                       "ms_per_step": round(ms, 2), "spot_check_vs_original": rs.spot_check(),
                       "roofline": stream_step_roofline(ms, 8, 1024, n_cus),
                       "breakdown": rs.breakdown()}
    rs.drop()
    del rs
    torch.cuda.empty_cache()
    # -- config 2 with caller-owned separate data / parity buffers -----------
    w = Encode(torch, ctx, dev, sh, 4, 2, 10 << 20, 1024,
               "RS encode k=4 m=2, 10 MiB chunks, 1024 objects, data [n][k][S] and parity [n][m][S] as two "
               "allocations (no pad)", SEED + 3, separate=True)
    torch.cuda.synchronize()
    ms = event_ms(torch, stream, w.step, max(5, steps // 4), warm=7)
    ok = w.spot_check()
    same = pattern_on_buffers(torch, stream, w)
    f4 = float4_copy_on_buffers(torch, stream, w)  # over the data allocation
    blk = hbm_block(w.alg_bytes, ms, w.kernel, dict(cal or {}, rs_pattern_same_buffers_GBps=same),
                    "rs_pattern_same_buffers_GBps")
    if f4:
        blk["float4_copy_data_buffer_GBps"] = f4
        blk["frac_of_float4_copy"] = round(blk["achieved"] / f4, 4)
    out["config2_separate_buffers"] = {"workload": w.name, "GiBps_payload": round(w.payload / GIB / (ms * 1e-3), 3),
                                       "spot_check_vs_oracle": ok, "roofline": blk}
    w.drop()
    del w
    torch.cuda.empty_cache()
    # -- PUT compute: encode + SHA-256 of all k+m chunks, config 2 shape -----
    w = make_workload("2", torch, ctx, dev, sh, 256, 0)
    kk, mm, SS, nn = w.k, w.m, w.S, w.n
    dig = torch.empty((nn, kk + mm, 32), dtype=torch.uint8, device=dev)
    ms = event_ms(torch, stream, lambda: ctx.encode_strided_device(
        kk, mm, SS, nn, w.data.data_ptr(), w.stride, w.sstride, w.parity.data_ptr(), w.pstride, w.sstride,
        digests_ptr=dig.data_ptr(), stream=sh), 2)
    out["put_path_encode_plus_sha256"] = {
        "GiBps_payload": round(nn * kk * SS / GIB / (ms * 1e-3), 3), "ms": round(ms, 2),
        "what": (f"RS encode + SHA-256 of every data and parity chunk, {nn} x 4+2 x 10 MiB (write_chunk + "
                 "compute_and_write_parity compute); bound by one 10 MiB chunk's SHA chain (163 840 blocks)")}
    del dig
    w.drop()
    del w
    torch.cuda.empty_cache()
    return out


# ---- device plan ----------------------------------------------------------------


class BenchRefusal(Exception):
    """bench.py cannot measure what was asked (exit status 2, no JSON line)."""


class Plan:
    """Which GPUs this process drives and what the JSON line reports.

    mode  "single"   --gpus 1, one device
          "devices"  --gpus N > 1 in ONE process: one mxec_ctx over N devices
                     (MaxIO's production shape), object i -> device i mod N,
                     each device's launches on its own stream and host thread
          "ranks"    under torch.distributed.run: WORLD_SIZE ranks, one GPU
                     each (LOCAL_RANK), --gpus must equal WORLD_SIZE
          "logical"  BENCH_REHEARSE_LOGICAL=1 and fewer visible GPUs than
                     --gpus: a labelled rehearsal on N logical devices of one
                     card (mxec_open_test logical_devices), never an N-GPU number
    """

    def __init__(self, mode, n_gpus, torch_devs, world=1, rank=0, logical=1, rehearsal=None):
        self.mode, self.n_gpus, self.torch_devs = mode, n_gpus, list(torch_devs)
        self.world, self.rank, self.logical, self.rehearsal = world, rank, logical, rehearsal

    @property
    def local_devices(self) -> int:
        return len(self.torch_devs)

    @property
    def device_mask(self) -> int:
        m = 0
        for d in self.torch_devs:
            m |= 1 << d
        return m


def plan_devices(gpus: int, env, visible: int) -> Plan:
    """The device plan for `bench.py --gpus N`, or BenchRefusal.  A line's
    n_gpus always equals --gpus; a run that cannot drive that many GPUs exits
    non-zero instead of printing a smaller measurement."""
    if gpus < 1:
        raise BenchRefusal(f"--gpus {gpus}: need at least one GPU")
    world = int(env.get("WORLD_SIZE", "1"))
    if world > 1:
        rank = int(env.get("RANK", "0"))
        if gpus != world:
            raise BenchRefusal(f"--gpus {gpus} but WORLD_SIZE={world}: under torch.distributed.run each rank "
                               "drives one GPU, so --gpus must equal --nproc-per-node")
        pinned = env.get("BENCH_GPU_OF_RANK")
        gpu = int(pinned if pinned is not None else env.get("LOCAL_RANK", "0"))
        if not 0 <= gpu < visible:
            raise BenchRefusal(f"rank {rank} wants GPU {gpu} but {visible} HIP device(s) are visible")
        reh = (f"BENCH_GPU_OF_RANK={pinned}: every rank on GPU {pinned} (rehearsal of the rank path, "
               "not an N-GPU measurement)") if pinned is not None else None
        return Plan("ranks", world, [gpu], world=world, rank=rank, rehearsal=reh)
    if gpus <= visible:
        return Plan("single" if gpus == 1 else "devices", gpus, range(gpus))
    if env.get("BENCH_REHEARSE_LOGICAL") == "1" and visible >= 1:
        if gpus > 8:
            raise BenchRefusal(f"--gpus {gpus}: logical rehearsals go up to 8 devices")
        return Plan("logical", gpus, [0] * gpus, logical=gpus,
                    rehearsal=(f"{gpus} logical devices of ONE card (mxec_open_test logical_devices={gpus}): "
                               "exercises the multi-device path, not an N-GPU measurement"))
    raise BenchRefusal(f"--gpus {gpus} asks for {gpus} GPUs but {visible} HIP device(s) are visible; run it on a "
                       f"node with {gpus} GPUs (or set BENCH_REHEARSE_LOGICAL=1 for a labelled rehearsal on "
                       "logical devices of one card)")


class DevView:
    """The context bound to one of its devices: every *_device call (and
    combiner_stats) goes to ctx device `di`."""

    _DEV_CALLS = frozenset((
        "rs_grid", "encode_strided_device", "encode_batch_device", "reconstruct_strided_device",
        "reconstruct_strided_device_async", "reconstruct_batch_device", "reconstruct_batch_device_async",
        "sha256_batch_device", "body_sums_device", "frames_device", "combiner_stats", "batch_alloc"))

    def __init__(self, ctx, di: int):
        self._ctx, self.di = ctx, di

    def __getattr__(self, name):
        a = getattr(self._ctx, name)
        if name in self._DEV_CALLS:
            import functools

            return functools.partial(a, dev=self.di)
        return a


def reduce_sum(value: float) -> float:
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return value
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_objects(obj) -> list:
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def sync_all(torch, devs) -> None:
    for d in sorted(set(devs)):
        torch.cuda.synchronize(d)


def tune_before_timing(torch, lanes, devs, max_launches: int = 12) -> dict:
    """Run the workload until the library's RS grid tuner has decided, before
    the warmup and the timed steps.  The tuner times launches 2-7 of a large
    uniform shape at three grids and keeps the fastest (ops.cpp
    rs_grid_pick); without this, a short --warmup would leave its trial
    launches (half and quarter grids) inside the timed region.  Each launch
    is waited on, so the trials' events complete and the next call reads
    them.  Workloads without one large uniform shape run 7 launches (their
    tuner shapes, if any, see as many)."""
    t0 = time.perf_counter()
    n = 0
    decided = True
    grid = None
    for w, stream, tdev in lanes:
        shape = (w.k, w.m, w.S) if isinstance(w, Encode) else None
        with torch.cuda.device(tdev):
            for i in range(max_launches):
                if shape is not None and i > 0 and w.ctx.rs_grid(*shape):
                    break
                if shape is None and i >= 7:
                    break
                w.step()
                torch.cuda.synchronize(tdev)
                n += 1
        if shape is not None:
            g = w.ctx.rs_grid(*shape)
            decided = decided and g > 0
            grid = g if grid is None else grid
    sync_all(torch, devs)
    return {"decided": decided, "launches": n, "grid_before_timing": grid,
            "seconds": round(time.perf_counter() - t0, 3),
            "what": "launches run before --warmup until the RS grid tuner decided (one sync each)"}


def run_steps(torch, lanes, steps: int, events: bool):
    """`steps` steps of every lane (device): one host thread per device when
    there are several, so each device's queue is fed independently (every
    call returns after enqueueing, except the reconstructs that read back
    verdicts).  Returns per-lane HIP event pairs bracketing each step on the
    lane's stream."""

    def one(lane):
        w, stream, tdev = lane
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)] if events else []
        with torch.cuda.device(tdev):
            for i in range(steps):
                if events:
                    ev[i][0].record(stream)
                w.step()
                if events:
                    ev[i][1].record(stream)
        return ev

    if len(lanes) == 1:
        return [one(lanes[0])]
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(len(lanes)) as ex:
        return list(ex.map(one, lanes))


# ---- end-to-end host leg (north_star: PCIe-inclusive rate) -----------------------


def _fill_random(buf, seed: int) -> None:
    """Random bytes without generating gigabytes of randomness: tile a 64 MiB block."""
    import numpy as np

    blk = np.random.default_rng(seed).integers(0, 256, 64 << 20, dtype=np.uint8)
    flat = buf.reshape(-1)
    for o in range(0, flat.size, blk.size):
        n = min(blk.size, flat.size - o)
        flat[o:o + n] = blk[:n]


def pcie_rates(torch, devs, nbytes: int = 1 << 30) -> dict:
    """The box's raw copy rates between pinned host memory and the devices:
    every device at once (one pinned buffer and one stream each), each
    direction alone, 4 copies per device, wall clock."""
    barrier()  # every rank measures at the same time, as its batches will run
    hb = [torch.empty(nbytes, dtype=torch.uint8).pin_memory() for _ in devs]
    db = [torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", d)) for d in devs]
    st = [torch.cuda.Stream(device=torch.device("cuda", d)) for d in devs]
    out = {}
    for name in ("h2d", "d2h"):
        def go(reps):
            for _ in range(reps):
                for h, d, s in zip(hb, db, st):
                    with torch.cuda.stream(s):
                        (d.copy_(h, non_blocking=True) if name == "h2d" else h.copy_(d, non_blocking=True))
            sync_all(torch, devs)

        go(1)
        t0 = time.perf_counter()
        go(4)
        out[f"{name}_GBps"] = round(4 * nbytes * len(devs) / (time.perf_counter() - t0) / 1e9, 1)
    # Both directions at once in the PUT / GET legs' 2:1 byte ratio (4 shards
    # up, 2 down per object): two bytes up for every byte down, on separate
    # streams, every device together.  A PCIe link is full duplex, but the
    # DMA engines and host memory are shared, so this sets the legs' real
    # bound when it is below the one-way rates added together.
    hb2 = [torch.empty(nbytes, dtype=torch.uint8).pin_memory() for _ in devs]
    db2 = [torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", d)) for d in devs]
    st2 = [torch.cuda.Stream(device=torch.device("cuda", d)) for d in devs]

    def duplex(reps):
        for _ in range(reps):
            for h, d, h2, d2, s, s2 in zip(hb, db, hb2, db2, st, st2):
                with torch.cuda.stream(s):
                    d.copy_(h, non_blocking=True)
                    d.copy_(h, non_blocking=True)
                with torch.cuda.stream(s2):
                    h2.copy_(d2, non_blocking=True)
        sync_all(torch, devs)

    duplex(1)
    t0 = time.perf_counter()
    duplex(2)
    el = time.perf_counter() - t0
    out["duplex_2to1_up_GBps"] = round(4 * nbytes * len(devs) / el / 1e9, 1)
    out["duplex_2to1_down_GBps"] = round(2 * nbytes * len(devs) / el / 1e9, 1)
    del hb, db, hb2, db2
    return out


def numa_nodes(addr: int, nbytes: int, samples: int = 4) -> list:
    """NUMA node of `samples` pages spread over a host buffer
    (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR), -errno where it fails."""
    import ctypes

    libc = ctypes.CDLL("libc.so.6", use_errno=True)
    out = []
    for i in range(samples):
        node = ctypes.c_int(-1)
        rc = libc.syscall(239, ctypes.byref(node), None, ctypes.c_ulong(0),
                          ctypes.c_void_p(addr + nbytes // samples * i), ctypes.c_ulong(3))
        out.append(node.value if rc == 0 else -ctypes.get_errno())
    return out


def gpu_numa_node(torch, d: int):
    try:
        pr = torch.cuda.get_device_properties(d)
        bus = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
            return int(f.read())
    except Exception:
        return None


def _copy_delta(c0: list, c1: list) -> dict:
    """Host-pipeline counters (Context.pipe_stats, one dict per device)
    accumulated over a leg; sdma_last_mbps / sdma_down_last_mbps are gauges
    (the last timed upload / download bracket's SDMA rate), reported as the
    lowest over the devices."""
    gauges = ("sdma_last_mbps", "sdma_down_last_mbps")
    out = {key: sum(b[key] - a[key] for a, b in zip(c0, c1)) for key in c1[0] if key not in gauges}
    for g in gauges:
        out[g] = min(b.get(g, 0) for b in c1)
    return out


def _leg_times(ts: list) -> dict:
    """Every timed batch of a leg, its median (the reported rate) and max."""
    med = statistics.median(ts)
    return {"s_per_batch": round(med, 4), "s_max": round(max(ts), 4),
            "max_over_median": round(max(ts) / med, 3), "s_each": [round(t, 4) for t in ts]}


def e2e_put_large(ctx, n: int = 512, reps: int = 3) -> dict:
    """PUT with every chunk's SHA-256 from page-locked host memory at a
    large batch (one GPU): n x 4+2 x 10 MiB through mxec_encode_batch_host,
    where the upload (not one chunk's chain) is the bound and the per-wave
    piece size goes to 4 MiB (pipeline.cpp piece_bytes).  Median of `reps`
    batches after a warm one, next to the same batch without digests; one
    object's parity and digests checked against the oracle."""
    import hashlib

    import numpy as np

    k, m, S = 4, 2, 10 << 20
    data = ctx.host_array(n * k * S).reshape(n, k, S)
    par = ctx.host_array(n * m * S).reshape(n, m, S)
    _fill_random(data, 17)
    dptr = [data[o, j].ctypes.data for o in range(n) for j in range(k)]
    pptr = [par[o, i].ctypes.data for o in range(n) for i in range(m)]
    objs = [(k, m, S)] * n
    res = {"workload": f"PUT compute from page-locked host memory, {n} x 4+2 x 10 MiB per batch, one GPU"}
    for sha in (False, True):
        dig = np.zeros(n * (k + m) * 32, np.uint8) if sha else None
        ctx.encode_batch_host(objs, dptr, pptr, digests=dig)  # warm
        c0 = ctx.pipe_stats()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ctx.encode_batch_host(objs, dptr, pptr, digests=dig)
            ts.append(time.perf_counter() - t0)
        el = statistics.median(ts)
        c1 = ctx.pipe_stats()
        res["rs_sha256" if sha else "rs_only"] = dict(_leg_times(ts), GiBps_payload=round(n * k * S / GIB / el, 2),
                                                      copies=_copy_delta([c0], [c1]))
        if sha:
            o = n // 2
            want = _oracle().encode(list(data[o]), m, S)
            res["spot_check_vs_oracle"] = bool(
                all(np.array_equal(par[o, i], want[i]) for i in range(m)) and
                all(bytes(dig[(o * (k + m) + j) * 32:(o * (k + m) + j + 1) * 32]) ==
                    hashlib.sha256((data[o, j] if j < k else par[o, j - k]).tobytes()).digest()
                    for j in range(k + m)))
    ctx.host_free(data)
    ctx.host_free(par)
    del data, par
    return res


def e2e_host_leg(ctx, torch, plan: Plan, per_dev: int, reps: int = 5, get_only: bool = False) -> dict:
    """mxec_encode_batch_host from mxec_host_alloc (page-locked) memory: the
    PUT path as MaxIO sees it -- request bodies in host memory, parity and
    digests back in host memory (filesystem.rs:1107-1135) -- over every
    device of the context, with and without the SHA-256 of every chunk; then
    the GET side, mxec_reconstruct_batch_host over the same objects with two
    erasures each, without and with verification.
    Payload GiB/s (k * chunk_size per object) over all ranks at the median
    of `reps` timed batches (each batch's time and the max listed), next to
    the box's raw pinned copy rates and the bounds they set.  get_only: the
    verified GET leg alone (one untimed PUT with digests first) -- the bench
    runs it again after the device-resident extras, so a process that has
    allocated and freed tens of GB of HBM is measured too.
    BENCH_GET_STAMPS=1 adds each timed GET batch's CLOCK_MONOTONIC start and
    end (ns) for lining the legs up with a rocprofv3 trace."""
    import numpy as np

    k, m, S = 4, 2, 10 << 20
    D = plan.local_devices
    n = per_dev * D
    rates = pcie_rates(torch, plan.torch_devs)
    data = ctx.host_array(n * k * S).reshape(n, k, S)
    par = ctx.host_array(n * m * S).reshape(n, m, S)
    _fill_random(data, 7 + plan.rank)
    # where the page-locked buffers landed against the GPUs (mxec_host_alloc
    # binds them to the GPUs' node with MXEC_HOST_NUMA=1)
    numa = {"gpu_nodes": [gpu_numa_node(torch, d) for d in sorted(set(plan.torch_devs))],
            "data_pages": numa_nodes(data.ctypes.data, data.nbytes),
            "parity_pages": numa_nodes(par.ctypes.data, par.nbytes)}
    dptr = [data[o, j].ctypes.data for o in range(n) for j in range(k)]
    pptr = [par[o, i].ctypes.data for o in range(n) for i in range(m)]
    objs = [(k, m, S)] * n
    res = {"workload": (f"PUT compute from page-locked host memory: {per_dev} objects per GPU x 4+2 x 10 MiB "
                        f"(mxec_encode_batch_host over {D} device(s) per process); H2D upload, RS encode, "
                        "optional SHA-256 of all 6 chunks, D2H of parity and digests, wall clock"),
           "objects_per_gpu": per_dev, "pcie_all_devices": rates, "numa": numa}
    # H2D and D2H overlap (separate DMA streams): the bound is the slower direction.
    h2d_s = n * k * S / (rates["h2d_GBps"] * 1e9)
    d2h_s = n * m * S / (rates["d2h_GBps"] * 1e9)
    bound_s = max(h2d_s, d2h_s)
    # The same bytes at the measured simultaneous 2:1 rates (pcie_rates).
    duplex_s = max(n * k * S / (rates["duplex_2to1_up_GBps"] * 1e9), n * m * S / (rates["duplex_2to1_down_GBps"] * 1e9))
    dig_all = None
    for sha in ((True,) if get_only else (False, True)):
        dig = np.zeros(n * (k + m) * 32, np.uint8) if sha else None
        if sha:
            dig_all = dig
        ctx.encode_batch_host(objs, dptr, pptr, digests=dig)  # warm: pools, tables
        if get_only:
            break
        c0 = [ctx.pipe_stats(i) for i in range(D)]
        ts = []
        for _ in range(reps):
            barrier()
            t0 = time.perf_counter()
            ctx.encode_batch_host(objs, dptr, pptr, digests=dig)
            ts.append(reduce_max(time.perf_counter() - t0))
        el = statistics.median(ts)
        payload = reduce_sum(float(n * k * S))
        key = "rs_sha256" if sha else "rs_only"
        c1 = [ctx.pipe_stats(i) for i in range(D)]
        res[key] = dict(_leg_times(ts), GiBps_payload=round(payload / GIB / el, 2),
                        frac_of_pcie_bound=round(bound_s / el, 4), frac_of_duplex_bound=round(duplex_s / el, 4),
                        copies=_copy_delta(c0, c1))
    # GET side (chunk_reader.rs:157-226 from the shard files in host memory):
    # mxec_reconstruct_batch_host over the same objects with two seeded
    # erasures each -- the 4 present shards go up, the 2 rebuilt ones come
    # back (the same bytes per object as the PUT leg moves) -- without and
    # with the SHA-256 verification of the present shards.
    sptr = []
    for o in range(n):
        sptr += [data[o, j].ctypes.data for j in range(k)] + [par[o, i].ctypes.data for i in range(m)]
    rng = np.random.default_rng(SEED + 11 + plan.rank)
    present0 = np.ones(n * (k + m), np.uint8)
    for o in range(n):
        for i in rng.choice(k + m, 2, replace=False):
            present0[o * (k + m) + i] = 0
    get_up_s = n * (k + m - 2) * S / (rates["h2d_GBps"] * 1e9)
    get_down_s = n * 2 * S / (rates["d2h_GBps"] * 1e9)
    get_duplex_s = max(n * (k + m - 2) * S / (rates["duplex_2to1_up_GBps"] * 1e9),
                       n * 2 * S / (rates["duplex_2to1_down_GBps"] * 1e9))
    stamps = os.environ.get("BENCH_GET_STAMPS") == "1"
    for verify in ((True,) if get_only else (False, True)):
        exp = dig_all if verify else None
        pr = present0.copy()
        rc, _ = ctx.reconstruct_batch_host(objs, sptr, pr, expected=exp)  # warm
        assert rc == 0, rc
        c0 = [ctx.pipe_stats(i) for i in range(D)]
        ts, marks = [], []
        for _ in range(reps):
            pr = present0.copy()
            barrier()
            t0 = time.perf_counter()
            m0 = time.monotonic_ns()
            rc, _ = ctx.reconstruct_batch_host(objs, sptr, pr, expected=exp)
            marks.append((m0, time.monotonic_ns()))
            ts.append(reduce_max(time.perf_counter() - t0))
            assert rc == 0, rc
        el = statistics.median(ts)
        payload = reduce_sum(float(n * k * S))
        res["get_verify_sha256" if verify else "get_rs_only"] = dict(
            _leg_times(ts), GiBps_payload=round(payload / GIB / el, 2),
            frac_of_pcie_bound=round(max(get_up_s, get_down_s) / el, 4),
            frac_of_duplex_bound=round(get_duplex_s / el, 4))
        # Which copy engine the timed batches used (MXEC_PIPE_COPY=auto: SDMA
        # unless its probe found it slow): the copy counters' difference.
        c1 = [ctx.pipe_stats(i) for i in range(D)]
        res["get_verify_sha256" if verify else "get_rs_only"]["copies"] = _copy_delta(c0, c1)
        if stamps:
            res["get_verify_sha256" if verify else "get_rs_only"]["monotonic_ns"] = marks
    if get_only:
        ctx.host_free(data)
        ctx.host_free(par)
        del data, par
        return res
    if plan.rank == 0:
        # the rebuilt shards of one object, scribbled first, come back exact
        o = n // 3
        want = [data[o, j].copy() for j in range(k)] + [par[o, i].copy() for i in range(m)]
        pr = present0.copy()
        for i in range(k + m):
            if not pr[o * (k + m) + i]:
                (data[o, i] if i < k else par[o, i - k])[:] = 0x5A
        rc, _ = ctx.reconstruct_batch_host(objs, sptr, pr, expected=dig_all)
        got = [data[o, j] for j in range(k)] + [par[o, i] for i in range(m)]
        res["get_spot_check"] = rc == 0 and all(np.array_equal(a, b) for a, b in zip(got, want))
    res["pcie_bound_s_per_batch"] = round(bound_s, 4)
    res["duplex_bound_s_per_batch"] = round(duplex_s, 4)
    res["bound"] = ("max(upload k*S*n / h2d_GBps, download m*S*n / d2h_GBps), the raw pinned copy rates "
                    "measured above on the same devices at once; duplex bound: the same bytes at the rates "
                    "measured with both directions running at once in a 2:1 ratio")
    if plan.rank == 0:
        o = n // 2
        want = _oracle().encode(list(data[o]), m, S)
        res["spot_check_vs_oracle"] = all(np.array_equal(par[o, i], want[i]) for i in range(m))
    ctx.host_free(data)
    ctx.host_free(par)
    del data, par
    return res


def _encoded_set(ctx, shapes, seed: int):
    """Objects of `shapes` in page-locked memory, parity and digests filled
    by one PUT: (rows per object, digests, data bytes)."""
    import numpy as np

    blk = np.random.default_rng(seed).integers(0, 256, (64 << 20) + 4096, dtype=np.uint8)
    rows, dptr, pptr = [], [], []
    for o, (k, m, S) in enumerate(shapes):
        a = ctx.host_array((k + m) * S).reshape(k + m, S)
        flat = a[:k].reshape(-1)
        sh = (o * 4099) % 4096  # a different phase of the block per object
        for x in range(0, flat.size, 64 << 20):
            w = min(64 << 20, flat.size - x)
            flat[x:x + w] = blk[sh:sh + w]
        rows.append(a)
        dptr += [a[j].ctypes.data for j in range(k)]
        pptr += [a[k + i].ctypes.data for i in range(m)]
    dig = np.zeros(sum(k + m for k, m, _ in shapes) * 32, np.uint8)
    st = ctx.encode_batch_host(shapes, dptr, pptr, digests=dig)
    assert (st == 0).all()
    return rows, dig, dptr, pptr, sum(k * S for k, _, S in shapes)


class _GetBatch:
    """A verified host GET over an encoded set: two seeded erasures per
    object (scribbled), every shard pointer, the expected digests."""

    def __init__(self, ctx, shapes, rows, dig, seed: int):
        import numpy as np

        self.ctx, self.shapes, self.rows, self.dig = ctx, shapes, rows, dig
        rng = np.random.default_rng(seed)
        self.ptrs, pres = [], []
        for (k, m, S), a in zip(shapes, rows):
            self.ptrs += [a[i].ctypes.data for i in range(k + m)]
            p = np.ones(k + m, np.uint8)
            p[rng.choice(k + m, 2, replace=False)] = 0
            pres.append(p)
        self.present0 = np.concatenate(pres)
        n = len(rows)
        self.ref = {o: rows[o].copy() for o in sorted({0, n // 3, n // 2, n - 1})}  # a sample

    def run(self):
        g = 0
        for (k, m, S), a in zip(self.shapes, self.rows):  # the lost shards' buffers scribbled
            for i in range(k + m):
                if not self.present0[g + i]:
                    a[i, :4096] = 0x5A
            g += k + m
        pr = self.present0.copy()
        rc, _ = self.ctx.reconstruct_batch_host(self.shapes, self.ptrs, pr, expected=self.dig)
        assert rc == 0 and pr.all(), rc

    def exact(self) -> bool:
        import numpy as np

        return all(np.array_equal(self.rows[o], r) for o, r in self.ref.items())


def e2e_concurrent(ctx, n: int = 128, reps: int = 3, stream_s: float = 5.0) -> dict:
    """Concurrent host-batch calls on one device (MaxIO
    serves PUTs and GETs at once, filesystem.rs:686-828, chunk_reader.rs:87-226,
    main.rs:81):

    * pair: a PUT with digests and a verified GET (two erasures per object),
      n x 4+2 x 10 MiB each from page-locked memory, each alone (median of
      `reps` after a warm one) and both started together from two threads
      (wall clock until both return) -- `pair_over_solo_sum` is the pair's
      time over the two solo times added;
    * mixed_stream: configs[4]'s shapes (4+2 / 8+4 / 10+4 at 64 KiB - 10 MiB
      chunks, 60 objects per batch) from page-locked memory, one thread
      issuing PUT-with-digests batches and one verified-GET batches back to
      back for `stream_s` seconds: payload GiB/s (k x chunk bytes per
      object) of each and together, per-call p50 / p99.
    Spot checks: the pair's GET objects equal their originals, a PUT object's
    parity against the oracle, the stream's GET objects after the stream."""
    import threading

    import numpy as np

    res = {"workload": f"concurrent host batches on one device: pair = PUT with digests + verified GET, "
                       f"{n} x 4+2 x 10 MiB each; mixed_stream = configs[4] shapes, two threads for {stream_s} s"}
    k, m, S = 4, 2, 10 << 20
    shapes = [(k, m, S)] * n
    put_rows, _, put_d, put_p, put_bytes = _encoded_set(ctx, shapes, 31)
    get_rows, get_dig, _, _, get_bytes = _encoded_set(ctx, shapes, 32)
    put_dig = np.zeros(n * (k + m) * 32, np.uint8)
    get = _GetBatch(ctx, shapes, get_rows, get_dig, SEED + 33)

    def put():
        st = ctx.encode_batch_host(shapes, put_d, put_p, digests=put_dig)
        assert (st == 0).all()

    def timed(fn):
        t0 = time.perf_counter()
        fn()
        return time.perf_counter() - t0

    def run_pair():
        go = threading.Barrier(3)
        t_end = {}

        def run(name, fn):
            go.wait()
            fn()
            t_end[name] = time.perf_counter()

        th = [threading.Thread(target=run, args=("put", put)), threading.Thread(target=run, args=("get", get.run))]
        for t in th:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        return max(t_end.values()) - t0, {kname: round(v - t0, 4) for kname, v in t_end.items()}

    # warm: each call alone, then a pair (the second call's lane -- its
    # pinned rings and device pool -- is created by the first pair)
    put(), get.run(), run_pair()
    s0 = ctx.pipe_stats()
    solo_put = statistics.median([timed(put) for _ in range(reps)])
    solo_get = statistics.median([timed(get.run) for _ in range(reps)])
    pair, each = [], []
    for _ in range(reps):
        el_i, each_i = run_pair()
        pair.append(el_i)
        each.append(each_i)
    s1 = ctx.pipe_stats()
    el = statistics.median(pair)
    o = n // 2
    want = _oracle().encode(list(put_rows[o][:k]), m, S)
    res["pair"] = {"solo_put_s": round(solo_put, 4), "solo_get_s": round(solo_get, 4),
                   "pair_s": round(el, 4), "pair_each_s": pair and [round(p, 4) for p in pair],
                   "finish_times_s": each,
                   "pair_over_solo_sum": round(el / (solo_put + solo_get), 4),
                   "payload_GiBps": round((put_bytes + get_bytes) / GIB / el, 2),
                   "counters": {key: s1[key] - s0[key] for key in ("calls", "calls_shared", "spec_pieces",
                                                                   "spec_redos", "pace_waits")},
                   "spot_check": bool(get.exact() and all(np.array_equal(put_rows[o][k + i], want[i])
                                                          for i in range(m)))}
    for a in put_rows + get_rows:
        ctx.host_free(a.reshape(-1))
    del put_rows, get_rows, get
    if stream_s <= 0:
        return res

    # configs[4]: mixed k+m at mixed chunk sizes, a continuous stream.
    kinds = [(4, 2), (8, 4), (10, 4)]
    sizes = [64 << 10, 256 << 10, 1 << 20, 4 << 20, 10 << 20]
    mshapes = [(*kinds[i % 3], sizes[(i // 3) % 5]) for i in range(60)]
    p_rows, _, p_d, p_p, p_bytes = _encoded_set(ctx, mshapes, 41)
    g_rows, g_dig, _, _, g_bytes = _encoded_set(ctx, mshapes, 42)
    p_dig = np.zeros(sum(kk + mm for kk, mm, _ in mshapes) * 32, np.uint8)
    gb = _GetBatch(ctx, mshapes, g_rows, g_dig, SEED + 43)

    def mput():
        st = ctx.encode_batch_host(mshapes, p_d, p_p, digests=p_dig)
        assert (st == 0).all()

    mput(), gb.run()  # warm
    times = {"put": [], "get": []}
    stop = time.perf_counter() + stream_s
    go = threading.Barrier(2)

    def loop(name, fn):
        go.wait()
        while time.perf_counter() < stop:
            times[name].append(timed(fn))

    s0 = ctx.pipe_stats()
    t0 = time.perf_counter()
    th = [threading.Thread(target=loop, args=("put", mput)), threading.Thread(target=loop, args=("get", gb.run))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    s1 = ctx.pipe_stats()

    def pct(v, q):
        v = sorted(v)
        return round(v[min(len(v) - 1, int(q * len(v)))], 4)

    res["mixed_stream"] = {
        "batch": "60 objects: (4+2, 8+4, 10+4) x (64 KiB, 256 KiB, 1 MiB, 4 MiB, 10 MiB) chunks, 4 of each",
        "seconds": round(wall, 3),
        "put": {"calls": len(times["put"]), "GiBps_payload": round(len(times["put"]) * p_bytes / GIB / wall, 2),
                "p50_s": pct(times["put"], 0.5), "p99_s": pct(times["put"], 0.99)},
        "get": {"calls": len(times["get"]), "GiBps_payload": round(len(times["get"]) * g_bytes / GIB / wall, 2),
                "p50_s": pct(times["get"], 0.5), "p99_s": pct(times["get"], 0.99)},
        "GiBps_payload": round((len(times["put"]) * p_bytes + len(times["get"]) * g_bytes) / GIB / wall, 2),
        "counters": {key: s1[key] - s0[key] for key in ("calls", "calls_shared", "spec_pieces", "spec_redos",
                                                        "pace_waits")},
        "spot_check": gb.exact(),
    }
    for a in p_rows + g_rows:
        ctx.host_free(a.reshape(-1))
    return res


# ---- main ------------------------------------------------------------------------


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # The driver's own command is --steps 20 --warmup 5; the RS grid tuner's
    # trial launches run before the warmup (tune_before_timing), so the grid
    # never changes inside the timed region whatever --warmup is.
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="2", choices=["2", "3", "3c", "ns", "4a", "4b", "5", "sums", "frames"])
    ap.add_argument("--workers", type=int, default=8, help="config 3c: concurrent batches")
    ap.add_argument("--objects", type=int, default=0, help="objects per GPU (0 = config default)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the secondary measurements that the default config-2 run adds "
                         "at N=1 (north-star shape, config 3 / 3c, PUT compute)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end host-memory leg")
    args = ap.parse_args()

    import torch

    try:
        plan = plan_devices(args.gpus, os.environ, torch.cuda.device_count())
    except BenchRefusal as e:
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        return 2
    if plan.mode == "ranks":
        import torch.distributed as dist

        # BENCH_GPU_OF_RANK=0 pins every rank to GPU 0 and BENCH_DIST_BACKEND=gloo
        # carries the timing collectives on the host: a rehearsal of the
        # multi-rank path on a one-GPU box.  Defaults: GPU = LOCAL_RANK, RCCL.
        gpu = plan.torch_devs[0]
        torch.cuda.set_device(gpu)
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(plan.torch_devs[0])
    rank, world = plan.rank, plan.world

    import maxio_amd

    D = plan.local_devices
    one_gpu = plan.n_gpus == 1
    # config 3c (and the default run's extras, which include it) needs one
    # slot per concurrent batch.
    with_extra = args.config == "2" and one_gpu and not args.no_extra
    ctx = maxio_amd.Context(device_mask=plan.device_mask,
                            streams_per_device=max(2, args.workers if args.config == "3c" or with_extra else 2),
                            test={"logical_devices": plan.logical} if plan.logical > 1 else None)
    if len(ctx.device_ids()) != D:
        print(f"bench.py: the context opened {len(ctx.device_ids())} device(s), the plan needs {D}",
              file=sys.stderr, flush=True)
        return 3
    # The host legs first, before the device-resident batch exists: a
    # long-lived server's state, not the seconds after this process frees
    # its 77 GB batch, when SDMA downloads crawl beside the verified GET's
    # chains; the verified GET runs again after the extras
    # (extra.e2e_get_after_extras), which measures that state.
    host_extra = {}
    if not args.no_e2e and args.config == "2":
        host_extra["e2e_host"] = e2e_host_leg(ctx, torch, plan, 128 if D == 1 and world == 1 else 64)
        if D == 1 and world == 1 and with_extra:
            host_extra["e2e_put_512"] = e2e_put_large(ctx)
            host_extra["e2e_concurrent"] = e2e_concurrent(ctx)
    lanes = []  # (workload, stream, torch device) per ctx device
    for di in range(D):
        tdev = torch.device("cuda", plan.torch_devs[di])
        with torch.cuda.device(tdev):
            # A dedicated stream per device: the kernels and the HIP events
            # that time them are on the same queue.
            stream = torch.cuda.Stream(device=tdev)
            w = make_workload(args.config, torch, DevView(ctx, di), tdev, stream.cuda_stream, args.objects,
                              rank * D + di, args.workers)
            torch.cuda.synchronize()
        lanes.append((w, stream, tdev))
    w, stream, dev = lanes[0]
    sh = stream.cuda_stream

    tuning = tune_before_timing(torch, lanes, plan.torch_devs)
    run_steps(torch, lanes, args.warmup, events=False)
    sync_all(torch, plan.torch_devs)
    spot_local = all(bool(l[0].spot_check()) for l in lanes)
    spot_ok = reduce_max(0.0 if spot_local else 1.0) == 0.0

    barrier()
    sync_all(torch, plan.torch_devs)
    t0 = time.perf_counter()
    evs = run_steps(torch, lanes, args.steps, events=True)
    sync_all(torch, plan.torch_devs)
    barrier()
    elapsed = reduce_max(time.perf_counter() - t0)
    ms_dev = [sum(a.elapsed_time(b) for a, b in ev) / len(ev) for ev in evs]
    if getattr(w, "wall_timed", False):  # work on the workers' streams, not `stream`
        ms_dev = [elapsed * 1e3 / args.steps] * D

    # The grid the RS grid tuner settled on for the encode shape (0: still
    # tuning), and whether it was the same grid before the timed steps.
    grid_bpc = w.ctx.rs_grid(w.k, w.m, w.S) if isinstance(w, Encode) else None
    if isinstance(w, Encode):
        tuning["grid_after_timing"] = grid_bpc
        tuning["same_grid_over_timed_steps"] = grid_bpc == tuning.get("grid_before_timing")
    payload_local = float(sum(l[0].payload for l in lanes))
    value = reduce_sum(payload_local) * args.steps / GIB / elapsed  # weak scaling: every GPU of every rank
    per_dev = [{"gpu": plan.torch_devs[i] if plan.mode != "logical" else f"logical {i} of card 0",
                "rank": rank, "ms_per_launch": round(ms_dev[i], 4),
                "achieved": round(lanes[i][0].alg_bytes / (ms_dev[i] * 1e-3) / 1e9, 1),
                "frac": round(lanes[i][0].alg_bytes / (ms_dev[i] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
               for i in range(D)]
    per_dev = [d for part in gather_objects(per_dev) for d in part]
    # The headline kernel time: the slowest device's (equal to the one device at N=1).
    ms_launch = max(d["ms_per_launch"] for d in per_dev)
    achieved = w.alg_bytes / (ms_launch * 1e-3) / 1e9

    # §8(d) second denominator: this box's rates for plain streams of the RS
    # kernel's own load/store forms (libmaxio_probe.so), on rank 0's first device.
    cal = calibrate(torch, dev, stream) if rank == 0 else None
    box_key = {(4, 2): "rs_pattern_k4m2_GBps", (8, 4): "rs_pattern_k8m4_GBps"}.get(
        (getattr(w, "k", 0), getattr(w, "m", 0)), "copy_GBps")
    if isinstance(w, Mixed):
        box_key = "rs_pattern_k4m2_GBps"  # as the default line's extra.config5
    elif not isinstance(w, Encode):
        box_key = "copy_GBps"
    elif cal is not None:
        same = pattern_on_buffers(torch, stream, w)
        if same:
            cal["rs_pattern_same_buffers_GBps"] = same
            box_key = "rs_pattern_same_buffers_GBps"
        f4 = float4_copy_on_buffers(torch, stream, w)
        if f4:
            cal["float4_copy_same_buffers_GBps"] = f4
            if not same:  # the pattern probe needs k % 4 == 0 (4a: k = 10)
                box_key = "float4_copy_same_buffers_GBps"
    copy_peak = cal.get(box_key) if cal else None

    extra = {}
    if rank == 0 and hasattr(w, "breakdown"):
        extra["breakdown"] = w.breakdown()
    if "crc32c" in extra.get("breakdown", {}):
        crc = extra["breakdown"]["crc32c"]
        # The HBM-bound kernel of this workload is the CRC pass; MD5 is a
        # serial chain per body (us_per_block in the breakdown).
        ms_launch = crc["ms"]
        achieved = w.alg_bytes / (ms_launch * 1e-3) / 1e9
        w.kernel = "crc_tiles_kernel + crc_finish_kernel (CRC32C alone)"
    cpu_spec = w.cpu_work() if (rank == 0 and one_gpu and args.cpu_seconds > 0) else None
    cpu_sha_ni = getattr(w, "cpu_sha_ni", None)  # set by cpu_work when the baseline hashes
    alg_bytes, w_name, w_kernel, w_bound, w_payload = w.alg_bytes, w.name, w.kernel, w.bound, w.payload
    w_placement = getattr(w, "placement", None)
    is_stream = isinstance(w, ReconstructStream)
    stream_dims = (len(w.parts), w.parts[0].n) if is_stream else None
    mixed_batch = args.config == "5" and getattr(w, "mode", "") == "batch"
    for l in lanes:
        l[0].drop()  # HBM for the secondary workloads
    del w
    lanes = []
    torch.cuda.empty_cache()
    extra.update(host_extra)
    if rank == 0 and with_extra:
        extra.update(extras(ctx, torch, dev, stream, args.steps, cal))
        if not args.no_e2e:
            # The verified GET again, now that the process has allocated and
            # freed the extras' tens of GB of HBM (a long-lived MaxIO server's
            # shape): its batches' max against their median.
            torch.cuda.empty_cache()
            # BENCH_GET_AFTER_SLEEP (s, lab): idle this long first -- the GET
            # stall study times the leg with and without a pause
            # after the extras' frees.
            pause = float(os.environ.get("BENCH_GET_AFTER_SLEEP", "0"))
            if pause > 0:
                time.sleep(pause)
            extra["e2e_get_after_extras"] = e2e_host_leg(ctx, torch, plan, 128, get_only=True)
            if pause > 0:
                extra["e2e_get_after_extras"]["slept_s_before"] = pause
    if cal is not None:
        extra["calibration"] = cal
    cpu = cpu_all = None
    if cpu_spec is not None:  # the CPU leg runs at N=1 only
        work, per_call, what = cpu_spec
        v, n, el = cpu_leg(work, per_call, args.cpu_seconds, 1)
        cpu = {"value": round(v, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
               "sample": f"{n} calls in {el:.1f}s, 1 thread: {what}"}
        if cpu_sha_ni is not None:
            cpu["sha_ni"] = cpu_sha_ni
        # The GPU box grants 16 host cores (OMP_NUM_THREADS) while
        # os.cpu_count() shows the whole machine.
        nc = os.cpu_count() or 1
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(nc, 64)
        v, n, el = cpu_leg(work, per_call, max(2.0, args.cpu_seconds / 2), threads)
        cpu_all = {"value": round(v, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
                   "sample": f"{n} calls in {el:.1f}s on {threads} threads "
                             f"(OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}, os.cpu_count()={nc})"}
        if cpu_sha_ni is not None:
            cpu_all["sha_ni"] = cpu_sha_ni

    if rank == 0:
        tag = {"2": ("k4m2", grid_bpc), "ns": ("k8m4", grid_bpc), "4a": ("k10m4", grid_bpc),
               "sums": ("crc_tiles", None), "frames": ("gcm_frames", None)}.get(args.config)
        if mixed_batch:
            tag = ("cfg5_grouped", RS_GROUP_BLOCKS_PER_CU)
        traffic, tsrc = pmc_traffic(tag[0], alg_bytes, tag[1]) if tag else (None, None)
        if plan.mode == "devices":
            par = (f"{plan.n_gpus} GPUs in one process: one mxec_ctx over {plan.n_gpus} devices, each GPU's "
                   "objects on its own stream and host thread, no collectives")
        elif plan.mode == "ranks":
            par = f"{plan.n_gpus} ranks (torch.distributed.run), one GPU each, no data-path collectives"
        elif plan.mode == "logical":
            par = f"REHEARSAL: {plan.n_gpus} logical devices of one card, no collectives"
        else:
            par = "one GPU, no collectives"
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": plan.n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: uniform random bytes (torch.randint on device, seeded per GPU)",
            "config": {
                "workload": w_name,
                "bench_config": args.config,
                "payload_bytes_per_step_per_gpu": int(w_payload),
                "placement": w_placement,
                "parallelism": par,
            },
            "roofline": {
                "bound": w_bound,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "kernel": w_kernel,
                "bytes_per_launch": float(alg_bytes),
                "ms_per_launch": round(ms_launch, 4),
                "traffic_source": tsrc,
                "blocks_per_cu": grid_bpc,
                "box_stream": box_key if copy_peak else None,
                "box_stream_GBps": round(copy_peak, 1) if copy_peak else None,
                "frac_of_box_stream": round(achieved / copy_peak, 4) if copy_peak else None,
            },
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "tuner_decided_before_timing": tuning["decided"],
            "tuning": tuning,
            "spot_check_vs_oracle": spot_ok,
            "extra": extra or None,
        }
        if w_bound != "hbm":
            line["roofline"]["frac_basis"] = (
                "the workload's algorithmic HBM bytes against 8 TB/s; the workload is VALU-bound, its binding "
                "roofline is the default line's extra.config3.roofline (chain) / extra.config3c.roofline")
        if cal and cal.get("float4_copy_same_buffers_GBps"):
            line["roofline"]["float4_copy_GBps"] = cal["float4_copy_same_buffers_GBps"]
            line["roofline"]["frac_of_float4_copy"] = round(achieved / cal["float4_copy_same_buffers_GBps"], 4)
        if plan.n_gpus > 1:
            line["roofline"]["per_gpu"] = per_dev
            line["config"]["launch"] = plan.mode
        if plan.rehearsal:
            line["config"]["rehearsal"] = plan.rehearsal
        if is_stream:
            n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
            line["roofline"] = dict(stream_step_roofline(elapsed * 1e3 / args.steps, *stream_dims, n_cus),
                                    traffic=None)
        print(json.dumps(line), flush=True)
    ctx.close()
    if os.environ.get("BENCH_DUMP_MAPS") == "1":
        # The loaded DSOs' address ranges, so a fault during process teardown
        # (after this point: static destructors, __cxa_finalize) resolves to
        # a library and an offset.
        with open("/proc/self/maps") as f:
            maps = [l.rstrip("\n") for l in f if " r-xp " in l or ".so" in l]
        print("BENCH_MAPS_BEGIN\n" + "\n".join(maps) + "\nBENCH_MAPS_END", file=sys.stderr, flush=True)
    if plan.mode == "ranks":
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

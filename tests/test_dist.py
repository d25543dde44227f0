"""CPU, world_size 2 over gloo: the bench's object partitioning (objects per
GPU, no data-path collective) covers the batch exactly once, and the timing
reduce takes the max over ranks.  Each rank encodes its objects with the
oracle (CPU stand-in for its GPU) and the union equals a single-rank run."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_obj, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle

    mine = bench.shard_objects(n_obj, rank, world)
    rng = np.random.default_rng(123)
    all_data = rng.integers(0, 256, (n_obj, 4, 256), dtype=np.uint8)
    parity = {o: np.stack(oracle.encode(list(all_data[o]), 2)) for o in mine}
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **{str(o): p for o, p in parity.items()})
    t = bench.reduce_max(float(rank + 1))
    with open(os.path.join(out_dir, f"t{rank}"), "w") as f:
        f.write(repr(t))
    bench.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_obj", [7, 8])
def test_partition_and_max_reduce_gloo(tmp_path, n_obj):
    import oracle

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), n_obj, str(tmp_path)), nprocs=world, join=True)
    got = {}
    for r in range(world):
        with np.load(tmp_path / f"r{r}.npz") as z:
            for key in z.files:
                assert int(key) not in got
                got[int(key)] = z[key]
        assert float(open(tmp_path / f"t{r}").read()) == 2.0
    assert sorted(got) == list(range(n_obj))
    rng = np.random.default_rng(123)
    all_data = rng.integers(0, 256, (n_obj, 4, 256), dtype=np.uint8)
    for o in range(n_obj):
        assert np.array_equal(got[o], np.stack(oracle.encode(list(all_data[o]), 2)))


def test_shard_objects_edges():
    assert list(bench.shard_objects(0, 0, 2)) == []
    assert list(bench.shard_objects(3, 1, 4)) == [1]
    assert list(bench.shard_objects(3, 3, 4)) == []
    assert list(bench.shard_objects(10, 1, 4)) == [1, 5, 9]  # object i -> GPU i mod G
    covered = [o for r in range(8) for o in bench.shard_objects(1024 * 8, r, 8)]
    assert sorted(covered) == list(range(1024 * 8))

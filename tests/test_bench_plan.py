"""CPU: bench.py's --gpus plumbing.  A line's n_gpus always equals --gpus:
one process drives N devices through one mxec_ctx, or torch.distributed.run
ranks drive one each (--gpus must equal WORLD_SIZE), and a run that cannot
reach N GPUs exits non-zero without a JSON line."""
from __future__ import annotations

import os
import re
import subprocess
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_single_and_in_process_devices():
    p = bench.plan_devices(1, {}, 8)
    assert (p.mode, p.n_gpus, p.torch_devs, p.device_mask) == ("single", 1, [0], 1)
    for n in (2, 4, 8):
        p = bench.plan_devices(n, {}, 8)
        assert p.mode == "devices" and p.n_gpus == n and p.torch_devs == list(range(n))
        assert p.device_mask == (1 << n) - 1 and p.local_devices == n and p.rehearsal is None


def test_refuses_more_gpus_than_visible():
    with pytest.raises(bench.BenchRefusal, match="asks for 2 GPUs but 1 HIP device"):
        bench.plan_devices(2, {}, 1)
    with pytest.raises(bench.BenchRefusal):
        bench.plan_devices(8, {}, 4)
    with pytest.raises(bench.BenchRefusal):
        bench.plan_devices(1, {}, 0)
    with pytest.raises(bench.BenchRefusal):
        bench.plan_devices(0, {}, 8)


def test_logical_rehearsal_is_labelled():
    p = bench.plan_devices(4, {"BENCH_REHEARSE_LOGICAL": "1"}, 1)
    assert p.mode == "logical" and p.n_gpus == 4 and p.torch_devs == [0, 0, 0, 0]
    assert p.logical == 4 and p.device_mask == 1 and "not an N-GPU measurement" in p.rehearsal
    with pytest.raises(bench.BenchRefusal):
        bench.plan_devices(16, {"BENCH_REHEARSE_LOGICAL": "1"}, 1)
    # enough real devices: no rehearsal even when asked
    assert bench.plan_devices(2, {"BENCH_REHEARSE_LOGICAL": "1"}, 8).mode == "devices"


def test_torchrun_ranks():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    p = bench.plan_devices(8, env, 8)
    assert (p.mode, p.n_gpus, p.torch_devs, p.world, p.rank) == ("ranks", 8, [3], 8, 3)
    with pytest.raises(bench.BenchRefusal, match="must equal --nproc-per-node"):
        bench.plan_devices(1, env, 8)
    with pytest.raises(bench.BenchRefusal, match="wants GPU 3"):
        bench.plan_devices(8, env, 2)
    p = bench.plan_devices(2, {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1", "BENCH_GPU_OF_RANK": "0"}, 1)
    assert p.torch_devs == [0] and "rehearsal" in p.rehearsal


@pytest.mark.parametrize("gpus", ["2", "8"])
def test_bench_exits_nonzero_without_the_gpus(gpus):
    """No GPU in this container: --gpus N must refuse (exit 2, no JSON line)
    before touching a device."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", gpus, "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == ""
    assert f"--gpus {gpus}" in r.stderr


def test_dev_view_binds_device():
    calls = []

    class Fake:
        def encode_strided_device(self, *a, dev=0, stream=None):
            calls.append(("enc", dev))

        def combiner_stats(self, dev=0):
            calls.append(("comb", dev))

        def close(self):
            calls.append(("close",))

    v = bench.DevView(Fake(), 5)
    v.encode_strided_device(1, 2, stream=7)
    v.combiner_stats()
    v.close()
    assert calls == [("enc", 5), ("comb", 5), ("close",)]


def test_blocks_per_cu_mirrors_rs_kernel():
    """bench.rs_blocks_per_cu (the PMC-traffic guard) restates
    rs_default_variant; fail when the kernel's choice moves."""
    src = open(os.path.join(ROOT, "maxio_amd", "csrc", "rs_kernel.hip")).read()
    body = src[src.index("RsVariant rs_default_variant("):]
    body = body[:body.index("\n}\n")]
    m = re.search(r"v\.blocks_per_cu = r_total <= (\d+) \? (\d+) : (\d+);", body)
    assert m, "rs_default_variant's blocks_per_cu expression changed: update bench.rs_blocks_per_cu"
    cut, lo, hi = map(int, m.groups())
    for r in range(1, 9):
        assert bench.rs_blocks_per_cu(r) == (lo if r <= cut else hi)
    g = src[src.index("RsVariant rs_group_variant("):]
    assert re.search(r"v\.blocks_per_cu = (\d+);", g).group(1) == str(bench.RS_GROUP_BLOCKS_PER_CU)


def test_pmc_traffic_needs_matching_grid(tmp_path, monkeypatch):
    import json

    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r9_pmc_k4m2_traffic.json").write_text(json.dumps(
        {"hbm_bytes_per_launch": 101.0, "algorithmic_bytes_per_launch": 100.0, "blocks_per_cu": 512}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_traffic("k4m2", 1000.0, 1024) == (None, None)
    t, src = bench.pmc_traffic("k4m2", 1000.0, 512)
    assert t == 1010.0 and src.endswith("r9_pmc_k4m2_traffic.json")


def test_sha_chain_block_reads_committed_clock():
    """Config 3's chain roofline: 905 consumer VALU x 4 cycles per block at
    the clock of the committed GRBM pass (profiles/r*/clock/clock_3.json)."""
    import bench

    d = bench.sha_chain_block("split", 1.669)
    assert d["bound"] == "valu-chain" and d["consumer_valu_per_block"] == 905
    assert 1.0 < d["clock_GHz_measured"] <= 2.4 and d["clock_source"].startswith("profiles/")
    assert abs(d["floor_us_per_block"] - 905 * 4 / (d["clock_GHz_measured"] * 1e3)) < 1e-3
    assert 0.5 < d["frac"] <= 1.0
    assert bench.sha_chain_block("stream", 1.0) is None

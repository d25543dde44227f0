#!/usr/bin/env python3
"""Where the host side of the pipeline lives: the GPU's NUMA node, the CPUs
this process may run on, and the node of the pages of a page-locked buffer
from mxec_host_alloc (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR), for each of
a few buffers.  Lab tool, not product."""
from __future__ import annotations

import ctypes
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def page_nodes(addr: int, nbytes: int, samples: int = 16) -> list[int]:
    libc = ctypes.CDLL("libc.so.6", use_errno=True)
    MPOL_F_NODE, MPOL_F_ADDR = 1, 2
    out = []
    for i in range(samples):
        a = addr + (nbytes // samples) * i
        node = ctypes.c_int(-1)
        rc = libc.syscall(239, ctypes.byref(node), None, ctypes.c_ulong(0), ctypes.c_void_p(a),
                          ctypes.c_ulong(MPOL_F_NODE | MPOL_F_ADDR))  # get_mempolicy
        out.append(node.value if rc == 0 else -ctypes.get_errno())
    return out


def main() -> int:
    import maxio_amd

    info = {"gpu_numa_nodes": {}, "cpus_allowed": sorted(os.sched_getaffinity(0))[:64]}
    for p in glob.glob("/sys/class/drm/card*/device/numa_node"):
        with open(p) as f:
            info["gpu_numa_nodes"][p.split("/")[4]] = f.read().strip()
    nodes = {}
    for p in glob.glob("/sys/devices/system/node/node*/cpulist"):
        with open(p) as f:
            nodes[p.split("/")[-2]] = f.read().strip()
    info["node_cpus"] = nodes
    info["cpus_allowed_count"] = len(os.sched_getaffinity(0))
    import torch

    pr = torch.cuda.get_device_properties(0)
    bus = f"{getattr(pr, 'pci_domain_id', 0):04x}:{getattr(pr, 'pci_bus_id', 0):02x}:{getattr(pr, 'pci_device_id', 0):02x}.0"
    info["hip_device0_pci"] = bus
    try:
        with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
            info["hip_device0_numa_node"] = f.read().strip()
    except OSError as e:
        info["hip_device0_numa_node"] = str(e)
    ctx = maxio_amd.Context(device_mask=1, streams_per_device=2)
    for i in range(3):
        a = ctx.host_array(1 << 30)
        a[::4096] = 1  # touch
        info[f"host_array_{i}_page_nodes"] = page_nodes(a.ctypes.data, a.nbytes)
    print(json.dumps(info))
    ctx.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

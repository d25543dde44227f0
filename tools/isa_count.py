#!/usr/bin/env python3
"""Instruction counts of the loop bodies of a HIP kernel file in its gfx950
ISA (the basis of bench.py's SHA_VALU_PER_BLOCK and of DESIGN §4's per-block
figures).

  python tools/isa_count.py maxio_amd/csrc/sha256_kernel.hip [--kernel split]

Compiles the file device-only to assembly (hipcc -S), then for every loop
(an "Inner Loop Header" label and the last branch back to it) prints the
VALU / SALU / VMEM / LDS instruction counts and the VALU mix.
"""
from __future__ import annotations

import argparse
import collections
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def assemble(src: str) -> list[str]:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-x", "hip",
                        "--cuda-device-only", "-S", "-o", out, src], check=True,
                       stderr=subprocess.DEVNULL)
        with open(out) as f:
            return f.read().splitlines()


def loops(lines: list[str]):
    """Blocks grouped by the loop they belong to: the header block
    ("Loop Header") and every block the compiler annotates
    "in Loop: Header=BBx_y" (latches placed before the header included)."""
    func, cur = None, None
    groups: dict[tuple[str, str], list[str]] = {}
    for ln in lines:
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            func, cur = m.group(1), None
            continue
        if re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:)", ln):
            h = re.search(r"Loop Header", ln)
            m = re.match(r"^\.LBB(\d+_\d+):", ln)
            if h and m:
                cur = "BB" + m.group(1)
            else:
                m2 = re.search(r"in Loop: Header=(BB\d+_\d+)", ln)
                cur = m2.group(1) if m2 else None
            continue
        if cur:
            groups.setdefault((func, cur), []).append(ln)
    for (func, lab), body in groups.items():
        yield func, lab, body


def count(body: list[str]) -> dict:
    ins = [ln.split()[0] for ln in body if ln.startswith("\t") and ln.strip() and not ln.strip().startswith((";", "."))]
    c = {
        "valu": sum(1 for x in ins if x.startswith("v_")),
        "salu": sum(1 for x in ins if x.startswith("s_")),
        "vmem": sum(1 for x in ins if x.startswith(("global_", "buffer_", "flat_"))),
        "lds": sum(1 for x in ins if x.startswith("ds_")),
        "barriers": sum(1 for x in ins if x == "s_barrier"),
    }
    c["valu_mix"] = dict(collections.Counter(x for x in ins if x.startswith("v_")).most_common(8))
    return c


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="?", default=os.path.join(ROOT, "maxio_amd", "csrc", "sha256_kernel.hip"))
    ap.add_argument("--kernel", default="", help="substring of the mangled kernel name")
    a = ap.parse_args()
    for func, lab, body in loops(assemble(a.src)):
        if a.kernel and a.kernel not in func:
            continue
        c = count(body)
        print(f"{func} {lab}: valu={c['valu']} salu={c['salu']} vmem={c['vmem']} lds={c['lds']} "
              f"barriers={c['barriers']} mix={c['valu_mix']}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

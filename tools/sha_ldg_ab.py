#!/usr/bin/env python3
"""A/B of the SHA-256 lag pair form's K + W read groups (sha256_kernel.hip
sha256_quad_kernel LDG; lab knob MXEC_SHA_LDG=1|2|4|15, lab build): each
setting in a fresh child process running tools/sha_alone.py (the configs[2]
hash launch alone, 10 240 x 1 MiB), rounds interleaved so box drift hits
every setting alike.  The parent never touches the GPU.

  python tools/sha_ldg_ab.py --rounds 3 --ldg 1,2,4
  python tools/sha_ldg_ab.py --ldg "" --libs maxilp:maxio_amd/lib/libmaxio_ec_sched_max-ilp.so
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ldg", default="1,2,4")
    ap.add_argument("--n", type=int, default=10240)
    ap.add_argument("--mib", type=int, default=1)
    ap.add_argument("--libs", default="", help="name:path,... other builds of the library to time beside")
    a = ap.parse_args()
    lab = os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_ec_lab.so")
    runs = [("product", {})] + [(f"lab_ldg{g}", {"MXEC_LIB": lab, "MXEC_SHA_LDG": g}) for g in a.ldg.split(",") if g]
    runs += [(n, {"MXEC_LIB": os.path.join(ROOT, pth)}) for n, pth in (x.split(":", 1) for x in a.libs.split(",") if x)]
    for r in range(a.rounds):
        for name, env in runs:
            e = dict(os.environ, **env)
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sha_alone.py"), "--n", str(a.n),
                                  "--mib", str(a.mib), "--reps", "5"], env=e, capture_output=True, text=True,
                                 timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                return out.returncode
            line = json.loads(out.stdout.strip().splitlines()[-1])
            print(json.dumps({"round": r, "setting": name, **line}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

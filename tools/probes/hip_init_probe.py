#!/usr/bin/env python3
"""Start N fresh hip_init_probe processes at once (a YARN wave of reduce task JVMs) and print each
one's init phases plus the median / max per phase. Build the probe first:

    python tools/probes/hip_init_probe.py --build          # here (hipcc cross-compiles for gfx950)
    python tools/probes/hip_init_probe.py -n 1 -n 15       # on the GPU box
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
EXE = os.path.join(ROOT, "uda_amd", "bin", "hip_init_probe")


def build() -> None:
    lib = os.path.join(ROOT, "uda_amd", "lib")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", os.path.join(HERE, "hip_init_probe.cc"),
           "-o", EXE, f"-L{lib}", "-luda", f"-Wl,-rpath,{lib}", "-lhsa-runtime64"]
    subprocess.run(cmd, check=True)
    print(EXE)


def wave(n: int) -> dict:
    procs = [subprocess.Popen([EXE], stdout=subprocess.PIPE, text=True) for _ in range(n)]
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=120)
        outs.append(json.loads(out.strip().splitlines()[-1]))
    keys = [k for k in outs[0] if k.endswith("_ms") and k != "t0_boot_ms"]
    summary = {k: {"median": round(statistics.median(o[k] for o in outs), 1), "max": round(max(o[k] for o in outs), 1)}
               for k in keys}
    return {"n": n, "ok": all(o["ok"] for o in outs), "phases": summary}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--build", action="store_true")
    ap.add_argument("-n", type=int, action="append", default=[])
    a = ap.parse_args()
    if a.build:
        build()
        return 0
    for n in a.n or [1, 15]:
        print(json.dumps(wave(n)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

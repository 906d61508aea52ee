#!/usr/bin/env python3
"""Nightly build: build every flavour, test, package, run a scaled regression, report.

Reference: scripts/build/{build.sh,config.ini,manage.sh} check out Hadoop
versions from SVN, apply the plugin patch map, build RPM/DEB per version plus a Bullseye coverage
build, and mail a report. Nothing here is fetched (no network): the stages run on the checked-out
tree, one after the other, each with its own log and status:

    build       tools/build.py (release libuda.so + pybind11 module, hipcc for gfx950)
    debug       tools/build.py --debug (separate build dir; catches -O0-only warnings/asserts)
    java        java/build.sh, when javac and Hadoop jars are present (else SKIP)
    tests       pytest -m "not gpu" (CPU tier)
    gpu_tests   pytest -m gpu, only when a HIP device is visible (else SKIP)
    sanitizers  tools/run_sanitizers.py (host code ASan/UBSan/TSan), with --sanitizers only
    package     tools/package.py -> dist/uda-amd-<version>-gfx950.tar.gz
    regression  tools/regression.py --scale <s> --samples 1 on benchmarks/regression_matrix.csv
    logs        tools/collect_logs.py over the regression output

    python tools/nightly.py --out results/nightly [--stages build,tests] [--sanitizers] [--scale 0.05]

Writes <out>/nightly.json and <out>/nightly.md (stage, status, seconds, log file); exit status 1
if any stage failed. A failing stage does not stop the later independent ones, but the stages
that need its output (tests/package/regression need build) are reported as SKIP.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import shutil
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable
ALL_STAGES = ["build", "debug", "java", "tests", "gpu_tests", "sanitizers", "package", "regression", "logs"]
NEEDS_BUILD = {"tests", "gpu_tests", "sanitizers", "package", "regression", "logs"}


def _gpu_visible() -> bool:
    # device count only (does not initialise HIP in this process)
    r = subprocess.run([PY, "-c", "import torch; print(torch.cuda.device_count())"], capture_output=True,
                       text=True, cwd=ROOT)
    return r.returncode == 0 and r.stdout.strip().isdigit() and int(r.stdout.strip()) > 0


def stage_commands(args) -> dict:
    reg_out = os.path.join(args.out, "regression")
    return {
        "build": [PY, "tools/build.py"],
        "debug": [PY, "tools/build.py", "--debug"],
        "java": ["bash", "java/build.sh"],
        "tests": [PY, "-m", "pytest", "tests", "-q", "-x", "-m", "not gpu"],
        "gpu_tests": [PY, "-u", "-m", "pytest", "tests", "-q", "-x", "-m", "gpu", "--timeout", "120",
                      "--timeout-method", "thread"],
        "sanitizers": [PY, "tools/run_sanitizers.py"],
        "package": [PY, "tools/package.py", "--out", os.path.join(args.out, "dist")],
        "regression": [PY, "tools/regression.py", "--out", reg_out, "--samples", "1", "--scale", str(args.scale)],
        "logs": [PY, "tools/collect_logs.py", os.path.join(reg_out, "logs"), "--out", os.path.join(args.out, "logs")],
    }


def skip_reason(stage: str, args, results: dict) -> str | None:
    if stage in NEEDS_BUILD and results.get("build", {}).get("status") == "FAIL":
        return "build failed"
    if stage == "java" and not (shutil.which("javac") and os.environ.get("HADOOP_HOME")):
        return "no javac/HADOOP_HOME"
    if stage == "gpu_tests" and not _gpu_visible():
        return "no HIP device visible"
    if stage == "sanitizers" and not args.sanitizers:
        return "not requested (--sanitizers)"
    if stage == "logs" and results.get("regression", {}).get("status") not in ("PASS", "FAIL"):
        return "no regression output"
    return None


def run(args) -> dict:
    os.makedirs(args.out, exist_ok=True)
    cmds = stage_commands(args)
    stages = [s for s in ALL_STAGES if s in set(args.stages.split(","))] if args.stages else ALL_STAGES
    results: dict = {}
    for s in stages:
        why = skip_reason(s, args, results)
        if why:
            results[s] = {"status": "SKIP", "reason": why}
            continue
        log = os.path.join(args.out, f"{s}.log")
        t0 = time.perf_counter()
        with open(log, "w") as f:
            f.write("$ " + " ".join(cmds[s]) + "\n")
            f.flush()
            try:
                rc = subprocess.run(cmds[s], cwd=ROOT, stdout=f, stderr=subprocess.STDOUT,
                                    timeout=args.stage_timeout).returncode
            except subprocess.TimeoutExpired:
                rc = 124
                f.write(f"\n[nightly] stage timed out after {args.stage_timeout}s\n")
        results[s] = {"status": "PASS" if rc == 0 else "FAIL", "rc": rc,
                      "seconds": round(time.perf_counter() - t0, 1), "log": log}
    meta = {"date": datetime.datetime.now().isoformat(timespec="seconds"), "host": socket.gethostname(),
            "git": _git_rev()}
    with open(os.path.join(args.out, "nightly.json"), "w") as f:
        json.dump({"meta": meta, "stages": results}, f, indent=1)
    md = [f"# Nightly {meta['date']} ({meta['git']})", "", "| stage | status | s | log / reason |", "|---|---|---|---|"]
    for s, r in results.items():
        md.append(f"| {s} | {r['status']} | {r.get('seconds', '-')} | {r.get('log') or r.get('reason')} |")
    with open(os.path.join(args.out, "nightly.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    return results


def _git_rev() -> str:
    r = subprocess.run(["git", "rev-parse", "--short", "HEAD"], cwd=ROOT, capture_output=True, text=True)
    return r.stdout.strip() or "unknown"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default="results/nightly")
    ap.add_argument("--stages", default="", help=f"comma list out of {','.join(ALL_STAGES)} (default: all)")
    ap.add_argument("--sanitizers", action="store_true", help="include the host sanitizer builds (slow)")
    ap.add_argument("--scale", type=float, default=0.05, help="regression data scale")
    ap.add_argument("--stage-timeout", type=int, default=3600)
    args = ap.parse_args(argv)
    args.out = os.path.abspath(args.out)
    res = run(args)
    for s, r in res.items():
        print(f"{s:11s} {r['status']:4s} {r.get('seconds', '')} {r.get('reason', '')}")
    return 1 if any(r["status"] == "FAIL" for r in res.values()) else 0


if __name__ == "__main__":
    sys.exit(main())

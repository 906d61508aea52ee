#!/usr/bin/env python3
"""Regression harness: run a test matrix of shuffle jobs, validate them, analyze the logs, report.

The reference's harness (scripts/regression/autoTester.sh and friends)
drives real Hadoop clusters from a CSV matrix: each test runs NSAMPLES times; job wall-clock
mean/stddev/min/max are reported (terasortAnallizer.sh:10-120); teravalidate checks the output
(mr-dstatExcel.sh:249-291); log analysis requires one provider/consumer version, as many
"closed" as "init" lines and no fallback (testStatusAnalyzer.sh:168-203); logs are collected per
test (utils/master/*.sh). This tool does the same on one node through uda_amd.models.jobs:

    python tools/regression.py --matrix benchmarks/regression_matrix.csv --out results/regress
    python tools/regression.py --matrix m.csv --only wordcount_cpu --samples 1 --scale 0.1

Matrix columns: name, program (terasort|wordcount|secondary), maps, reducers, gb, codec
(none|snappy|lzo), backend (cpu|gpu), approach (1 online | 2 hybrid), transport (loopback|tcp),
samples, plus any other ShuffleJobSpec field (e.g. gpu_merge_bytes). GPU rows are skipped when no
HIP device is visible (reported as SKIP, never as PASS).

Writes <out>/report.json, <out>/report.md and <out>/logs/<test>/sample<k>.log; exit status 1 if a
test failed.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import re
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VERSION_RE = re.compile(r"The version is (\S+)")


def analyze_logs(lines: list[str], reducers: int) -> list[str]:
    """Health checks of testStatusAnalyzer.sh on the native log lines of one sample."""
    errors = []
    prov = {m.group(1) for ln in lines if "role=MOFSupplier" in ln for m in [VERSION_RE.search(ln)] if m}
    cons = {m.group(1) for ln in lines if "role=NetMerger" in ln for m in [VERSION_RE.search(ln)] if m}
    if not prov or not cons:
        errors.append("provider or consumers were not loaded")
    elif prov != cons or len(prov) != 1:
        errors.append(f"providers/consumers report different versions: {sorted(prov | cons)}")
    opened = sum("role=NetMerger" in ln for ln in lines)
    closed = sum("reduce task closed" in ln for ln in lines)
    if opened != reducers or closed != opened:
        errors.append(f"{opened} reduce tasks started, {closed} closed, {reducers} expected")
    if any("[consumer 2]" in ln or "[consumer 1]" in ln for ln in lines):
        errors.append("error lines in the consumer log")
    return errors


def summarize(xs: list[float]) -> dict:
    if not xs:
        return {}
    return {"mean": statistics.fmean(xs), "stddev": statistics.pstdev(xs) if len(xs) > 1 else 0.0,
            "min": min(xs), "max": max(xs)}


def run_test(row: dict, samples: int, scale: float, out_dir: str, gpu: bool, telemetry: float = 0.0) -> dict:
    from uda_amd.models.jobs import ShuffleJobSpec, run_job
    from uda_amd.utils.telemetry import Telemetry
    name = row["name"]
    spec_fields = {k: v for k, v in row.items() if k not in ("name", "samples")}
    spec = ShuffleJobSpec.from_dict(spec_fields)
    spec.gb *= scale
    res = {"name": name, "spec": row, "samples": []}
    if spec.backend == "gpu" and not gpu:
        res["status"] = "SKIP"
        res["reason"] = "no HIP device visible"
        return res
    log_dir = os.path.join(out_dir, "logs", name)
    os.makedirs(log_dir, exist_ok=True)
    errors = []
    for k in range(samples):
        spec.seed = 7 + k
        # dstat-equivalent per-sample telemetry (mr-dstatExcel.sh:89-201)
        tel = Telemetry(os.path.join(log_dir, f"sample{k}.dstat.csv"), telemetry) if telemetry > 0 else None
        try:
            if tel:
                tel.start()
            r = run_job(spec)
        except Exception as e:  # noqa: BLE001  (a crashing sample is a failed test, keep going)
            errors.append(f"sample {k}: {type(e).__name__}: {e}")
            continue
        finally:
            if tel:
                tel.stop()
                res.setdefault("telemetry", []).append(tel.summary())
        with open(os.path.join(log_dir, f"sample{k}.log"), "w") as f:
            f.write("\n".join(r["logs"]) + "\n")
        health = analyze_logs(r["logs"], spec.reducers)
        if not r["valid"]:
            bad = [p for p in r["reducers"] if not p["valid"]]
            errors.append(f"sample {k}: validation failed {r['failures'] or bad[:1]}")
        errors += [f"sample {k}: {h}" for h in health]
        res["samples"].append({"wall_s": r["wall_s"], "gbps": r["gbps"], "bytes": r["bytes"], "valid": r["valid"],
                               "records": sum(p["records"] for p in r["reducers"])})
    res["wall_s"] = summarize([s["wall_s"] for s in res["samples"]])
    res["gbps"] = summarize([s["gbps"] for s in res["samples"]])
    res["status"] = "PASS" if not errors and res["samples"] else "FAIL"
    res["errors"] = errors
    return res


def write_report(results: list[dict], out_dir: str, meta: dict) -> None:
    with open(os.path.join(out_dir, "report.json"), "w") as f:
        json.dump({"meta": meta, "tests": results}, f, indent=1)
    lines = [f"# Regression report ({meta['date']})", "",
             f"host: {meta['host']}, GPU visible: {meta['gpu']}, samples: {meta['samples']}, scale: {meta['scale']}", "",
             "| test | status | GB | wall s (mean ± sd) | min / max s | GB/s (mean) | notes |",
             "|---|---|---|---|---|---|---|"]
    for r in results:
        w, g = r.get("wall_s") or {}, r.get("gbps") or {}
        gb = r["samples"][0]["bytes"] / 1e9 if r.get("samples") else 0
        note = r.get("reason") or "; ".join(r.get("errors", [])[:2])
        if w:
            lines.append(f"| {r['name']} | {r['status']} | {gb:.2f} | {w['mean']:.3f} ± {w['stddev']:.3f} | "
                         f"{w['min']:.3f} / {w['max']:.3f} | {g['mean']:.3f} | {note} |")
        else:
            lines.append(f"| {r['name']} | {r['status']} | - | - | - | - | {note} |")
    with open(os.path.join(out_dir, "report.md"), "w") as f:
        f.write("\n".join(lines) + "\n")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--matrix", default=os.path.join(os.path.dirname(__file__), "..", "benchmarks",
                                                     "regression_matrix.csv"))
    ap.add_argument("--out", default="results/regression")
    ap.add_argument("--only", action="append", default=[], help="run only these test names")
    ap.add_argument("--samples", type=int, default=0, help="override the matrix NSAMPLES")
    ap.add_argument("--scale", type=float, default=1.0, help="multiply every test's data size")
    ap.add_argument("--telemetry", type=float, default=0.0, metavar="SECONDS",
                    help="sample CPU/mem/disk/net/GPU every SECONDS into logs/<test>/sample<k>.dstat.csv")
    a = ap.parse_args(argv)
    from uda_amd import native
    gpu = native().device_count() > 0
    os.makedirs(a.out, exist_ok=True)
    with open(a.matrix) as f:
        rows = [r for r in csv.DictReader(f) if not a.only or r["name"] in a.only]
    results = []
    for row in rows:
        samples = a.samples or int(row.get("samples") or 1)
        t0 = time.perf_counter()
        r = run_test(row, samples, a.scale, a.out, gpu, a.telemetry)
        r["elapsed_s"] = time.perf_counter() - t0
        print(f"{r['status']:4s} {r['name']:28s} "
              + (f"{r['gbps']['mean']:.3f} GB/s" if r.get("gbps") else r.get("reason", "")), flush=True)
        for e in r.get("errors", []):
            print("     " + e, flush=True)
        results.append(r)
    meta = {"date": time.strftime("%Y-%m-%d %H:%M:%S"), "host": os.uname().nodename, "gpu": gpu,
            "samples": a.samples or "matrix", "scale": a.scale, "matrix": os.path.abspath(a.matrix)}
    write_report(results, a.out, meta)
    return 0 if all(r["status"] in ("PASS", "SKIP") for r in results) else 1


if __name__ == "__main__":
    sys.exit(main())

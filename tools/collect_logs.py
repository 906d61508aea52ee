#!/usr/bin/env python3
"""Log collector: gather native/job logs from every node (or rank) directory into one bundle.

Reference: utils/master/*.sh + utils/slave/*  ssh to every slave, copy the
UDA/TaskTracker logs of a job and grep snippets around errors. Here the "nodes" are directories:
per-rank log dirs (`-g` / `UDA_LOG_DIR`, files `uda<role>.log`), regression outputs
(`results/<run>/logs/<test>/sample<k>.log`), or a `gpurun_out/` tree merged back from a GPU box.

    python tools/collect_logs.py results/regression gpurun_out --out results/logbundle
    python tools/collect_logs.py /scratch/rank* --context 3 --tar

Writes <out>/summary.json and <out>/summary.md (per file: line count, counts per severity, the
UDA version lines, fallback/failure lines) plus <out>/snippets/<node>__<file>.txt holding every
ERROR/FATAL/failure line with `--context` lines around it. `--tar` also packs the collected logs
into <out>/logs.tar.gz. Exit status 1 when any file holds an ERROR/FATAL line or a fallback.
"""
from __future__ import annotations

import argparse
import fnmatch
import json
import os
import re
import sys
import tarfile

PATTERNS = ("uda*.log", "sample*.log", "*.log")
# "<date> <time> LEVEL [tid N] file:line func() msg" (log file sink), "[uda LEVEL] ..." (stderr),
# "[provider N] ..." / "[consumer N] ..." (Python sink: N is the reference's severity number)
SEV_RE = re.compile(r"(?:^\S+ \S+ (FATAL|ERROR|WARN|INFO|DEBUG|TRACE)\s)|(?:^\[uda (\w+)\])|"
                    r"(?:^\[(?:provider|consumer) (\d)\])")
SEV_NUM = {"1": "FATAL", "2": "ERROR", "3": "WARN", "4": "INFO", "5": "DEBUG", "6": "TRACE"}
VERSION_RE = re.compile(r"The version is (\S+)")
BAD_RE = re.compile(r"failure reported|failureInUda|fallbackPlugin|falling back to vanilla|Traceback|Segmentation fault|"
                    r"hipError|ncclInternalError|RCCL .*(abort|timeout)", re.IGNORECASE)


def severity(line: str) -> str | None:
    m = SEV_RE.search(line)
    if not m:
        return None
    if m.group(1):
        return m.group(1)
    if m.group(2):
        return m.group(2).upper()
    return SEV_NUM.get(m.group(3))


def find_logs(root: str, patterns=PATTERNS) -> list[str]:
    if os.path.isfile(root):
        return [root]
    out = []
    for d, _, files in os.walk(root):
        for f in sorted(files):
            if any(fnmatch.fnmatch(f, p) for p in patterns):
                out.append(os.path.join(d, f))
    return sorted(set(out))


def analyze_file(path: str, context: int) -> dict:
    with open(path, errors="replace") as f:
        lines = f.read().splitlines()
    counts: dict[str, int] = {}
    versions = set()
    hits = []
    for i, ln in enumerate(lines):
        s = severity(ln)
        if s:
            counts[s] = counts.get(s, 0) + 1
        m = VERSION_RE.search(ln)
        if m:
            versions.add(m.group(1))
        if s in ("ERROR", "FATAL") or BAD_RE.search(ln):
            hits.append(i)
    snippets = []
    last = -1
    for i in hits:
        lo, hi = max(0, i - context, last + 1), min(len(lines), i + context + 1)
        if lo > last + 1 and snippets:
            snippets.append("--")
        snippets += [f"{k + 1}: {lines[k]}" for k in range(lo, hi)]
        last = hi - 1
    return {"lines": len(lines), "severity": counts, "versions": sorted(versions), "problems": len(hits),
            "fallback": any(re.search(r"fallbackPlugin|failure reported|failureInUda", lines[i]) for i in hits),
            "snippet": snippets}


def node_name(root: str, path: str) -> str:
    rel = os.path.relpath(path, root) if os.path.isdir(root) else os.path.basename(path)
    base = os.path.basename(os.path.normpath(root)) or "root"
    return (base + "/" + rel).replace(os.sep, "/")


def collect(roots: list[str], out: str, context: int = 2, tar: bool = False) -> dict:
    os.makedirs(os.path.join(out, "snippets"), exist_ok=True)
    files = {}
    for root in roots:
        for p in find_logs(root):
            if os.path.abspath(p).startswith(os.path.abspath(out) + os.sep):
                continue  # never re-collect our own bundle
            files[node_name(root, p)] = (p, analyze_file(p, context))
    summary = {"files": {}, "versions": sorted({v for _, a in files.values() for v in a["versions"]}),
               "problem_files": 0}
    for name, (p, a) in sorted(files.items()):
        snip = a.pop("snippet")
        if snip:
            sp = os.path.join(out, "snippets", name.replace("/", "__") + ".txt")
            with open(sp, "w") as f:
                f.write("\n".join(snip) + "\n")
        a["path"] = p
        summary["files"][name] = a
        summary["problem_files"] += a["problems"] > 0
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    md = ["# Collected logs", "", f"{len(files)} file(s); UDA versions seen: {', '.join(summary['versions']) or '-'}",
          "", "| file | lines | ERROR | WARN | problems |", "|---|---|---|---|---|"]
    for name, a in summary["files"].items():
        sv = a["severity"]
        md.append(f"| {name} | {a['lines']} | {sv.get('ERROR', 0) + sv.get('FATAL', 0)} | {sv.get('WARN', 0)} | "
                  f"{a['problems']} |")
    if len(summary["versions"]) > 1:
        md += ["", "**Mixed UDA versions across nodes** (testStatusAnalyzer.sh treats this as a failure)."]
    with open(os.path.join(out, "summary.md"), "w") as f:
        f.write("\n".join(md) + "\n")
    if tar:
        with tarfile.open(os.path.join(out, "logs.tar.gz"), "w:gz") as t:
            for name, (p, _) in sorted(files.items()):
                t.add(p, arcname=name)
    return summary


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("roots", nargs="+", help="node/rank log directories, regression outputs or log files")
    ap.add_argument("--out", default="results/logbundle")
    ap.add_argument("--context", type=int, default=2, help="lines of context around each problem line")
    ap.add_argument("--tar", action="store_true", help="also write logs.tar.gz of every collected file")
    args = ap.parse_args(argv)
    s = collect(args.roots, args.out, args.context, args.tar)
    print(f"{len(s['files'])} log file(s), {s['problem_files']} with problems -> {args.out}/summary.md")
    return 1 if s["problem_files"] or len(s["versions"]) > 1 else 0


if __name__ == "__main__":
    sys.exit(main())

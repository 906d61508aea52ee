"""Aux tooling on the CPU: the log collector (reference utils/master + utils/slave)
and the nightly pipeline driver (reference scripts/build, B4)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import collect_logs  # noqa: E402
import nightly  # noqa: E402


def _node(tmp_path, name, lines):
    d = tmp_path / name
    d.mkdir()
    (d / "udaNetMerger.log").write_text("\n".join(lines) + "\n")
    return d


def test_collect_logs_flags_errors_and_mixed_versions(tmp_path):
    good = _node(tmp_path, "node1", [
        "2026-01-01 10:00:00.001 INFO  [tid 7] supplier.cc:10 start() UDA: The version is v1 role=MOFSupplier",
        "2026-01-01 10:00:00.002 INFO  [tid 7] reduce_task.cc:20 run() reduce task closed",
    ])
    bad = _node(tmp_path, "node2", [
        "[consumer 4] x UDA: The version is v2 role=NetMerger",
        "[consumer 4] fetching",
        "[consumer 2] reduce_task.cc:99 fetch() fetch failed: peer reset",
        "[uda ERROR] error.cc:5 report() failure reported: fetch failed",
        "[consumer 4] after",
    ])
    out = tmp_path / "bundle"
    rc = collect_logs.main([str(good), str(bad), "--out", str(out), "--context", "1", "--tar"])
    s = json.load(open(out / "summary.json"))
    assert rc == 1
    assert s["versions"] == ["v1", "v2"] and s["problem_files"] == 1
    f2 = s["files"]["node2/udaNetMerger.log"]
    assert f2["severity"]["ERROR"] == 2 and f2["severity"]["INFO"] == 3 and f2["fallback"]
    assert s["files"]["node1/udaNetMerger.log"]["problems"] == 0
    snip = (out / "snippets" / "node2__udaNetMerger.log.txt").read_text()
    assert "2: [consumer 4] fetching" in snip and "5: [consumer 4] after" in snip
    assert "Mixed UDA versions" in (out / "summary.md").read_text()
    assert (out / "logs.tar.gz").stat().st_size > 0
    # re-collecting a tree that contains the bundle does not pick the bundle up
    s2 = collect_logs.collect([str(tmp_path)], str(out))
    assert all(not k.startswith("tmp") or "bundle" not in k for k in s2["files"])


def test_collect_logs_clean_tree_passes(tmp_path):
    d = _node(tmp_path, "n", ["[provider 4] UDA: The version is v1 role=MOFSupplier"])
    assert collect_logs.main([str(d), "--out", str(tmp_path / "o")]) == 0


def test_nightly_reports_skips_and_stage_status(tmp_path):
    out = tmp_path / "nightly"
    rc = nightly.main(["--out", str(out), "--stages", "java,sanitizers,logs"])
    rep = json.load(open(out / "nightly.json"))
    st = {k: v["status"] for k, v in rep["stages"].items()}
    assert rc == 0 and set(st.values()) == {"SKIP"}, st  # no javac / not requested / no regression
    assert "| sanitizers | SKIP |" in (out / "nightly.md").read_text()


def test_nightly_build_stage_installs_release(tmp_path):
    out = tmp_path / "nightly"
    assert nightly.main(["--out", str(out), "--stages", "build"]) == 0
    rep = json.load(open(out / "nightly.json"))
    assert rep["stages"]["build"]["status"] == "PASS"
    assert os.path.exists(os.path.join(ROOT, "uda_amd", "lib", "libuda.so"))


def test_telemetry_sampler_writes_csv(tmp_path):
    import csv
    import time

    from uda_amd.utils.telemetry import Telemetry
    path = tmp_path / "t.csv"
    with Telemetry(str(path), interval=0.05) as t:
        time.sleep(0.3)
    rows = list(csv.DictReader(open(path)))
    assert len(rows) >= 3 and float(rows[-1]["t_s"]) >= 0.25
    s = t.summary()
    assert s["samples"] == len(rows) and s["cpu_pct"]["peak"] >= 0 and s["mem_used_gb"]["mean"] > 0


def test_regression_records_telemetry(tmp_path):
    import regression
    m = tmp_path / "m.csv"
    m.write_text("name,program,maps,reducers,gb,codec,backend,approach,transport,samples\n"
                 "wc,wordcount,3,2,0.002,none,cpu,1,loopback,1\n")
    out = tmp_path / "out"
    assert regression.main(["--matrix", str(m), "--out", str(out), "--telemetry", "0.05"]) == 0
    assert (out / "logs" / "wc" / "sample0.dstat.csv").exists()
    rep = json.load(open(out / "report.json"))
    assert rep["tests"][0]["telemetry"][0]["samples"] >= 1

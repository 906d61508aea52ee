"""The regression harness (tools/regression.py) and the job runner it drives, on the CPU backends:
a scaled-down matrix must pass end to end (teravalidate + log health), the log analyzer must flag
the reference harness's failure patterns, and the native stream validator must catch framing and
order errors."""
import csv
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import regression  # noqa: E402

from uda_amd.utils.ifile import encode_stream, text  # noqa: E402


def test_matrix_end_to_end(tmp_path):
    m = tmp_path / "m.csv"
    rows = [
        dict(name="wc", program="wordcount", maps=6, reducers=3, gb=0.004, codec="none", backend="cpu", approach=1,
             transport="loopback", samples=2),
        dict(name="ts_hybrid_lzo", program="terasort", maps=9, reducers=2, gb=0.004, codec="lzo", backend="cpu",
             approach=2, transport="loopback", samples=1),
        dict(name="ss_tcp", program="secondary", maps=5, reducers=2, gb=0.003, codec="snappy", backend="cpu",
             approach=1, transport="tcp", samples=1),
        dict(name="gpu_row", program="terasort", maps=4, reducers=1, gb=0.001, codec="none", backend="gpu",
             approach=1, transport="loopback", samples=1),
    ]
    with open(m, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    out = tmp_path / "out"
    rc = regression.main(["--matrix", str(m), "--out", str(out)])
    rep = json.load(open(out / "report.json"))
    status = {t["name"]: t["status"] for t in rep["tests"]}
    assert rc == 0, rep
    assert status["wc"] == status["ts_hybrid_lzo"] == status["ss_tcp"] == "PASS"
    assert status["gpu_row"] in ("SKIP", "PASS")  # SKIP here (no HIP device), never a silent pass
    wc = next(t for t in rep["tests"] if t["name"] == "wc")
    assert len(wc["samples"]) == 2 and set(wc["wall_s"]) == {"mean", "stddev", "min", "max"}
    assert (out / "logs" / "wc" / "sample1.log").read_text().count("The version is") == 4  # provider + 3
    assert "| wc | PASS |" in (out / "report.md").read_text()


def test_log_analyzer_flags_reference_failure_patterns():
    ok = ["[provider 4] x UDA: The version is v1 role=MOFSupplier",
          "[consumer 4] x UDA: The version is v1 role=NetMerger", "[consumer 4] reduce task closed: {}"]
    assert regression.analyze_logs(ok, 1) == []
    mixed = ok[:1] + ["[consumer 4] x UDA: The version is v2 role=NetMerger", ok[2]]
    assert "different versions" in regression.analyze_logs(mixed, 1)[0]
    assert "started" in regression.analyze_logs(ok[:2], 1)[0]  # opened but never closed
    assert "not loaded" in regression.analyze_logs(ok[1:], 1)[0]
    assert any("error lines" in e for e in regression.analyze_logs(ok + ["[consumer 2] boom"], 1))


def test_stream_validator_catches_errors(native):
    T = "org.apache.hadoop.io.Text"
    recs = [(text(b"a%03d" % i), b"v" * (i % 7)) for i in range(50)]
    s = encode_stream(recs)
    v = native.StreamValidator(T)
    v.feed(s[:120])
    assert v.framing_errors == 1  # a record split across two buffers
    v = native.StreamValidator(T)
    v.feed(encode_stream(list(reversed(recs))))
    assert v.order_errors == 49 and v.eof
    v = native.StreamValidator(T)
    v.feed(s)
    v.feed(b"\x01")
    assert v.framing_errors == 1  # data after EOF
    n_rec, n_bytes, ck = native.ifile_checksum(s)
    assert n_rec == 50 and n_bytes == len(s) - 2
    v = native.StreamValidator(T)
    half = len(encode_stream(recs[:25], eof=False))
    v.feed(s[:half])
    v.feed(s[half:])
    assert v.records == 50 and v.checksum == ck and v.eof and v.order_errors == 0 and v.framing_errors == 0

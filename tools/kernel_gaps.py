"""Timeline of one merge from a rocprofv3 kernel trace: every kernel from the last launch of `--first`
to the next `--last`, with its start offset, duration and the idle gap before it.

usage: python tools/kernel_gaps.py <kernel_trace.csv> --first f1_fn_kernel --last gather_var_kernel"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", required=True)
    ap.add_argument("--last", required=True)
    ap.add_argument("--occurrence", type=int, default=-1, help="which launch of --first starts the window")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.first in r[2]]
    i0 = starts[a.occurrence]
    i1 = next(i for i in range(i0, len(rows)) if a.last in rows[i][2])
    t0 = rows[i0][0]
    busy, prev_end = 0, rows[i0][0]
    print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>8}  kernel")
    for s, e, n in rows[i0:i1 + 1]:
        gap = max(0, s - prev_end)
        short = n.replace("(anonymous namespace)::", "").replace("uda::gpu::", "").split("(")[0]
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap / 1e3:8.1f}  {short[:70]}")
        busy += e - max(s, prev_end) if e > prev_end else 0
        prev_end = max(prev_end, e)
    span = prev_end - t0
    print(f"span {span / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()

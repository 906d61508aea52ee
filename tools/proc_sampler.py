"""Samples another process's threads from outside it: every --every-ms, the state and kernel wait channel of
each thread of the first process that has --match as one of its arguments; prints a sample when at least
--min-blocked threads are in uninterruptible sleep (D) or any is stopped (T, t: job control or a tracer),
with the count of threads per state and every running, blocked or stopped thread (name, state, wait
channel); and any late wake-up of the sampler itself. An outside reader needs nothing of the sampled
process (its address-space lock included), so it keeps sampling while that process is frozen;
CLOCK_BOOTTIME ms, as UDA_START_TRACE.

    python3 tools/proc_sampler.py --match=--daemon-fd --seconds 90 > gpurun_out/sampler.txt &
"""
import argparse
import os
import sys
import time


def now():
    return time.clock_gettime(time.CLOCK_BOOTTIME) * 1e3


def read(path):
    try:
        with open(path, "rb") as f:
            return f.read().decode(errors="replace").strip()
    except OSError:
        return ""


def find(match, me):  # a process with `match` as one of its arguments (not inside a longer one)
    for d in os.listdir("/proc"):
        if d.isdigit() and int(d) != me:
            try:
                with open(f"/proc/{d}/cmdline", "rb") as f:
                    argv = f.read().decode(errors="replace").split("\0")
            except OSError:
                continue
            if match in argv[1:]:
                return int(d)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--match", required=True)
    ap.add_argument("--seconds", type=float, default=90.0)
    ap.add_argument("--every-ms", type=float, default=5.0)
    ap.add_argument("--min-blocked", type=int, default=4)
    a = ap.parse_args()
    end = now() + a.seconds * 1e3
    pid = None
    while pid is None and now() < end:
        pid = find(a.match, os.getpid())
        time.sleep(0.05)
    if pid is None:
        print("[proc-sampler] no process matches", flush=True)
        return 1
    print(f"[proc-sampler] pid {pid} at {now():.3f}", flush=True)
    printed = 0
    last = now()
    while now() < end and printed < 20000 and os.path.exists(f"/proc/{pid}"):
        t = now()
        rows = []
        try:
            tids = os.listdir(f"/proc/{pid}/task")
        except OSError:
            break
        counts = {}
        for tid in tids:
            st = read(f"/proc/{pid}/task/{tid}/stat")
            rp = st.rfind(")")
            if rp < 0 or rp + 2 >= len(st):
                continue
            s = st[rp + 2]
            counts[s] = counts.get(s, 0) + 1
            if s in "RDTt":
                rows.append((s, tid, read(f"/proc/{pid}/task/{tid}/comm"), read(f"/proc/{pid}/task/{tid}/wchan")))
        took = now() - t
        if t - last > 4 * a.every_ms + 20:  # this sampler itself held up
            print(f"[proc-sampler] {t:.3f} own gap {t - last:.1f} ms", flush=True)
        last = t
        stopped = counts.get("T", 0) + counts.get("t", 0)
        if counts.get("D", 0) >= a.min_blocked or stopped:
            hist = " ".join(f"{k}:{v}" for k, v in sorted(counts.items()))
            print(f"[proc-sampler] {t:.3f} (sweep {took:.1f} ms) states {hist}", flush=True)
            for s, tid, comm, wchan in sorted(rows)[:40]:
                print(f"[proc-sampler] {t:.3f} tid {tid} {comm} {s} wchan {wchan}", flush=True)
                printed += 1
        time.sleep(max(0.0, a.every_ms / 1e3 - (now() - t) / 1e3))
    print(f"[proc-sampler] end {now():.3f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

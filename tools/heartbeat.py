"""A 1 ms heartbeat: prints every wake-up more than --gap-ms late (CLOCK_BOOTTIME ms, as UDA_START_TRACE
and UDA_STALL_PROBE stamp), to tell a stall of one process from one of the whole machine or cgroup.

    python3 tools/heartbeat.py --seconds 60 > gpurun_out/heartbeat.txt &
"""
import argparse
import sys
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--gap-ms", type=float, default=20.0)
    a = ap.parse_args()
    now = lambda: time.clock_gettime(time.CLOCK_BOOTTIME) * 1e3
    end = now() + a.seconds * 1e3
    last = now()
    print(f"[heartbeat] start {last:.3f}", flush=True)
    while last < end:
        time.sleep(0.001)
        t = now()
        if t - last > a.gap_ms:
            print(f"[heartbeat] {t:.3f} gap {t - last:.1f} ms", flush=True)
        last = t
    print(f"[heartbeat] end {last:.3f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

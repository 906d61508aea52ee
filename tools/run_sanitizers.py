#!/usr/bin/env python3
"""Host-code sanitizer runs (SURVEY.md §5 "Race detection / sanitizers").

For each of address / undefined / thread: build libuda.so + the pybind11 module with
`-Xarch_host -fsanitize=<s>` (device code is never instrumented: no GPU sanitizers on this pool),
run the CPU test suite with the matching clang runtime preloaded into Python, and report the
sanitizer findings; the release build is restored at the end.

  python tools/run_sanitizers.py [--only thread] [--tests tests/test_bridge_loopback.py ...]
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = {
    "address": ("libclang_rt.asan-x86_64.so", {"ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1"}),
    "undefined": ("libclang_rt.ubsan_standalone-x86_64.so", {"UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
    "thread": ("libclang_rt.tsan-x86_64.so", {"TSAN_OPTIONS": "halt_on_error=0:report_signal_unsafe=0"}),
}
# torch's own gloo threads are not instrumented and trip TSan; the thread run covers our runtime
DEFAULT_TESTS = {
    "thread": ["tests/test_bridge_loopback.py", "tests/test_codec.py", "tests/test_jni_shim.py",
               "tests/test_properties.py", "tests/test_dist_cpu.py::test_tcp_transport_across_processes"],
}


def runtime(name: str) -> str:
    clang = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin", "clang++")
    out = subprocess.run([clang, f"-print-file-name={name}"], capture_output=True, text=True, check=True)
    return out.stdout.strip()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=sorted(RT), action="append")
    ap.add_argument("--tests", nargs="*")
    a = ap.parse_args()
    failed = []
    try:
        for san in a.only or ["address", "undefined", "thread"]:
            lib, opts = RT[san]
            subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build.py"), "--sanitize", san], check=True)
            logdir = tempfile.mkdtemp(prefix=f"uda_{san}_")
            env = dict(os.environ, LD_PRELOAD=runtime(lib))
            for k, v in opts.items():
                env[k] = v + f":log_path={logdir}/log"
            tests = a.tests or DEFAULT_TESTS.get(san, ["tests"])
            r = subprocess.run([sys.executable, "-m", "pytest", *tests, "-q", "-m", "not gpu", "-p", "no:cacheprovider"],
                               cwd=ROOT, env=env)
            reports = glob.glob(os.path.join(logdir, "log*"))
            print(f"[{san}] pytest rc={r.returncode}, sanitizer reports: {len(reports)} ({logdir})", flush=True)
            if r.returncode != 0 or reports:
                failed.append(san)
    finally:
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build.py")], check=True)
    print("sanitizers clean" if not failed else f"findings under: {failed}")
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())

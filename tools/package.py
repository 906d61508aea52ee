#!/usr/bin/env python3
"""Binary distribution of the framework (reference: build/buildrpm.sh, build/uda.spec,
build/debian/*).

    python tools/package.py                 # dist/uda-amd-<version>-gfx950.tar.gz
    python tools/package.py --rpm           # + rpmbuild -tb with packaging/uda-amd.spec (if rpmbuild exists)

Layout of the tarball (installs under /usr/lib64/uda-amd like the reference's /usr/lib64/uda):
    lib/libuda.so                      native runtime + JNI entry points (gfx950 code objects inside)
    lib/uda-amd-hadoop-*.jar           Hadoop plugin jars, when java/build.sh produced them
    java/                              plugin sources (build them against the cluster's Hadoop)
    python/uda_amd/                    Python package incl. the pybind11 module
    bin/uda_mof_supplier               the node daemon libuda.so starts (found at <libuda dir>/../bin)
    bin/uda_reduce_task                a reduce task in a process of its own (node-shape runs, tests)
    bin/uda-regression, bin/uda-bench  entry points
    share/doc/                         README, ARCHITECTURE, BENCHMARKS
    VERSION                            version string reported by libuda.so ("The version is ...")
The build step is tools/build.py; nothing is downloaded.
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
import tarfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VERSION = "0.1.0"


def stage(dest: str) -> None:
    lib = os.path.join(ROOT, "uda_amd", "lib", "libuda.so")
    if not os.path.exists(lib):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build.py")], check=True)
    os.makedirs(os.path.join(dest, "lib"))
    shutil.copy2(lib, os.path.join(dest, "lib"))
    for jar in glob.glob(os.path.join(ROOT, "build", "java", "*.jar")):
        shutil.copy2(jar, os.path.join(dest, "lib"))
    shutil.copytree(os.path.join(ROOT, "java"), os.path.join(dest, "java"))
    shutil.copytree(os.path.join(ROOT, "uda_amd"), os.path.join(dest, "python", "uda_amd"),
                    ignore=shutil.ignore_patterns("__pycache__", "*.pyc"))
    os.makedirs(os.path.join(dest, "bin"))
    for exe in ("uda_mof_supplier", "uda_reduce_task"):  # next to lib/: NodeDaemonClient::default_exe
        shutil.copy2(os.path.join(ROOT, "uda_amd", "bin", exe), os.path.join(dest, "bin", exe))
    for name, target in (("uda-regression", "tools/regression.py"), ("uda-bench", "bench.py")):
        src = os.path.join(ROOT, target)
        shutil.copy2(src, os.path.join(dest, "bin", os.path.basename(target)))
        with open(os.path.join(dest, "bin", name), "w") as f:
            f.write("#!/bin/sh\nhere=$(dirname \"$0\")\nPYTHONPATH=\"$here/../python:$PYTHONPATH\" "
                    f"exec python3 \"$here/{os.path.basename(target)}\" \"$@\"\n")
        os.chmod(os.path.join(dest, "bin", name), 0o755)
    docs = os.path.join(dest, "share", "doc")
    os.makedirs(docs)
    for d in ("README.md", "docs/ARCHITECTURE.md", "docs/BENCHMARKS.md", "java/README.md"):
        shutil.copy2(os.path.join(ROOT, d), os.path.join(docs, d.replace("/", "_")))
    with open(os.path.join(dest, "VERSION"), "w") as f:
        f.write(VERSION + "\n")


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default=os.path.join(ROOT, "dist"))
    ap.add_argument("--rpm", action="store_true")
    a = ap.parse_args()
    name = f"uda-amd-{VERSION}"
    work = os.path.join(a.out, "stage")
    shutil.rmtree(work, ignore_errors=True)
    stage(os.path.join(work, name))
    shutil.copy2(os.path.join(ROOT, "packaging", "uda-amd.spec"), os.path.join(work, name, "uda-amd.spec"))
    tgz = os.path.join(a.out, f"{name}-gfx950.tar.gz")
    with tarfile.open(tgz, "w:gz") as t:
        t.add(os.path.join(work, name), arcname=name)
    shutil.rmtree(work)
    print(tgz)
    if a.rpm:
        if not shutil.which("rpmbuild"):
            print("rpmbuild not found: tarball only", file=sys.stderr)
            return 0
        subprocess.run(["rpmbuild", "-tb", tgz], check=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Build the native runtime in-tree for gfx950 (MI355X).

Produces
  uda_amd/lib/libuda.so                    -- the native library (C ABI `uda_*` + engine + HIP kernels +
                                              the UdaBridge JNI entry points, declared in-tree, no JDK needed)
  uda_amd/_uda_native<EXT_SUFFIX>          -- pybind11 module linked against libuda.so

Everything is compiled with hipcc (`--offload-arch=gfx950`); `.hip` files carry device code, `.cc`
files are host C++. A build.ninja is generated under build/ and ninja does the incremental,
parallel work (MAX_JOBS / -j, default 8).
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def sources() -> tuple[list[str], list[str]]:
    lib = []
    for pat in ("common/*.cc", "engine/*.cc", "provider/*.cc", "consumer/*.cc", "transport/*.cc",
                "io/*.cc", "codec/*.cc", "gpu/*.cc", "gpu/*.hip", "service/*.cc", "bridge/*.cc"):
        lib += sorted(glob.glob(os.path.join(ROOT, "csrc", pat)))
    mod = sorted(glob.glob(os.path.join(ROOT, "csrc", "python", "*.cc")))
    return lib, mod


def app_sources() -> list[str]:
    """Executables: csrc/apps/<name>_main.cc -> uda_amd/bin/uda_<name>, linked against libuda.so."""
    return sorted(glob.glob(os.path.join(ROOT, "csrc", "apps", "*_main.cc")))


def app_name(src: str) -> str:
    return "uda_" + os.path.basename(src)[: -len("_main.cc")]


def installed_outputs() -> list[str]:
    ext = sysconfig.get_config_var("EXT_SUFFIX")
    return ([os.path.join(ROOT, "uda_amd", "lib", "libuda.so"), os.path.join(ROOT, "uda_amd", "_uda_native" + ext)] +
            [os.path.join(ROOT, "uda_amd", "bin", app_name(s)) for s in app_sources()])


def staged_outputs(build_dir: str) -> list[str]:
    ext = sysconfig.get_config_var("EXT_SUFFIX")
    return ([os.path.join(build_dir, "lib", "libuda.so"), os.path.join(build_dir, "_uda_native" + ext)] +
            [os.path.join(build_dir, "bin", app_name(s)) for s in app_sources()])


def install(build_dir: str) -> None:
    """Copy the flavour's link outputs in-tree; os.replace keeps a running process's mapping valid."""
    for src, dst in zip(staged_outputs(build_dir), installed_outputs()):
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        tmp = dst + ".tmp"
        shutil.copy2(src, tmp)
        os.replace(tmp, dst)


def write_ninja(build_dir: str, debug: bool, sanitize: str | None) -> str:
    import pybind11

    lib_srcs, mod_srcs = sources()
    opt = "-O1 -g" if debug else "-O3 -g1"
    common = (f"-std=c++17 -fPIC {opt} -Wall -Wno-unused-function -Wno-unused-variable "
              f"-Wno-unused-command-line-argument -Wno-pass-failed "
              f"-I{ROOT}/csrc/include -I{ROOT}/csrc -I{ROOT}/csrc/gpu -I{ROCM}/include "
              f"-D__HIP_PLATFORM_AMD__=1")
    host_san = ""
    if sanitize:
        # sanitizers apply to host code only (no GPU ASan on this pool)
        host_san = f" -Xarch_host -fsanitize={sanitize} -fno-omit-frame-pointer"
    py_inc = f"-I{pybind11.get_include()} -I{sysconfig.get_paths()['include']}"
    # link inside the flavour's build dir; install() copies into uda_amd/ (ninja alone would keep
    # a stale in-tree .so written by another flavour, its mtime being newer than our objects)
    lib_out, mod_out = staged_outputs(build_dir)[:2]
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    lines = [
        "ninja_required_version = 1.5",
        f"hipcc = {hipcc}",
        f"cflags = {common}{host_san}",
        f"pyflags = {py_inc}",
        f"rule hip\n  command = $hipcc -x hip --offload-arch={ARCH} $cflags -MD -MF $out.d -c $in -o $out\n"
        f"  depfile = $out.d\n  deps = gcc\n  description = HIPCC $in",
        f"rule cxx\n  command = $hipcc --offload-arch={ARCH} $cflags -MD -MF $out.d -c $in -o $out\n"
        f"  depfile = $out.d\n  deps = gcc\n  description = CXX $in",
        f"rule cxxpy\n  command = $hipcc --offload-arch={ARCH} $cflags $pyflags -MD -MF $out.d -c $in -o $out\n"
        f"  depfile = $out.d\n  deps = gcc\n  description = CXX(py) $in",
        f"rule solib\n  command = $hipcc -shared -fPIC --offload-arch={ARCH}{host_san} $in -o $out "
        f"-L{ROCM}/lib -lrccl -lamdhip64 -lhsa-runtime64 -lpthread -ldl -Wl,-rpath,{ROCM}/lib -Wl,-soname,libuda.so\n"
        f"  description = LINK $out",
        f"rule pymod\n  command = $hipcc -shared -fPIC{host_san} $in -o $out -L{os.path.dirname(lib_out)} "
        f"-luda -Wl,-rpath,'$$ORIGIN/lib' -L{ROCM}/lib -lamdhip64\n  description = LINK $out",
        f"rule app\n  command = $hipcc{host_san} $in -o $out -L{os.path.dirname(lib_out)} "
        f"-luda -Wl,-rpath,'$$ORIGIN/../lib' -L{ROCM}/lib -lamdhip64 -lpthread -Wl,-rpath,{ROCM}/lib\n"
        f"  description = LINK $out",
    ]
    objs = []
    for s in lib_srcs:
        rel = os.path.relpath(s, os.path.join(ROOT, "csrc"))
        o = os.path.join(build_dir, rel + ".o")
        rule = "hip" if s.endswith(".hip") else "cxx"
        lines.append(f"build {o}: {rule} {s}")
        objs.append(o)
    mobjs = []
    for s in mod_srcs:
        rel = os.path.relpath(s, os.path.join(ROOT, "csrc"))
        o = os.path.join(build_dir, rel + ".o")
        lines.append(f"build {o}: cxxpy {s}")
        mobjs.append(o)
    lines.append(f"build {lib_out}: solib {' '.join(objs)}")
    lines.append(f"build {mod_out}: pymod {' '.join(mobjs)} | {lib_out}")
    apps = []
    for s, out in zip(app_sources(), staged_outputs(build_dir)[2:]):
        rel = os.path.relpath(s, os.path.join(ROOT, "csrc"))
        o = os.path.join(build_dir, rel + ".o")
        lines.append(f"build {o}: cxx {s}")
        lines.append(f"build {out}: app {o} | {lib_out}")
        apps.append(out)
    os.makedirs(os.path.join(build_dir, "bin"), exist_ok=True)
    lines.append(f"default {mod_out} {' '.join(apps)}")
    path = os.path.join(build_dir, "build.ninja")
    os.makedirs(build_dir, exist_ok=True)
    os.makedirs(os.path.dirname(lib_out), exist_ok=True)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def build(jobs: int | None = None, debug: bool = False, sanitize: str | None = None,
          verbose: bool = False) -> None:
    build_dir = os.path.join(ROOT, "build", "san-" + sanitize if sanitize else ("debug" if debug else "release"))
    write_ninja(build_dir, debug, sanitize)
    jobs = jobs or int(os.environ.get("MAX_JOBS", "8"))
    ninja = shutil.which("ninja") or "ninja"
    cmd = [ninja, "-C", build_dir, f"-j{min(jobs, 16)}"]
    if verbose:
        cmd.append("-v")
    subprocess.run(cmd, check=True)
    install(build_dir)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--sanitize", default=None, help="host-only sanitizer, e.g. address or thread")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    build(a.jobs, a.debug, a.sanitize, a.verbose)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Packaging (offline): `pip install --no-build-isolation .` builds the native runtime in-tree with
tools/build.py (hipcc, gfx950) and installs the `uda_amd` package with libuda.so and the pybind11
module as package data. `python setup.py build_native` only builds."""
import os
import subprocess
import sys

from setuptools import Command, find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


def _build_native():
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build.py")], check=True, cwd=ROOT)


class BuildNative(Command):
    description = "build libuda.so and the pybind11 module for gfx950"
    user_options = []

    def initialize_options(self):
        pass

    def finalize_options(self):
        pass

    def run(self):
        _build_native()


class BuildPy(build_py):
    def run(self):
        _build_native()
        super().run()


setup(
    name="uda_amd",
    version="0.1.0",
    description="MI355X-native MapReduce shuffle/merge engine (UDA-compatible UdaBridge API)",
    packages=find_packages(include=["uda_amd", "uda_amd.*"]),
    package_data={"uda_amd": ["lib/libuda.so", "_uda_native*.so"]},
    python_requires=">=3.10",
    install_requires=["numpy", "torch"],
    cmdclass={"build_native": BuildNative, "build_py": BuildPy},
    zip_safe=False,
)

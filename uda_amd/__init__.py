"""uda_amd — an MI355X-native MapReduce shuffle/merge engine with UDA's capabilities.

Layers (see SURVEY.md §7 and docs/ARCHITECTURE.md):
  uda_amd._native      loader of the native runtime (C++ / HIP for gfx950 / RCCL)
  uda_amd.ops          Python views of the HIP kernels (key normalize, merge, serialize, decode)
  uda_amd.parallel     one-process-per-GPU bootstrap, RCCL ids, key-range round planning
  uda_amd.models       workloads ("model families"): TeraSort, WordCount, SecondarySort
  uda_amd.utils        IFile codec, J2CQueue-equivalent reader, synthetic data, validators
  uda_amd.bridge       the UdaBridge host API (fake JVM host over the C ABI)
"""
from ._native import available, native  # noqa: F401

__version__ = "0.1.0"

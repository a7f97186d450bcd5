"""kgpu -- MI355X-native node evaluation for kube-scheduler (host side of libkgpu.so).

Modules:
  api        v1 object accessors, quantities, resource classes (host half of PreFilter)
  compile    objects -> dictionary-encoded SoA + pod queries (include/kgpu.h)
  abi        numpy/ctypes mirrors of the C ABI structs
  native     ctypes binding of libkgpu.so (no fallback: raises if the library is missing)
  framework  GpuFramework: the plugin-side mirror (cycle / scheduleOne loop)
  cluster    synthetic clusters for the BASELINE configs
"""
from .compile import Profile, Cluster, Compiler, CompileError  # noqa: F401

"""CPU checks of the drop-in boundary: libkgpu.so loads, exports every kgpu.h entry point, and the
Python ABI mirror has the C struct layout."""
import ctypes
import os
import re

from kgpu import abi, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "kgpu.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(kgpu_\w+)\(", src, re.M)))


def test_every_declared_symbol_is_exported():
    lib = ctypes.CDLL(native.LIB_PATH)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert set(declared_functions()) == set(native.EXPORTS)


def test_struct_layouts_match():
    assert native.check_layout()


def test_abi_version():
    assert native.lib().kgpu_abi_version() == abi.ABI_VERSION


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        return
    cfg = abi.Config()
    cfg.abi_version = abi.ABI_VERSION
    h = ctypes.c_void_p()
    rc = native.lib().kgpu_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc == abi.E_DEVICE


def test_allocation_failure_returns_error_code():
    """The exception barrier (include/kgpu.h conventions: no exception crosses the ABI): a host
    allocation failure injected inside kgpu_create comes back as KGPU_E_NOMEM, not as a C++
    exception unwinding into the caller (cgo would abort the scheduler)."""
    cfg = abi.Config()
    cfg.abi_version = abi.ABI_VERSION
    h = ctypes.c_void_p()
    native.debug_fail_alloc(1)
    try:
        rc = native.lib().kgpu_create(ctypes.byref(cfg), ctypes.byref(h))
    finally:
        native.debug_fail_alloc(0)
    assert rc == abi.E_NOMEM
    assert not h.value
    # the hook is spent: the next call reaches the device check again
    import torch
    if not torch.cuda.is_available():
        assert native.lib().kgpu_create(ctypes.byref(cfg), ctypes.byref(h)) == abi.E_DEVICE

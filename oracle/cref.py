"""ORACLE (test infrastructure only) -- ctypes binding of the C restatement (oracle/c/kgpu_ref.c).

Consumes the same compiled SoA inputs as libkgpu.so (include/kgpu.h).  Used by tests/ for
parity at sizes the pure-Python oracle cannot reach, and by bench.py's cpu_baseline leg.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# KGPU_REF_LIB: another build of the same source (tests/test_sanitizers.py loads the ASan/UBSan one)
LIB = os.environ.get("KGPU_REF_LIB") or os.path.join(HERE, "build", "libkgpu_ref.so")
_lib = None


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "c")])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.kgpu_ref_create.argtypes = [vp, vp, C.c_int, C.POINTER(vp)]
        L.kgpu_ref_destroy.argtypes = [vp]
        L.kgpu_ref_schedule.argtypes = [vp, vp, C.c_int, vp, C.c_int64, vp, vp, vp, vp]
        L.kgpu_ref_read_nodes.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.kgpu_ref_broken_linear.argtypes = [vp, vp, C.c_int, vp]
        _lib = L
    return _lib


def broken_linear(points, utilizations):
    """buildBrokenLinearFunction over unscaled `points` at `utilizations` (the C restatement)."""
    from kgpu import abi
    cfg = abi.Config()
    cfg.n_shape = len(points)
    for i, (u, sc) in enumerate(points):
        cfg.shape[i].utilization, cfg.shape[i].score = int(u), int(sc)
    p = np.ascontiguousarray(utilizations, np.int64)
    out = np.zeros(len(p), np.int64)
    if lib().kgpu_ref_broken_linear(C.addressof(cfg), p.ctypes.data, len(p), out.ctypes.data):
        raise ValueError("no shape points")
    return [int(x) for x in out]


class RefEngine:
    def __init__(self, config, snap, threads=1):
        self.h = C.c_void_p()
        self.n = snap.n_nodes
        lib().kgpu_ref_create(C.addressof(config), C.addressof(snap), threads, C.byref(self.h))

    def close(self):
        if self.h:
            lib().kgpu_ref_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def schedule(self, queries, pools, first_seq=0, diag=False):
        from kgpu import abi
        q = np.ascontiguousarray(queries, dtype=abi.QUERY)
        res = np.zeros(len(q), abi.RESULT)
        st = np.zeros(self.n, np.uint32) if diag else None
        raw = np.zeros((abi.NUM_SCORES, self.n), np.int64) if diag else None
        norm = np.zeros((abi.NUM_SCORES, self.n), np.int64) if diag else None
        lib().kgpu_ref_schedule(self.h, q.ctypes.data, len(q), C.addressof(pools), first_seq, res.ctypes.data,
                                st.ctypes.data if diag else None, raw.ctypes.data if diag else None,
                                norm.ctypes.data if diag else None)
        return (res, st, raw, norm) if diag else res

    def read_nodes(self):
        n = self.n
        cols = [np.zeros(n, np.int64) for _ in range(5)] + [np.zeros(n, np.int32)]
        lib().kgpu_ref_read_nodes(self.h, *[c.ctypes.data for c in cols])
        return dict(zip(["req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods"], cols))

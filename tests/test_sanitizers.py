"""AddressSanitizer + UndefinedBehaviorSanitizer over the C restatement (the reference
runs its tests under Go's -race, hack/make-rules/test.sh:71,165-166).

oracle/c is built a second time with -fsanitize=address,undefined (oracle/c/Makefile `sanitize`) and
loaded in a child interpreter with libasan preloaded; it schedules the configs (a)-(d) and (e) at
small sizes -- single-threaded and with the 16-worker parallelize.Until structure -- and must finish
without a sanitizer report and with the placements of the regular build."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np
sys.path[:0] = [%(root)r, %(root)r + "/kubernetes-1_amd"]
from kgpu import cluster
from kgpu.framework import GpuFramework
from oracle.cref import RefEngine
out = {}
for name, gen in (("a", lambda: cluster.scheduling_basic(n_nodes=120, n_init=0, n_pods=80)),
                  ("b", lambda: cluster.fit_least_balanced(n_nodes=300, n_pods=200)),
                  ("c", lambda: cluster.taints_affinity_spread(n_nodes=300, n_pods=120)),
                  ("d", lambda: cluster.pod_affinity(n_nodes=200, n_existing=200, n_pods=96)),
                  ("e", lambda: cluster.sharded_spread(n_nodes=400, n_pods=80))):
    w = gen()
    nodes, pods, prof = w[0], w[-2], w[-1]
    existing = w[1] if len(w) == 4 and name != "a" else []
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods[:16], create_engine=False)
    q, pc, _, errs = fw.compile_pods(pods)
    assert not errs
    for th in (1, 4):
        r = RefEngine(fw.config, fw.snap, threads=th).schedule(q, pc)
        out["%%s%%d" %% (name, th)] = r["node"]
np.savez(sys.argv[1], **out)
print("sanitized run ok")
"""


def _run(lib, out, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    env["KGPU_REF_LIB"] = lib
    code = CHILD % {"root": ROOT}
    return subprocess.run([sys.executable, "-c", code, out], env=env, capture_output=True, text=True, timeout=600)


def test_c_restatement_under_asan_ubsan(tmp_path):
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle", "c"), "all", "sanitize"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.exists(asan):
        pytest.skip("libasan not available")
    san_lib = os.path.join(ROOT, "oracle", "build", "libkgpu_ref_san.so")
    plain_lib = os.path.join(ROOT, "oracle", "build", "libkgpu_ref.so")
    got_p, want_p = str(tmp_path / "san.npz"), str(tmp_path / "plain.npz")
    # the ASan runtime goes first; whatever the environment already preloads stays preloaded after it
    pre = " ".join(x for x in (asan, os.environ.get("LD_PRELOAD", "")) if x)
    san = _run(san_lib, got_p, {"LD_PRELOAD": pre,
                                "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1:halt_on_error=1",
                                "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert san.returncode == 0 and "sanitized run ok" in san.stdout, (san.stdout[-2000:], san.stderr[-4000:])
    assert "runtime error" not in san.stderr and "AddressSanitizer" not in san.stderr, san.stderr[-4000:]
    plain = _run(plain_lib, want_p, {})
    assert plain.returncode == 0, plain.stderr[-2000:]
    got, want = np.load(got_p), np.load(want_p)
    assert sorted(got.files) == sorted(want.files)
    for k in want.files:
        assert np.array_equal(got[k], want[k]), k
        assert (want[k] >= 0).any(), k

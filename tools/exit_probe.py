"""Which library's exit handler faults after rocprofv3's tool finalization?

Runs one small step of a chosen variant, then copies /proc/self/maps to a file so that the
addresses of a crash report from the same process can be resolved to libraries:
  torch   -- torch only: one device tensor and a synchronize
  kgpu    -- libkgpu.so only (no torch import): create a context, upload 64 nodes, one batch, destroy
  both    -- torch first, then the kgpu variant
Usage: python3 tools/exit_probe.py <variant> <maps-out> [--os-exit]
  --os-exit: leave through os._exit(0) after the work (no exit handlers run: does rocprofv3 still write
             its files?  It does not: the tool finalizes in an exit handler)
  --no-persistent: no persistent (cooperative) launch, one k_eval launch per pod
  --no-coop: persistent kernels through ordinary launches (KGPU_OPT_COOPERATIVE = 0)
  --reset:   hipDeviceReset() before a normal exit (the runtime's queues and allocations released while
             the profiler is still attached)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "kubernetes-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def run_torch():
    import torch
    x = torch.zeros(1024, device="cuda")
    x += 1
    torch.cuda.synchronize()


def run_kgpu():
    from kgpu.cluster import fit_least_balanced
    from kgpu.framework import GpuFramework
    nodes, existing, pods, prof = fit_least_balanced(n_nodes=64, n_pods=32)
    fw = GpuFramework(prof, nodes, existing, pods_hint=pods, device=0)
    from kgpu import abi
    if "--no-persistent" in sys.argv:  # k_eval launches only: no cooperative launch in the process
        fw.engine.set_option(abi.OPT_PERSISTENT, 0)
    if "--no-coop" in sys.argv:  # the persistent kernels through ordinary launches
        fw.engine.set_option(abi.OPT_COOPERATIVE, 0)
    res = fw.schedule(pods, first_seq=0)
    assert (res["node"] >= 0).sum() > 0
    fw.engine.close()


def main():
    variant, out = sys.argv[1], sys.argv[2]
    if variant in ("torch", "both"):
        run_torch()
    if variant in ("kgpu", "both"):
        run_kgpu()
    with open("/proc/self/maps") as src, open(out, "w") as dst:
        dst.write(src.read())
    print("exit_probe %s: done, maps in %s" % (variant, out), flush=True)
    if "--reset" in sys.argv:
        # tear the HIP runtime's device state down now, while a profiler's tool is still alive
        import ctypes
        rc = ctypes.CDLL("libamdhip64.so").hipDeviceReset()
        print("exit_probe: hipDeviceReset rc=%d" % rc, flush=True)
    if "--os-exit" in sys.argv:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


if __name__ == "__main__":
    main()

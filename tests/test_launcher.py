"""bench.py --gpus N without a launcher starts its N rank processes itself (CPU: the gloo probe)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT", "KGPU_BENCH_LAUNCHER")}
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                         text=True, timeout=240)
    return out


def test_bench_spawns_n_ranks():
    out = _run(["--gpus", "3", "--probe-launch"])
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 alone prints
    rec = json.loads(lines[0])
    assert rec["world"] == 3 and rec["sum"] == 1 + 2 + 3
    assert sorted(r["rank"] for r in rec["ranks"]) == [0, 1, 2]
    assert sorted(r["local_rank"] for r in rec["ranks"]) == [0, 1, 2]
    assert len({r["pid"] for r in rec["ranks"]}) == 3
    assert rec["launcher"].startswith("bench.py --gpus 3")


def test_bench_under_external_launcher_does_not_spawn():
    """With WORLD_SIZE set (torch.distributed.run) the process is one rank: no children."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = _run(["--gpus", "1", "--probe-launch"], {"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0",
                                                   "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    assert out.returncode == 0, out.stderr
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["world"] == 1 and rec["launcher"] == "external"


def test_failing_rank_fails_the_launch():
    """A rank that dies ends the launch with its exit code; the rank left waiting in the
    rendezvous is ended instead of hanging the launch."""
    import time
    t = time.time()
    out = _run(["--gpus", "2", "--probe-launch"], {"KGPU_PROBE_FAIL_RANK": "1"})
    assert out.returncode == 3
    assert time.time() - t < 120

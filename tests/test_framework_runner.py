"""The reference's framework runner table TestFilterPlugins (framework_test.go:838, tests/golden/
framework.json) on the device.

The table's test plugins return injected codes.  The device evaluates real plugins, so each injected
outcome is realised by a real filter plugin that yields exactly that code on the table's one node:
Success -> NodeName (the pod names no node), then NodePorts (it asks for no host port),
Unschedulable -> NodeResourcesFit (the pod asks for more
cpu than the node has: "Insufficient cpu"), UnschedulableAndUnresolvable -> NodeUnschedulable (an
unschedulable node).  The device's status word must then name the same plugin position and code as
RunFilterPlugins + Merge does for the test plugins.

Not on the device, and why:
  * rows injecting Error: the device's filters never return Error -- the Go runner turns any code
    other than Unschedulable(AndUnresolvable) into an Error itself (framework.go:486-492), and that
    code stays in the Go framework around the plugin;
  * runAllFilters rows run on the device too (KGPU_OPT_RUN_ALL_FILTERS): the merged code and the map of
    every failing plugin (tests/test_run_all_filters.py holds the cluster-level cases);
  * TestRunScorePlugins: its plugins inject raw and normalized scores the device's plugins cannot
    produce.  Weights, NormalizeScore and the sum run on the device for the real plugins and are
    pinned by TestZeroRequest and every score table; the range check guards plugin bugs the
    device's plugins cannot have.
Those rows are pinned on the oracle's runner (tests/test_oracle_golden.py)."""
import pytest

from conftest import load_golden
from kgpu.compile import Profile
from kgpu.framework import GpuFramework

REAL = {0: ["NodeName", "NodePorts"], 2: ["NodeResourcesFit"], 3: ["NodeUnschedulable"]}
ROWS = [c for c in load_golden("framework") if c["kind"] == "run_filter"
        and all(code in REAL for code in c["profile"]["fake"]["injected_filters"].values())]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ROWS, ids=["%s:%s" % (c["src"].rsplit(":", 1)[1], c["name"]) for c in ROWS])
def test_filter_runner_on_device(case):
    fake = [(p, case["profile"]["fake"]["injected_filters"][p]) for p in case["profile"]["filters"]]
    used = {code: 0 for code in REAL}
    real = []
    for _, code in fake:  # distinct real plugins for repeated outcomes
        real.append(REAL[code][used[code]])
        used[code] += 1
    node = {"metadata": {"name": "node1"}, "spec": {"unschedulable": True},
            "status": {"allocatable": {"cpu": "1", "memory": "1Gi", "pods": "10"}}}
    pod = {"metadata": {"name": "p", "namespace": "default", "uid": "p"},
           "spec": {"containers": [{"name": "c", "resources": {"requests": {"cpu": "2"}}}]}}
    run_all = case["run_all_filters"]
    fw = GpuFramework(Profile(filters=real, scores=[], run_all_filters=run_all), [node], [], pods_hint=[pod])
    res = fw.cycle(pod)
    want = case["expect_merged"]
    if want is None:
        assert res.statuses == {} and res.host == "node1", res.statuses
    else:
        code, plugin, _ = res.statuses["node1"]
        first = next(i for i, (_, c) in enumerate(fake) if c != 0)
        assert (code, plugin) == (want["code"], real[first]), (case["name"], code, plugin)
        if not run_all:
            assert list(case["expect_status_map"]) == [fake[first][0]]
        else:  # the PluginToStatus map: every failing plugin with its own code
            to_fake = dict(zip(real, (f for f, _ in fake)))
            got = {to_fake[pl]: c for pl, (c, _) in res.plugin_statuses["node1"].items()}
            assert got == {f: st["code"] for f, st in case["expect_status_map"].items()}, (case["name"], got)
    fw.engine.close()

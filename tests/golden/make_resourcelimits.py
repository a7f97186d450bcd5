"""Golden vectors transcribed from pkg/scheduler/framework/plugins/noderesources/resource_limits_test.go
(TestResourceLimits).  The "preScore skipped" entry checks a plugin-misuse error path and is not
transcribed."""
from gen_common import case, make_node_cpu_mem, pod

SRC = "pkg/scheduler/framework/plugins/noderesources/resource_limits_test.go"


def limits(cpu, mem):
    return {"name": "c", "resources": {"limits": {"cpu": cpu, "memory": mem}}}


def all_cases():
    m = make_node_cpu_mem
    no_res = pod(containers=[])
    cpu_only = pod(node_name="machine1", containers=[limits("1000m", "0"), limits("2000m", "0")])
    mem_only = pod(node_name="machine2", containers=[limits("0", "2000"), limits("0", "3000")])
    cpu_mem = pod(node_name="machine2", containers=[limits("1000m", "2000"), limits("2000m", "3000")])
    rows = [
        ("pod does not specify its resource limits", 143, no_res,
         [m("machine1", 4000, 10000), m("machine2", 4000, 0), m("machine3", 0, 10000), m("machine4", 0, 0)],
         [0, 0, 0, 0]),
        ("pod only specifies  cpu limits", 149, cpu_only, [m("machine1", 3000, 10000), m("machine2", 2000, 10000)],
         [1, 0]),
        ("pod only specifies  mem limits", 155, mem_only, [m("machine1", 4000, 4000), m("machine2", 5000, 10000)],
         [0, 1]),
        ("pod specifies both cpu and  mem limits", 161, cpu_mem, [m("machine1", 4000, 4000),
                                                                 m("machine2", 5000, 10000)], [1, 1]),
        ("node does not advertise its allocatables", 167, cpu_mem, [m("machine1", 0, 0)], [0]),
    ]
    return [case(name, SRC + ":%d" % line, kind="score", plugin="NodeResourceLimits", args={}, pod=p, pods=[],
                 nodes=nodes, expect_scores={n["metadata"]["name"]: s for n, s in zip(nodes, exp)})
            for name, line, p, nodes, exp in rows]

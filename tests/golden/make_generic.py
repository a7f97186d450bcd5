"""Golden vectors transcribed from pkg/scheduler/core/generic_scheduler_test.go."""
from gen_common import case, container, node, pod

SRC = "pkg/scheduler/core/generic_scheduler_test.go"
DEF_CPU, DEF_MEM = 100, 200 * 1024 * 1024


def make_node(name, milli_cpu, memory):
    """generic_scheduler_test.go:995 makeNode (pods: 100)."""
    return node(name, {"cpu": "%dm" % milli_cpu, "memory": str(memory), "pods": "100"})


def zero_request():
    no_res = dict(containers=[container()])
    small = dict(containers=[container({"cpu": "%dm" % DEF_CPU, "memory": str(DEF_MEM)})])
    large = dict(containers=[container({"cpu": "%dm" % (DEF_CPU * 3), "memory": str(DEF_MEM * 3)})])
    nodes = [make_node("machine1", 1000, DEF_MEM * 10), make_node("machine2", 1000, DEF_MEM * 10)]
    existing = [pod(node_name="machine1", **large), pod(node_name="machine1", **no_res),
                pod(node_name="machine2", **large), pod(node_name="machine2", **small)]
    prof = {"filters": [], "prefilters": [], "prescores": ["DefaultPodTopologySpread"],
            "scores": [["NodeResourcesLeastAllocated", 1], ["NodeResourcesBalancedAllocation", 1],
                       ["DefaultPodTopologySpread", 1]]}
    out = []
    for name, line, spec, want in [
            ("test priority of zero-request pod with machine with zero-request pod", 1074, no_res, 250),
            ("test priority of nonzero-request pod with machine with zero-request pod", 1084, small, 250),
            ("test priority of larger pod with machine with zero-request pod", 1095, large, 230)]:
        out.append(case(name, SRC + ":%d" % line, kind="schedule", profile=prof, nodes=nodes, pods=existing,
                        schedule_pods=[pod(name="p", **spec)],
                        expect_totals=[{"machine1": want, "machine2": want}]))
    return out


def select_host():
    out = []
    for name, line, lst, possible in [
            ("unique properly ordered scores", 314, [["machine1.1", 1], ["machine2.1", 2]], ["machine2.1"]),
            ("equal scores", 322, [["machine1.1", 1], ["machine1.2", 2], ["machine1.3", 2], ["machine2.1", 2]],
             ["machine1.2", "machine1.3", "machine2.1"]),
            ("out of order scores", 333, [["machine1.1", 3], ["machine1.2", 3], ["machine2.1", 2],
                                         ["machine3.1", 1], ["machine1.3", 3]],
             ["machine1.1", "machine1.2", "machine1.3"]),
            ("empty priority list", 345, [], None)]:
        c = case(name, SRC + ":%d" % line, kind="select", list=lst)
        if possible is None:
            c["expect_error"] = "empty priorityList"
        else:
            c["expect_possible"] = possible
        out.append(c)
    return out


def num_feasible():
    out = []
    for name, line, pct, n, want in [
            ("not set percentageOfNodesToScore and nodes number not more than 50", 2477, 0, 10, 10),
            ("set percentageOfNodesToScore and nodes number not more than 50", 2482, 40, 10, 10),
            ("not set percentageOfNodesToScore and nodes number more than 50", 2488, 0, 1000, 420),
            ("set percentageOfNodesToScore and nodes number more than 50", 2493, 40, 1000, 400),
            ("not set percentageOfNodesToScore and nodes number more than 50*125", 2499, 0, 6000, 300),
            ("set percentageOfNodesToScore and nodes number more than 50*125", 2504, 40, 6000, 2400)]:
        out.append(case(name, SRC + ":%d" % line, kind="num_feasible", pct=pct, num_all_nodes=n, expect_num=want))
    return out


def all_cases():
    return zero_request() + select_host() + num_feasible()

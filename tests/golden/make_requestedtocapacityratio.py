"""Golden vectors transcribed from
pkg/scheduler/framework/plugins/noderesources/requested_to_capacity_ratio_test.go
(TestRequestedToCapacityRatio, TestBrokenLinearFunction, TestResourceBinPackingSingleExtended,
TestResourceBinPackingMultipleExtended).  Score only (the plugin has no NormalizeScore)."""
from gen_common import case, container, make_node_cpu_mem, node, pod

SRC = "pkg/scheduler/framework/plugins/noderesources/requested_to_capacity_ratio_test.go"
MIB = 1024 * 1024


def make_pod(node_name, milli_cpu, memory):
    """requested_to_capacity_ratio_test.go:101 makePod: explicit (possibly zero) cpu / memory requests."""
    return pod(node_name=node_name or None, containers=[container({"cpu": "%dm" % milli_cpu, "memory": str(memory)})])


def ext_node(name, milli_cpu, memory, ext):
    """test_util.go:41 makeNodeWithExtendedResource."""
    al = {"cpu": "%dm" % milli_cpu, "memory": str(memory)}
    al.update({k: str(v) for k, v in ext.items()})
    return node(name, al)


def ext_pod(reqs, node_name=None):
    return pod(node_name=node_name, containers=[container({k: str(v) for k, v in reqs.items()})] if reqs else [])


def score_cases():
    out = []

    def sc(name, line, p, nodes, pods, exp, shape, resources):
        out.append(case(name, SRC + ":%d" % line, kind="score", plugin="RequestedToCapacityRatio",
                        args={"shape": shape, "resources": resources}, pod=p, pods=pods, nodes=nodes,
                        expect_scores={n["metadata"]["name"]: s for n, s in zip(nodes, exp)}))

    shape, res = [[0, 10], [100, 0]], [["memory", 1], ["cpu", 1]]
    n44 = [make_node_cpu_mem("node1", 4000, 10000), make_node_cpu_mem("node2", 4000, 10000)]
    n46 = [make_node_cpu_mem("node1", 4000, 10000), make_node_cpu_mem("node2", 6000, 10000)]
    sc("nothing scheduled, nothing requested (default - least requested nodes have priority)", 44,
       make_pod("", 0, 0), n44, [make_pod("node1", 0, 0), make_pod("node2", 0, 0)], [100, 100], shape, res)
    sc("nothing scheduled, resources requested, differently sized machines (default - least requested nodes have "
       "priority)", 51, make_pod("", 3000, 5000), n46, [make_pod("node1", 0, 0), make_pod("node2", 0, 0)], [38, 50],
       shape, res)
    sc("no resources requested, pods scheduled with resources (default - least requested nodes have priority)", 58,
       make_pod("", 0, 0), n46, [make_pod("node1", 3000, 5000), make_pod("node2", 3000, 5000)], [38, 50], shape, res)

    # ---- TestResourceBinPackingSingleExtended (:183): shape (0,0),(100,1), intel.com/foo weight 1
    foo = "intel.com/foo"
    shape1, res1 = [[0, 0], [100, 1]], [[foo, 1]]
    nodes1 = [ext_node("machine1", 4000, 10000 * MIB, {foo: 8}), ext_node("machine2", 4000, 10000 * MIB, {foo: 4})]
    p1, p2 = {foo: 2}, {foo: 4}
    sc("nothing scheduled, nothing requested", 253, ext_pod({}), nodes1, [], [0, 0], shape1, res1)
    sc("resources requested, pods scheduled with less resources", 275, ext_pod(p1), nodes1, [ext_pod({})], [2, 5],
       shape1, res1)
    sc("resources requested, pods scheduled with resources, on node with existing pod running ", 299, ext_pod(p1),
       nodes1, [ext_pod(p1, "machine2")], [2, 10], shape1, res1)
    sc("resources requested, pods scheduled with more resources", 323, ext_pod(p2), nodes1, [ext_pod({})], [5, 10],
       shape1, res1)

    # ---- TestResourceBinPackingMultipleExtended (:352): foo weight 3, bar weight 5
    bar = "intel.com/bar"
    res2 = [[foo, 3], [bar, 5]]
    nodes2 = [ext_node("machine1", 4000, 10000 * MIB, {foo: 8, bar: 4}),
              ext_node("machine2", 4000, 10000 * MIB, {foo: 4, bar: 8})]
    q1, q2 = {foo: 2, bar: 2}, {foo: 4, bar: 2}
    sc("nothing scheduled, nothing requested", 440, ext_pod({}), nodes2, [], [0, 0], shape1, res2)
    sc("resources requested, pods scheduled with less resources", 471, ext_pod(q1), nodes2, [ext_pod({})], [4, 3],
       shape1, res2)
    sc("resources requested, pods scheduled with resources, on node with existing pod running ", 502, ext_pod(q1),
       nodes2, [ext_pod(q1, "machine2")], [4, 7], shape1, res2)
    sc("resources requested, pods scheduled with more resources", 545, ext_pod(q2), nodes2, [ext_pod({})], [5, 5],
       shape1, res2)
    return out


def broken_linear_cases():
    """TestBrokenLinearFunction (:119): the shape function itself (points already on the 0-100 scale)."""
    rows = [([[10, 1], [90, 9]], [(-10, 1), (0, 1), (9, 1), (10, 1), (15, 1), (19, 1), (20, 2), (89, 8), (90, 9),
                                  (99, 9), (100, 9), (110, 9)]),
            ([[0, 2], [40, 10], [100, 0]], [(-10, 2), (0, 2), (20, 6), (30, 8), (40, 10), (70, 5), (100, 0),
                                             (110, 0)]),
            ([[0, 2], [40, 2], [100, 2]], [(-10, 2), (0, 2), (20, 2), (30, 2), (40, 2), (70, 2), (100, 2), (110, 2)])]
    return [case("broken linear %d" % i, SRC + ":119", kind="broken_linear", points=pts,
                 expect_values=[[p, v] for p, v in asserts]) for i, (pts, asserts) in enumerate(rows)]


def all_cases():
    return score_cases() + broken_linear_cases()

"""Golden vectors transcribed from pkg/scheduler/framework/plugins/noderesources/*_test.go."""
from gen_common import case, container, pod, make_node_cpu_mem, resource_pod, node, rl_from_resource

LA = "pkg/scheduler/framework/plugins/noderesources/least_allocated_test.go"
MA = "pkg/scheduler/framework/plugins/noderesources/most_allocated_test.go"
BA = "pkg/scheduler/framework/plugins/noderesources/balanced_allocation_test.go"
FT = "pkg/scheduler/framework/plugins/noderesources/fit_test.go"

L1 = {"foo": "bar", "baz": "blah"}
L2 = {"bar": "foo", "baz": "blah"}


def _cm(cpu, mem):
    return container({"cpu": cpu, "memory": mem})


def spec_pods():
    no_res = dict(containers=[])
    cpu_only = dict(node_name="machine1", containers=[_cm("1000m", "0"), _cm("2000m", "0")])
    cpu_only2 = dict(cpu_only, node_name="machine2")
    cpu_mem = dict(node_name="machine2", containers=[_cm("1000m", "2000"), _cm("2000m", "3000")])
    big = dict(node_name="machine1", containers=[_cm("2000m", "4000"), _cm("3000m", "5000")])
    return no_res, cpu_only, cpu_only2, cpu_mem, big


def _incoming(spec):
    # the incoming pod keeps the spec's NodeName field (the Score call ignores it)
    return pod(**spec)


def scored(plugin, src, name, spec, nodes, expect, pods=(), args=None):
    return case(name, src, kind="score", plugin=plugin, args=args or {}, pod=_incoming(spec),
                pods=list(pods), nodes=nodes, expect_scores=expect)


def least_most_balanced():
    no_res, cpu_only, cpu_only2, cpu_mem, big = spec_pods()
    m = make_node_cpu_mem
    out = []
    dflt = {"resources": [["cpu", 1], ["memory", 1]]}
    sched4 = [pod(labels=L2, **dict(node_name="machine1", containers=[])),
              pod(labels=L1, **dict(node_name="machine1", containers=[])),
              pod(labels=L1, **dict(node_name="machine2", containers=[])),
              pod(labels=L1, **dict(node_name="machine2", containers=[]))]
    sched_res4 = [pod(labels=L2, **cpu_only), pod(labels=L1, **cpu_only), pod(labels=L1, **cpu_only2),
                  pod(labels=L1, **cpu_mem)]
    sched2 = [pod(**cpu_only), pod(**cpu_mem)]
    P = "NodeResourcesLeastAllocated"
    out += [
        scored(P, LA + ":128", "nothing scheduled, nothing requested", no_res,
               [m("machine1", 4000, 10000), m("machine2", 4000, 10000)], {"machine1": 100, "machine2": 100}, args=dflt),
        scored(P, LA + ":142", "nothing scheduled, resources requested, differently sized machines", cpu_mem,
               [m("machine1", 4000, 10000), m("machine2", 6000, 10000)], {"machine1": 37, "machine2": 50}, args=dflt),
        scored(P, LA + ":156", "no resources requested, pods scheduled", no_res,
               [m("machine1", 4000, 10000), m("machine2", 4000, 10000)], {"machine1": 100, "machine2": 100},
               sched4, args=dflt),
        scored(P, LA + ":176", "no resources requested, pods scheduled with resources", no_res,
               [m("machine1", 10000, 20000), m("machine2", 10000, 20000)], {"machine1": 70, "machine2": 57},
               sched_res4, args=dflt),
        scored(P, LA + ":196", "resources requested, pods scheduled with resources", cpu_mem,
               [m("machine1", 10000, 20000), m("machine2", 10000, 20000)], {"machine1": 57, "machine2": 45},
               sched2, args=dflt),
        scored(P, LA + ":214", "resources requested, pods scheduled with resources, differently sized machines",
               cpu_mem, [m("machine1", 10000, 20000), m("machine2", 10000, 50000)],
               {"machine1": 57, "machine2": 60}, sched2, args=dflt),
        scored(P, LA + ":232", "requested resources exceed node capacity", cpu_only,
               [m("machine1", 4000, 10000), m("machine2", 4000, 10000)], {"machine1": 50, "machine2": 25},
               sched2, args=dflt),
        scored(P, LA + ":243", "zero node resources, pods scheduled with resources", no_res,
               [m("machine1", 0, 0), m("machine2", 0, 0)], {"machine1": 0, "machine2": 0}, sched2, args=dflt),
        scored(P, LA + ":260", "different weight on CPU and memory, differently sized machines", cpu_mem,
               [m("machine1", 4000, 10000), m("machine2", 6000, 10000)], {"machine1": 41, "machine2": 50},
               args={"resources": [["memory", 2], ["cpu", 1]]}),
        case("resource with negtive weight", LA + ":269", kind="score", plugin=P,
             args={"resources": [["memory", -1], ["cpu", 1]]}, pod=_incoming(cpu_mem), pods=[],
             nodes=[m("machine", 4000, 10000)],
             expect_error="resource Weight of memory should be a positive value, got -1"),
        case("resource with zero weight", LA + ":277", kind="score", plugin=P,
             args={"resources": [["memory", 1], ["cpu", 0]]}, pod=_incoming(cpu_mem), pods=[],
             nodes=[m("machine", 4000, 10000)],
             expect_error="resource Weight of cpu should be a positive value, got 0"),
        case("resource weight larger than MaxNodeScore", LA + ":285", kind="score", plugin=P,
             args={"resources": [["memory", 120]]}, pod=_incoming(cpu_mem), pods=[],
             nodes=[m("machine", 4000, 10000)],
             expect_error="resource Weight of memory should be less than 100, got 120"),
    ]
    P = "NodeResourcesMostAllocated"
    mdflt = {"resources": [["cpu", 1], ["cpu", 1], ["memory", 1]]}
    out += [
        scored(P, MA + ":128", "nothing scheduled, nothing requested", no_res,
               [m("machine1", 4000, 10000), m("machine2", 4000, 10000)], {"machine1": 0, "machine2": 0}, args=mdflt),
        scored(P, MA + ":142", "nothing scheduled, resources requested, differently sized machines", cpu_mem,
               [m("machine1", 4000, 10000), m("machine2", 6000, 10000)], {"machine1": 62, "machine2": 50},
               args=mdflt),
        scored(P, MA + ":156", "no resources requested, pods scheduled with resources", no_res,
               [m("machine1", 10000, 20000), m("machine2", 10000, 20000)], {"machine1": 30, "machine2": 42},
               sched_res4, args=mdflt),
        scored(P, MA + ":176", "resources requested, pods scheduled with resources", cpu_mem,
               [m("machine1", 10000, 20000), m("machine2", 10000, 20000)], {"machine1": 42, "machine2": 55},
               sched2, args=mdflt),
        scored(P, MA + ":194", "resources requested with more than the node, pods scheduled with resources", big,
               [m("machine1", 4000, 10000), m("machine2", 10000, 8000)], {"machine1": 45, "machine2": 25},
               args=mdflt),
        scored(P, MA + ":208", "nothing scheduled, resources requested with different weight", cpu_mem,
               [m("machine1", 4000, 10000), m("machine2", 6000, 10000)], {"machine1": 58, "machine2": 50},
               args={"resources": [["memory", 2], ["cpu", 1]]}),
        case("resource with negtive weight", MA + ":216", kind="score", plugin=P,
             args={"resources": [["memory", -1], ["cpu", 1]]}, pod=_incoming(cpu_mem), pods=[],
             nodes=[m("machine", 4000, 10000)],
             expect_error="resource Weight of memory should be a positive value, got -1"),
        case("resource with zero weight", MA + ":223", kind="score", plugin=P,
             args={"resources": [["memory", 1], ["cpu", 0]]}, pod=_incoming(cpu_mem), pods=[],
             nodes=[m("machine", 4000, 10000)],
             expect_error="resource Weight of cpu should be a positive value, got 0"),
        case("resource weight larger than MaxNodeScore", MA + ":230", kind="score", plugin=P,
             args={"resources": [["memory", 120]]}, pod=_incoming(cpu_mem), pods=[],
             nodes=[m("machine", 4000, 10000)],
             expect_error="resource Weight of memory should be less than 100, got 120"),
    ]
    P = "NodeResourcesBalancedAllocation"
    out += [
        scored(P, BA + ":231", "nothing scheduled, nothing requested", no_res,
               [m("machine1", 4000, 10000), m("machine2", 4000, 10000)], {"machine1": 100, "machine2": 100}),
        scored(P, BA + ":245", "nothing scheduled, resources requested, differently sized machines", cpu_mem,
               [m("machine1", 4000, 10000), m("machine2", 6000, 10000)], {"machine1": 75, "machine2": 100}),
        scored(P, BA + ":259", "no resources requested, pods scheduled", no_res,
               [m("machine1", 4000, 10000), m("machine2", 4000, 10000)], {"machine1": 100, "machine2": 100}, sched4),
        scored(P, BA + ":279", "no resources requested, pods scheduled with resources", no_res,
               [m("machine1", 10000, 20000), m("machine2", 10000, 20000)], {"machine1": 40, "machine2": 65},
               sched_res4),
        scored(P, BA + ":299", "resources requested, pods scheduled with resources", cpu_mem,
               [m("machine1", 10000, 20000), m("machine2", 10000, 20000)], {"machine1": 65, "machine2": 90}, sched2),
        scored(P, BA + ":317", "resources requested, pods scheduled with resources, differently sized machines",
               cpu_mem, [m("machine1", 10000, 20000), m("machine2", 10000, 50000)],
               {"machine1": 65, "machine2": 60}, sched2),
        scored(P, BA + ":335", "requested resources exceed node capacity", cpu_only,
               [m("machine1", 4000, 10000), m("machine2", 4000, 10000)], {"machine1": 0, "machine2": 0}, sched2),
        scored(P, BA + ":345", "zero node resources, pods scheduled with resources", no_res,
               [m("machine1", 0, 0), m("machine2", 0, 0)], {"machine1": 0, "machine2": 0}, sched2),
        # BA:357 ("Include volume count ...") needs BalanceAttachedNodeVolumes=true: out of scope.
    ]
    return out


EXT_A, EXT_B = "example.com/aaa", "example.com/bbb"
K8S_A, K8S_B = "kubernetes.io/something", "subdomain.kubernetes.io/something"
HUGE_A = "hugepages-2Mi"


def _alloc(milli_cpu, memory, pods, ext_a, storage, huge_a):
    """fit_test.go:54 makeAllocatableResources."""
    return {"cpu": "%dm" % milli_cpu, "memory": str(memory), "pods": str(pods), EXT_A: str(ext_a),
            "ephemeral-storage": str(storage), HUGE_A: str(huge_a)}


def _fit(name, src, in_pod, existing, alloc, code=0, reasons=(), ignored=()):
    e = dict(existing)
    e["spec"] = dict(e["spec"], nodeName="n")
    return case(name, src, kind="filter", plugin="NodeResourcesFit", args={"ignored": list(ignored)},
                pod=in_pod, pods=[e], nodes=[node("n", alloc)],
                expect_filter={"n": {"code": code, "reasons": list(reasons)}})


def R(**kw):
    return kw


def init_pod(p, *usages):
    p["spec"]["initContainers"] = [container(rl_from_resource(**u)) for u in usages]
    return p


def fit():
    A = _alloc(10, 20, 32, 5, 20, 5)
    U = 2  # Unschedulable
    ins = lambda r: "Insufficient " + r  # noqa: E731
    out = [
        _fit("no resources requested always fits", FT + ":102", pod(), resource_pod(R(milli_cpu=10, memory=20)), A),
        _fit("too many resources fails", FT + ":109", resource_pod(R(milli_cpu=1, memory=1)),
             resource_pod(R(milli_cpu=10, memory=20)), A, U, [ins("cpu"), ins("memory")]),
        _fit("too many resources fails due to init container cpu", FT + ":116",
             init_pod(resource_pod(R(milli_cpu=1, memory=1)), R(milli_cpu=3, memory=1)),
             resource_pod(R(milli_cpu=8, memory=19)), A, U, [ins("cpu")]),
        _fit("too many resources fails due to highest init container cpu", FT + ":123",
             init_pod(resource_pod(R(milli_cpu=1, memory=1)), R(milli_cpu=3, memory=1), R(milli_cpu=2, memory=1)),
             resource_pod(R(milli_cpu=8, memory=19)), A, U, [ins("cpu")]),
        _fit("too many resources fails due to init container memory", FT + ":130",
             init_pod(resource_pod(R(milli_cpu=1, memory=1)), R(milli_cpu=1, memory=3)),
             resource_pod(R(milli_cpu=9, memory=19)), A, U, [ins("memory")]),
        _fit("too many resources fails due to highest init container memory", FT + ":137",
             init_pod(resource_pod(R(milli_cpu=1, memory=1)), R(milli_cpu=1, memory=3), R(milli_cpu=1, memory=2)),
             resource_pod(R(milli_cpu=9, memory=19)), A, U, [ins("memory")]),
        _fit("init container fits because it's the max, not sum", FT + ":144",
             init_pod(resource_pod(R(milli_cpu=1, memory=1)), R(milli_cpu=1, memory=1)),
             resource_pod(R(milli_cpu=9, memory=19)), A),
        _fit("multiple init containers fit because it's the max, not sum", FT + ":150",
             init_pod(resource_pod(R(milli_cpu=1, memory=1)), R(milli_cpu=1, memory=1), R(milli_cpu=1, memory=1)),
             resource_pod(R(milli_cpu=9, memory=19)), A),
        _fit("both resources fit", FT + ":156", resource_pod(R(milli_cpu=1, memory=1)),
             resource_pod(R(milli_cpu=5, memory=5)), A),
        _fit("one resource memory fits", FT + ":162", resource_pod(R(milli_cpu=2, memory=1)),
             resource_pod(R(milli_cpu=9, memory=5)), A, U, [ins("cpu")]),
        _fit("one resource cpu fits", FT + ":169", resource_pod(R(milli_cpu=1, memory=2)),
             resource_pod(R(milli_cpu=5, memory=19)), A, U, [ins("memory")]),
        _fit("equal edge case", FT + ":176", resource_pod(R(milli_cpu=5, memory=1)),
             resource_pod(R(milli_cpu=5, memory=19)), A),
        _fit("equal edge case for init container", FT + ":182",
             init_pod(resource_pod(R(milli_cpu=4, memory=1)), R(milli_cpu=5, memory=1)),
             resource_pod(R(milli_cpu=5, memory=19)), A),
        _fit("extended resource fits", FT + ":188", resource_pod(R(scalars={EXT_A: 1})), resource_pod(R()), A),
        _fit("extended resource fits for init container", FT + ":193",
             init_pod(resource_pod(R()), R(scalars={EXT_A: 1})), resource_pod(R()), A),
        _fit("extended resource capacity enforced", FT + ":198",
             resource_pod(R(milli_cpu=1, memory=1, scalars={EXT_A: 10})),
             resource_pod(R(scalars={EXT_A: 0})), A, U, [ins(EXT_A)]),
        _fit("extended resource capacity enforced for init container", FT + ":206",
             init_pod(resource_pod(R()), R(milli_cpu=1, memory=1, scalars={EXT_A: 10})),
             resource_pod(R(scalars={EXT_A: 0})), A, U, [ins(EXT_A)]),
        _fit("extended resource allocatable enforced", FT + ":214",
             resource_pod(R(milli_cpu=1, memory=1, scalars={EXT_A: 1})),
             resource_pod(R(scalars={EXT_A: 5})), A, U, [ins(EXT_A)]),
        _fit("extended resource allocatable enforced for init container", FT + ":222",
             init_pod(resource_pod(R()), R(milli_cpu=1, memory=1, scalars={EXT_A: 1})),
             resource_pod(R(scalars={EXT_A: 5})), A, U, [ins(EXT_A)]),
        _fit("extended resource allocatable enforced for multiple containers", FT + ":230",
             resource_pod(R(milli_cpu=1, memory=1, scalars={EXT_A: 3}), R(milli_cpu=1, memory=1, scalars={EXT_A: 3})),
             resource_pod(R(scalars={EXT_A: 2})), A, U, [ins(EXT_A)]),
        _fit("extended resource allocatable admits multiple init containers", FT + ":239",
             init_pod(resource_pod(R()), R(milli_cpu=1, memory=1, scalars={EXT_A: 3}),
                      R(milli_cpu=1, memory=1, scalars={EXT_A: 3})),
             resource_pod(R(scalars={EXT_A: 2})), A),
        _fit("extended resource allocatable enforced for multiple init containers", FT + ":248",
             init_pod(resource_pod(R()), R(milli_cpu=1, memory=1, scalars={EXT_A: 6}),
                      R(milli_cpu=1, memory=1, scalars={EXT_A: 3})),
             resource_pod(R(scalars={EXT_A: 2})), A, U, [ins(EXT_A)]),
        _fit("extended resource allocatable enforced for unknown resource", FT + ":258",
             resource_pod(R(milli_cpu=1, memory=1, scalars={EXT_B: 1})), resource_pod(R()), A, U, [ins(EXT_B)]),
        _fit("extended resource allocatable enforced for unknown resource for init container", FT + ":266",
             init_pod(resource_pod(R()), R(milli_cpu=1, memory=1, scalars={EXT_B: 1})), resource_pod(R()), A, U,
             [ins(EXT_B)]),
        _fit("kubernetes.io resource capacity enforced", FT + ":274",
             resource_pod(R(milli_cpu=1, memory=1, scalars={K8S_A: 10})), resource_pod(R()), A, U, [ins(K8S_A)]),
        _fit("kubernetes.io resource capacity enforced for init container", FT + ":282",
             init_pod(resource_pod(R()), R(milli_cpu=1, memory=1, scalars={K8S_B: 10})), resource_pod(R()), A, U,
             [ins(K8S_B)]),
        _fit("hugepages resource capacity enforced", FT + ":290",
             resource_pod(R(milli_cpu=1, memory=1, scalars={HUGE_A: 10})), resource_pod(R(scalars={HUGE_A: 0})),
             A, U, [ins(HUGE_A)]),
        _fit("hugepages resource capacity enforced for init container", FT + ":298",
             init_pod(resource_pod(R()), R(milli_cpu=1, memory=1, scalars={HUGE_A: 10})),
             resource_pod(R(scalars={HUGE_A: 0})), A, U, [ins(HUGE_A)]),
        _fit("hugepages resource allocatable enforced for multiple containers", FT + ":306",
             resource_pod(R(milli_cpu=1, memory=1, scalars={HUGE_A: 3}), R(milli_cpu=1, memory=1, scalars={HUGE_A: 3})),
             resource_pod(R(scalars={HUGE_A: 2})), A, U, [ins(HUGE_A)]),
        _fit("skip checking ignored extended resource", FT + ":315",
             resource_pod(R(milli_cpu=1, memory=1, scalars={EXT_B: 1})), resource_pod(R()), A, ignored=[EXT_B]),
        _fit("resources + pod overhead fits", FT + ":324",
             dict(resource_pod(R(milli_cpu=1, memory=1)), ),
             resource_pod(R(milli_cpu=5, memory=5)), A),
        _fit("requests + overhead does not fit for memory", FT + ":332",
             resource_pod(R(milli_cpu=1, memory=1)),
             resource_pod(R(milli_cpu=5, memory=5)), A, U, [ins("memory")]),
    ]
    out[-2]["pod"]["spec"]["overhead"] = {"cpu": "3m", "memory": "13"}
    out[-1]["pod"]["spec"]["overhead"] = {"cpu": "1m", "memory": "15"}
    A1 = _alloc(10, 20, 1, 0, 0, 0)
    tm = ["Too many pods"]
    out += [
        _fit("even without specified resources predicate fails when there's no space for additional pod",
             FT + ":425", pod(), resource_pod(R(milli_cpu=10, memory=20)), A1, U, tm),
        _fit("even if both resources fit predicate fails when there's no space for additional pod", FT + ":431",
             resource_pod(R(milli_cpu=1, memory=1)), resource_pod(R(milli_cpu=5, memory=5)), A1, U, tm),
        _fit("even for equal edge case predicate fails when there's no space for additional pod", FT + ":437",
             resource_pod(R(milli_cpu=5, memory=1)), resource_pod(R(milli_cpu=5, memory=19)), A1, U, tm),
        _fit("even for equal edge case ... due to init container", FT + ":443",
             init_pod(resource_pod(R(milli_cpu=5, memory=1)), R(milli_cpu=5, memory=1)),
             resource_pod(R(milli_cpu=5, memory=19)), A1, U, tm),
        _fit("due to container scratch disk", FT + ":483", resource_pod(R(milli_cpu=1, memory=1)),
             resource_pod(R(milli_cpu=10, memory=10)), A, U, [ins("cpu")]),
        _fit("pod fit", FT + ":490", resource_pod(R(milli_cpu=1, memory=1)),
             resource_pod(R(milli_cpu=2, memory=10)), A),
        _fit("storage ephemeral local storage request exceeds allocatable", FT + ":496",
             resource_pod(R(eph=25)), resource_pod(R(milli_cpu=2, memory=2)), A, U, [ins("ephemeral-storage")]),
        _fit("pod fits (ephemeral)", FT + ":503", resource_pod(R(eph=10)),
             resource_pod(R(milli_cpu=2, memory=2)), A),
    ]
    return out


def all_cases():
    return least_most_balanced() + fit()

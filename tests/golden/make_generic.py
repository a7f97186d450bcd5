"""Golden vectors transcribed from pkg/scheduler/core/generic_scheduler_test.go (TestGenericScheduler,
TestFindFitAllError, TestFindFitSomeError, TestSelectHost, TestZeroRequest, TestNumFeasibleNodesToFind).

TestGenericScheduler and TestFindFit* drive the fake plugins of that file (tests/fake_plugins.py); they
pin the oracle's orchestration (filter early exit, FitError statuses, normalize, weights, score
errors, PVC basic checks) and run on the oracle only."""
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


U, UR = 2, 3
FAKE = "Nodes failed the fake predicate"


def generic_scheduler():
    out = []

    def gs(name, line, nodes, p, hosts=None, filters=(), scores=(), existing=(), pvcs=(), fake=None,
           message=None, fit=None, prefilters=()):
        prof = {"filters": list(filters), "prefilters": list(prefilters), "prescores": [],
                "scores": [list(x) for x in scores], "fake": fake or {}}
        kw = {}
        if hosts is not None:
            kw["expect_hosts"] = [sorted(hosts)]
            kw["expect_evaluated"] = [len(nodes)]
        else:
            kw["expect_hosts"] = [None]
        if message is not None:
            kw["expect_messages"] = [message]
        if fit is not None:
            kw["expect_fit"] = [fit]
        # generic_scheduler_test.go:816-821: every node carries the label hostname=<name>; NewSnapshot
        # lists a map, so the cases hold for any node order (kept as given here)
        ns = [node(n, {}, labels={"hostname": n}) for n in nodes]
        out.append(case(name, SRC + ":%d" % line, kind="schedule", profile=prof, nodes=ns, pods=list(existing),
                        schedule_pods=[p], pvcs=list(pvcs), order="given", **kw))

    def named(n):
        return pod(name=n, uid=n)

    m12 = ["machine1", "machine2"]
    gs("test 1", 398, m12, named("2"), filters=["FalseFilter"], message="0/2 nodes are available",
       fit={"machine1": [U, [FAKE]], "machine2": [U, [FAKE]]})
    gs("test 2", 415, m12, named("ignore"), hosts=m12, filters=["TrueFilter"])
    gs("test 3", 427, m12, named("machine2"), hosts=["machine2"], filters=["MatchFilter"])
    gs("test 4", 438, ["3", "2", "1"], named("ignore"), hosts=["3"], filters=["TrueFilter"],
       scores=[("NumericMap", 1)])
    gs("test 5", 449, ["3", "2", "1"], named("2"), hosts=["2"], filters=["MatchFilter"], scores=[("NumericMap", 1)])
    gs("test 6", 461, ["3", "2", "1"], named("2"), hosts=["1"], filters=["TrueFilter"],
       scores=[("NumericMap", 1), ("ReverseNumericMap", 2)])
    gs("test 7", 473, ["3", "2", "1"], named("2"), filters=["TrueFilter", "FalseFilter"], scores=[("NumericMap", 1)],
       message="0/3 nodes are available", fit={"3": [U, [FAKE]], "2": [U, [FAKE]], "1": [U, [FAKE]]})
    running2 = pod(name="2", uid="2", node_name="2")
    running2["status"] = {"phase": "Running"}
    gs("test 8", 502, ["1", "2"], named("2"), filters=["NoPodsFilter", "MatchFilter"], scores=[("NumericMap", 1)],
       existing=[running2], message="0/2 nodes are available", fit={"1": [U, [FAKE]], "2": [U, [FAKE]]})

    def with_pvc(claim):
        p = named("ignore")
        p["spec"]["volumes"] = [{"persistentVolumeClaim": {"claimName": claim}}]
        return p

    pvc = {"metadata": {"name": "existingPVC", "namespace": ""}}
    gs("existing PVC", 525, m12, with_pvc("existingPVC"), hosts=m12, filters=["TrueFilter"], pvcs=[pvc])
    gs("unknown PVC", 547, m12, with_pvc("unknownPVC"), filters=["TrueFilter"],
       message='persistentvolumeclaim "unknownPVC" not found')
    deleting = {"metadata": {"name": "existingPVC", "namespace": "", "deletionTimestamp": "0001-01-01T00:00:00Z"}}
    gs("deleted PVC", 569, m12, with_pvc("existingPVC"), filters=["TrueFilter"], pvcs=[deleting],
       message='persistentvolumeclaim "existingPVC" is being deleted')
    gs("test error with priority map", 580, ["2", "1"], pod(name="2"), filters=["TrueFilter"],
       scores=[("FalseMap", 1), ("TrueMap", 2)],
       message='error while running score plugin for pod "2": priority map encounters an error')

    def spread_pod(skew):
        p = pod(name="p", uid="p", labels={"foo": ""})
        p["spec"]["topologySpreadConstraints"] = [{
            "maxSkew": skew, "topologyKey": "hostname", "whenUnsatisfiable": "DoNotSchedule",
            "labelSelector": {"matchExpressions": [{"key": "foo", "operator": "Exists"}]}}]
        return p

    def running(name, nn):
        p = pod(name=name, uid=name, labels={"foo": ""}, node_name=nn)
        p["status"] = {"phase": "Running"}
        return p

    gs("test podtopologyspread plugin - 2 nodes with maxskew=1", 591, m12, spread_pod(1), hosts=["machine2"],
       filters=["PodTopologySpread"], prefilters=["PodTopologySpread"], existing=[running("pod1", "machine1")])
    gs("test podtopologyspread plugin - 3 nodes with maxskew=2", 637, ["machine1", "machine2", "machine3"],
       spread_pod(2), hosts=["machine2", "machine3"], filters=["PodTopologySpread"],
       prefilters=["PodTopologySpread"],
       existing=[running("pod1a", "machine1"), running("pod1b", "machine1"), running("pod2", "machine2")])
    tf = pod(name="test-filter", uid="test-filter")
    gs("test with filter plugin returning Unschedulable status", 699, ["3"], tf, filters=["FakeFilter"],
       scores=[("NumericMap", 1)], fake={"FakeFilter": {"3": U}}, message="0/1 nodes are available",
       fit={"3": [U, ["injecting failure for pod test-filter"]]})
    gs("test with filter plugin returning UnschedulableAndUnresolvable status", 721, ["3"], tf,
       filters=["FakeFilter"], scores=[("NumericMap", 1)], fake={"FakeFilter": {"3": UR}},
       message="0/1 nodes are available", fit={"3": [UR, ["injecting failure for pod test-filter"]]})
    gs("test with partial failed filter plugin", 743, ["1", "2"], tf, hosts=["2"], filters=["FakeFilter"],
       scores=[("NumericMap", 1)], fake={"FakeFilter": {"1": U}})
    return out


def find_fit():
    """TestFindFitAllError (:862) / TestFindFitSomeError (:899): nodes 3, 2, 1; TrueFilter then
    MatchFilter; every node fails with the fake reason except, in the second, the node named like the
    pod ("1")."""
    out = []
    prof = {"filters": ["TrueFilter", "MatchFilter"], "prefilters": [], "prescores": [],
            "scores": [["NumericMap", 1]], "fake": {}}
    ns = [node(n, {}) for n in ["3", "2", "1"]]
    out.append(case("find fit all error", SRC + ":862", kind="schedule", profile=prof, nodes=ns, pods=[],
                    schedule_pods=[pod(name="")], order="given", expect_hosts=[None],
                    expect_fit=[{"3": [U, [FAKE]], "2": [U, [FAKE]], "1": [U, [FAKE]]}]))
    out.append(case("find fit some error", SRC + ":899", kind="schedule", profile=prof, nodes=ns, pods=[],
                    schedule_pods=[pod(name="1", uid="1")], order="given", expect_hosts=[["1"]],
                    expect_evaluated=[3]))
    return out


def all_cases():
    return zero_request() + select_host() + num_feasible() + generic_scheduler() + find_fit()

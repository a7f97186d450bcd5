"""Golden vectors transcribed from pkg/scheduler/core/generic_scheduler_test.go: TestSelectNodesForPreemption
(:1273), TestPickOneNodeForPreemption (:1652), TestNodesWherePreemptionMightHelp (:1931) and TestPreempt
(:2047).

The preemption tables prepend a FakeFilter whose return code is the case's filterReturnCode (Success
unless stated); with Success it is a no-op, so those cases also run through the HIP path
("gpu": true).  Pods without a status.startTime get the test's assignDefaultStartTime value, one
`now` later than every fixed start time (:2523-2531)."""
from gen_common import case, container, node, pod

SRC = "pkg/scheduler/core/generic_scheduler_test.go"
DEF_CPU, DEF_MEM = 100, 200 * 1024 * 1024
NEG, LOW, MID, HIGH, VHIGH = -100, 0, 100, 1000, 10000
NOW = "2030-01-01T00:00:00Z"   # assignDefaultStartTime's metav1.Now(), later than every fixed time
ST = {"": "2019-01-01T01:01:01Z", "0102": "2019-01-02T01:01:01Z", "0103": "2019-01-03T01:01:01Z",
      "0104": "2019-01-04T01:01:01Z", "0105": "2019-01-05T01:01:01Z", "0106": "2019-01-06T01:01:01Z",
      "0107": "2019-01-07T01:01:01Z"}
U, UR = 2, 3


def ctr(mult):
    return [container({"cpu": "%dm" % (DEF_CPU * mult), "memory": str(DEF_MEM * mult)})]


SMALL, MEDIUM, LARGE, VLARGE = ctr(1), ctr(2), ctr(3), ctr(5)


def p(name, prio, node_name=None, containers=None, start=None, uid=True, labels=None, **spec):
    o = pod(name=name, uid=name if uid else None, node_name=node_name, containers=containers, labels=labels,
            priority=prio, **spec)
    o["status"] = {"startTime": ST[start] if start is not None else NOW}
    return o


def make_node(name, milli_cpu, memory, labels=None):
    """generic_scheduler_test.go:995 makeNode (pods: 100)."""
    return node(name, {"cpu": "%dm" % milli_cpu, "memory": str(memory), "pods": "100"}, labels=labels)


def select_nodes():
    out = []
    label_keys = ["hostname", "zone", "region"]

    def sel(name, line, nodes, preemptor, pods, plugins, expected, code=0, pdbs=()):
        ns = []
        for n in nodes:
            lab = {label_keys[i]: part for i, part in enumerate(n.split("/"))}
            ns.append(make_node(lab["hostname"], 1000 * 5, DEF_MEM * 5, labels=lab))
        filters = ["FakeFilter"] + [x for x in plugins if x != "prefilter-only"]
        prefilters = [x for x in plugins if x in ("NodeResourcesFit", "InterPodAffinity", "PodTopologySpread")]
        prof = {"filters": filters, "prefilters": prefilters, "prescores": [], "scores": [],
                "fake": {"FakeFilter": {n["metadata"]["name"]: code for n in ns}}}
        gpu = code == 0 and all(x in ("NodeResourcesFit", "InterPodAffinity", "PodTopologySpread") for x in plugins)
        exp = {k: {"pods": sorted(v[0]), "pdb": v[1]} for k, v in expected.items()}
        out.append(case(name, SRC + ":%d" % line, kind="preempt_select", profile=prof, nodes=ns, pods=pods,
                        pod=preemptor, pdbs=list(pdbs), now=NOW, order="given", gpu=gpu, expect_victims=exp))

    m12 = ["machine1", "machine2"]
    two_mid = [p("a", MID, "machine1"), p("b", MID, "machine2")]
    sel("a pod that does not fit on any machine", 1286, m12, p("new", HIGH), two_mid, ["FalseFilter"], {})
    sel("a pod that fits with no preemption", 1301, m12, p("new", HIGH), two_mid, ["TrueFilter"],
        {"machine1": ([], 0), "machine2": ([], 0)})
    sel("a pod that fits on one machine with no preemption", 1316, m12, p("machine1", HIGH), two_mid,
        ["MatchFilter"], {"machine1": ([], 0)})
    fit = ["NodeResourcesFit"]
    sel("a pod that fits on both machines when lower priority pods are preempted", 1331, m12,
        p("machine1", HIGH, containers=LARGE),
        [p("a", MID, "machine1", LARGE), p("b", MID, "machine2", LARGE)], fit,
        {"machine1": (["a"], 0), "machine2": (["b"], 0)})
    sel("a pod that would fit on the machines, but other pods running are higher priority", 1346, m12,
        p("machine1", LOW, containers=LARGE),
        [p("a", MID, "machine1", LARGE), p("b", MID, "machine2", LARGE)], fit, {})
    sel("medium priority pod is preempted, but lower priority one stays as it is small", 1361, m12,
        p("machine1", HIGH, containers=LARGE),
        [p("a", LOW, "machine1", SMALL), p("b", MID, "machine1", LARGE), p("c", MID, "machine2", LARGE)], fit,
        {"machine1": (["b"], 0), "machine2": (["c"], 0)})
    sel("mixed priority pods are preempted", 1377, m12, p("machine1", HIGH, containers=LARGE),
        [p("a", MID, "machine1", SMALL), p("b", LOW, "machine1", SMALL), p("c", MID, "machine1", MEDIUM),
         p("d", HIGH, "machine1", SMALL), p("e", HIGH, "machine2", LARGE)], fit,
        {"machine1": (["b", "c"], 0)})
    sel("mixed priority pods are preempted, pick later StartTime one when priorities are equal", 1395, m12,
        p("machine1", HIGH, containers=LARGE),
        [p("a", LOW, "machine1", SMALL, "0107"), p("b", LOW, "machine1", SMALL, "0106"),
         p("c", MID, "machine1", MEDIUM, "0105"), p("d", HIGH, "machine1", SMALL, "0104"),
         p("e", HIGH, "machine2", LARGE, "0103")], fit,
        {"machine1": (["a", "c"], 0)})
    anti = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [{
        "labelSelector": {"matchExpressions": [{"key": "pod", "operator": "In", "values": ["preemptor", "value2"]}]},
        "topologyKey": "hostname"}]}}
    sel("pod with anti-affinity is preempted", 1413, m12,
        p("machine1", HIGH, containers=SMALL, uid=False, labels={"pod": "preemptor"}),
        [p("a", LOW, "machine1", SMALL, labels={"service": "securityscan"}, affinity=anti),
         p("b", MID, "machine1", SMALL), p("d", HIGH, "machine1", SMALL), p("e", HIGH, "machine2", LARGE)],
        ["NodeResourcesFit", "InterPodAffinity"], {"machine1": (["a"], 0), "machine2": ([], 0)})
    foo = {"matchExpressions": [{"key": "foo", "operator": "Exists"}]}
    tsc = [{"maxSkew": 1, "topologyKey": "zone", "whenUnsatisfiable": "DoNotSchedule", "labelSelector": foo},
           {"maxSkew": 1, "topologyKey": "hostname", "whenUnsatisfiable": "DoNotSchedule", "labelSelector": foo}]

    def running(name, prio, nn):
        o = p(name, prio, nn, labels={"foo": ""})
        o["status"]["phase"] = "Running"
        return o

    sel("preemption to resolve even pods spread FitError", 1449, ["node-a/zone1", "node-b/zone1", "node-x/zone2"],
        p("p", HIGH, uid=False, labels={"foo": ""}, topologySpreadConstraints=tsc),
        [running("pod-a1", MID, "node-a"), running("pod-a2", LOW, "node-a"), running("pod-b1", LOW, "node-b"),
         running("pod-x1", HIGH, "node-x"), running("pod-x2", HIGH, "node-x")],
        ["PodTopologySpread"], {"node-a": (["pod-a2"], 0), "node-b": (["pod-b1"], 0)})
    sel("get Unschedulable in the preemption phase when the filter plugins filtering the nodes", 1532, m12,
        p("machine1", HIGH, containers=LARGE),
        [p("a", MID, "machine1", LARGE), p("b", MID, "machine2", LARGE)], fit, {}, code=U)
    pdb = {"namespace": "", "selector": {"matchLabels": {"app": "foo"}}, "disruptionsAllowed": 1}
    sel("preemption with violation of same pdb", 1548, ["machine1"], p("pod1", HIGH, containers=VLARGE),
        [p("a", MID, "machine1", MEDIUM, labels={"app": "foo"}), p("b", MID, "machine1", MEDIUM, labels={"app": "foo"})],
        fit, {"machine1": (["a", "b"], 1)}, pdbs=[pdb])
    return out


def pick_one():
    out = []

    def pick(name, line, nodes, preemptor, pods, expected):
        ns = [make_node(n, DEF_CPU * 5, DEF_MEM * 5) for n in nodes]
        prof = {"filters": ["NodeResourcesFit"], "prefilters": ["NodeResourcesFit"], "prescores": [], "scores": []}
        out.append(case(name, SRC + ":%d" % line, kind="preempt_pick", profile=prof, nodes=ns, pods=pods,
                        pod=preemptor, pdbs=[], now=NOW, order="given", gpu=True, expect_possible=expected))

    pick("No node needs preemption", 1662, ["machine1"], p("machine1", HIGH, containers=LARGE),
         [p("m1.1", MID, "machine1", SMALL, "")], ["machine1"])
    m12, m123 = ["machine1", "machine2"], ["machine1", "machine2", "machine3"]
    pick("a pod that fits on both machines when lower priority pods are preempted", 1675, m12,
         p("machine1", HIGH, containers=LARGE),
         [p("m1.1", MID, "machine1", LARGE, ""), p("m2.1", MID, "machine2", LARGE, "")], m12)
    pick("a pod that fits on a machine with no preemption", 1690, m123, p("machine1", HIGH, containers=LARGE),
         [p("m1.1", MID, "machine1", LARGE, ""), p("m2.1", MID, "machine2", LARGE, "")], ["machine3"])
    pick("machine with min highest priority pod is picked", 1705, m123, p("machine1", HIGH, containers=VLARGE),
         [p("m1.1", MID, "machine1", MEDIUM, ""), p("m1.2", MID, "machine1", LARGE, ""),
          p("m2.1", MID, "machine2", MEDIUM, ""), p("m2.2", LOW, "machine2", MEDIUM, ""),
          p("m3.1", LOW, "machine3", MEDIUM, ""), p("m3.2", LOW, "machine3", MEDIUM, "")], ["machine3"])
    pick("when highest priorities are the same, minimum sum of priorities is picked", 1726, m123,
         p("machine1", HIGH, containers=VLARGE),
         [p("m1.1", MID, "machine1", MEDIUM, ""), p("m1.2", MID, "machine1", LARGE, ""),
          p("m2.1", MID, "machine2", LARGE, ""), p("m2.2", LOW, "machine2", MEDIUM, ""),
          p("m3.1", MID, "machine3", MEDIUM, ""), p("m3.2", MID, "machine3", MEDIUM, "")], ["machine2"])
    pick("when highest priority and sum are the same, minimum number of pods is picked", 1747, m123,
         p("machine1", HIGH, containers=VLARGE),
         [p("m1.1", MID, "machine1", SMALL, ""), p("m1.2", NEG, "machine1", SMALL, ""),
          p("m1.3", MID, "machine1", SMALL, ""), p("m1.4", NEG, "machine1", SMALL, ""),
          p("m2.1", MID, "machine2", LARGE, ""), p("m2.2", NEG, "machine2", MEDIUM, ""),
          p("m3.1", MID, "machine3", MEDIUM, ""), p("m3.2", NEG, "machine3", SMALL, ""),
          p("m3.3", LOW, "machine3", SMALL, "")], ["machine2"])
    pick("sum of adjusted priorities is considered", 1773, m123, p("machine1", HIGH, containers=VLARGE),
         [p("m1.1", MID, "machine1", SMALL, ""), p("m1.2", NEG, "machine1", SMALL, ""),
          p("m1.3", NEG, "machine1", SMALL, ""),
          p("m2.1", MID, "machine2", LARGE, ""), p("m2.2", NEG, "machine2", MEDIUM, ""),
          p("m3.1", MID, "machine3", MEDIUM, ""), p("m3.2", NEG, "machine3", SMALL, ""),
          p("m3.3", LOW, "machine3", SMALL, "")], ["machine2"])
    pick("non-overlapping lowest high priority, sum priorities, and number of pods", 1796,
         ["machine1", "machine2", "machine3", "machine4"], p("pod1", VHIGH, containers=VLARGE),
         [p("m1.1", MID, "machine1", SMALL, ""), p("m1.2", LOW, "machine1", SMALL, ""),
          p("m1.3", LOW, "machine1", SMALL, ""),
          p("m2.1", HIGH, "machine2", LARGE, ""),
          p("m3.1", MID, "machine3", MEDIUM, ""), p("m3.2", LOW, "machine3", SMALL, ""),
          p("m3.3", LOW, "machine3", SMALL, ""), p("m3.4", LOW, "machine3", MEDIUM, ""),
          p("m4.1", MID, "machine4", MEDIUM, ""), p("m4.2", MID, "machine4", SMALL, ""),
          p("m4.3", MID, "machine4", SMALL, ""), p("m4.4", NEG, "machine4", SMALL, "")], ["machine1"])
    pick("same priority, same number of victims, different start time for each machine's pod", 1824, m123,
         p("machine1", HIGH, containers=VLARGE),
         [p("m1.1", MID, "machine1", MEDIUM, "0103"), p("m1.2", MID, "machine1", MEDIUM, "0103"),
          p("m2.1", MID, "machine2", MEDIUM, "0104"), p("m2.2", MID, "machine2", MEDIUM, "0104"),
          p("m3.1", MID, "machine3", MEDIUM, "0102"), p("m3.2", MID, "machine3", MEDIUM, "0102")], ["machine2"])
    pick("same priority, same number of victims, different start time for all pods", 1845, m123,
         p("machine1", HIGH, containers=VLARGE),
         [p("m1.1", MID, "machine1", MEDIUM, "0105"), p("m1.2", MID, "machine1", MEDIUM, "0103"),
          p("m2.1", MID, "machine2", MEDIUM, "0106"), p("m2.2", MID, "machine2", MEDIUM, "0102"),
          p("m3.1", MID, "machine3", MEDIUM, "0104"), p("m3.2", MID, "machine3", MEDIUM, "0107")], ["machine3"])
    pick("different priority, same number of victims, different start time for all pods", 1866, m123,
         p("machine1", HIGH, containers=VLARGE),
         [p("m1.1", LOW, "machine1", MEDIUM, "0105"), p("m1.2", MID, "machine1", MEDIUM, "0103"),
          p("m2.1", MID, "machine2", MEDIUM, "0107"), p("m2.2", LOW, "machine2", MEDIUM, "0102"),
          p("m3.1", LOW, "machine3", MEDIUM, "0104"), p("m3.2", MID, "machine3", MEDIUM, "0106")], ["machine2"])
    return out


def might_help():
    out = []
    names = ["machine%d" % i for i in range(1, 5)]

    def mh(name, line, statuses, expected):
        out.append(case(name, SRC + ":%d" % line, kind="preempt_might_help", node_names=names,
                        statuses=statuses, expect_set=sorted(expected)))

    mh("No node should be attempted", 1944, {"machine1": UR, "machine2": UR, "machine3": UR, "machine4": UR}, [])
    mh("ErrReasonAffinityNotMatch should be tried as it indicates that the pod is unschedulable due to inter-pod "
       "affinity or anti-affinity", 1954, {"machine1": U, "machine2": UR, "machine3": UR}, ["machine1", "machine4"])
    mh("pod with both pod affinity and anti-affinity should be tried", 1963, {"machine1": U, "machine2": UR},
       ["machine1", "machine3", "machine4"])
    mh("ErrReasonAffinityRulesNotMatch should not be tried as it indicates that the pod is unschedulable due to "
       "inter-pod affinity, but ErrReasonAffinityNotMatch should be tried as it indicates that the pod is "
       "unschedulable due to inter-pod affinity or anti-affinity", 1971, {"machine1": UR, "machine2": U},
       ["machine2", "machine3", "machine4"])
    mh("Mix of failed predicates works fine", 1979, {"machine1": UR, "machine2": U},
       ["machine2", "machine3", "machine4"])
    mh("Node condition errors should be considered unresolvable", 1987, {"machine1": UR},
       ["machine2", "machine3", "machine4"])
    mh("ErrVolume... errors should not be tried as it indicates that the pod is unschedulable due to no matching "
       "volumes for pod on node", 1994, {"machine1": UR, "machine2": UR, "machine3": UR}, ["machine4"])
    mh("ErrTopologySpreadConstraintsNotMatch should be tried as it indicates that the pod is unschedulable due to "
       "topology spread constraints", 2003, {"machine1": U, "machine2": UR, "machine3": U},
       ["machine1", "machine3", "machine4"])
    mh("UnschedulableAndUnresolvable status should be skipped but Unschedulable should be tried", 2012,
       {"machine2": UR, "machine3": U, "machine4": UR}, ["machine1", "machine3"])
    return out


def preempt_cases():
    """TestPreempt (:2047): genericScheduler.Preempt after a FitError whose statuses are the table's
    failedNodeToStatusMap (default: machine1..3 Unschedulable), with the table's extenders
    (FakeExtender predicates, tests/fake_plugins.py).  Then the reference marks the victims deleted,
    nominates the preemptor to the node and calls Preempt again: no more pods may be preempted."""
    out = []
    label_keys = ["hostname", "zone", "region"]
    lower, never = "PreemptLowerPriority", "Never"

    def pre(name, line, preemptor, pods, expected_node, expected, plugins=("NodeResourcesFit",), node_names=None,
            statuses=None, extenders=()):
        ns = []
        for n in node_names or ["machine1", "machine2", "machine3"]:
            lab = {label_keys[i]: part for i, part in enumerate(n.split("/"))}
            ns.append(make_node(lab["hostname"], 1000 * 5, DEF_MEM * 5, labels=lab))
        names = [n["metadata"]["name"] for n in ns]
        st = statuses or {nm: U for nm in names[:3]}
        prof = {"filters": list(plugins), "prefilters": list(plugins), "prescores": [], "scores": []}
        out.append(case(name, SRC + ":%d" % line, kind="preempt", profile=prof, nodes=ns, pods=pods, pod=preemptor,
                        statuses=st, extenders=list(extenders), pdbs=[], now=NOW, order="given",
                        expect_preempt={"node": expected_node, "victims": sorted(expected)}))

    def running(name, prio, nn, containers=None, labels=None):
        o = p(name, prio, nn, containers, labels=labels)
        o["status"]["phase"] = "Running"
        return o

    def pod1(policy=lower):
        o = p("pod1", HIGH, containers=VLARGE)
        if policy is not None:
            o["spec"]["preemptionPolicy"] = policy
        return o

    base = lambda: [running("m1.1", LOW, "machine1", SMALL), running("m1.2", LOW, "machine1", SMALL),  # noqa: E731
                    running("m2.1", HIGH, "machine2", LARGE), running("m3.1", MID, "machine3", MEDIUM)]
    ext_pods = lambda: [running("m1.1", MID, "machine1", SMALL), running("m1.2", LOW, "machine1", SMALL),  # noqa: E731
                        running("m2.1", MID, "machine2", LARGE)]
    pre("basic preemption logic", 2074, pod1(), base(), "machine1", ["m1.1", "m1.2"])
    pre("One node doesn't need any preemption", 2095, pod1(), base()[:3], "machine3", [])
    foo = {"matchExpressions": [{"key": "foo", "operator": "Exists"}]}
    tsc = [{"maxSkew": 1, "topologyKey": "zone", "whenUnsatisfiable": "DoNotSchedule", "labelSelector": foo},
           {"maxSkew": 1, "topologyKey": "hostname", "whenUnsatisfiable": "DoNotSchedule", "labelSelector": foo}]
    fl = {"foo": ""}
    pre("preemption for topology spread constraints", 2116,
        p("p", HIGH, uid=False, labels=fl, topologySpreadConstraints=tsc),
        [running("pod-a1", HIGH, "node-a", labels=fl), running("pod-a2", HIGH, "node-a", labels=fl),
         running("pod-b1", LOW, "node-b", labels=fl), running("pod-x1", HIGH, "node-x", labels=fl),
         running("pod-x2", HIGH, "node-x", labels=fl)],
        "node-b", ["pod-b1"], plugins=("PodTopologySpread",), node_names=["node-a/zone1", "node-b/zone1", "node-x/zone2"],
        statuses={"node-a": U, "node-b": U, "node-x": U})
    pre("Scheduler extenders allow only machine1, otherwise machine3 would have been chosen", 2201, pod1(), ext_pods(),
        "machine1", ["m1.1", "m1.2"], extenders=[{"predicates": ["true"]}, {"predicates": ["machine1"]}])
    pre("Scheduler extenders do not allow any preemption", 2230, pod1(), ext_pods(), "", [],
        extenders=[{"predicates": ["false"]}])
    pre("One scheduler extender allows only machine1, the other returns error but ignorable. Only machine1 would be "
        "chosen", 2256, pod1(), ext_pods(), "machine1", ["m1.1", "m1.2"],
        extenders=[{"predicates": ["error"], "ignorable": True}, {"predicates": ["machine1"]}])
    pre("One scheduler extender allows only machine1, but it is not interested in given pod, otherwise machine1 would "
        "have been chosen", 2286, pod1(), ext_pods(), "machine3", [],
        extenders=[{"predicates": ["machine1"], "uninterested": True}, {"predicates": ["true"]}])
    pre("no preempting in pod", 2316, pod1(never), base(), "", [])
    pre("PreemptionPolicy is nil", 2337, pod1(None), base(), "machine1", ["m1.1", "m1.2"])
    return out


def all_cases():
    return select_nodes() + pick_one() + might_help() + preempt_cases()

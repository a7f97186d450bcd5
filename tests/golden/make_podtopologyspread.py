"""Golden vectors transcribed from pkg/scheduler/framework/plugins/podtopologyspread/
{filtering_test.go (TestPreFilterState, TestPreFilterStateAddPod, TestPreFilterStateRemovePod,
TestSingleConstraint, TestMultipleConstraints), scoring_test.go (TestPreScoreStateEmptyNodes,
TestPodTopologySpreadScore)}.

The state tables (kind pts_state) compare cycle state (pairs, critical paths, constraints).  They run
on the oracle (tests/test_oracle_golden.py) and on the device (tests/test_pts_state_device.py): the
PreFilter / PreScore rows through kgpu_debug_pts_state, the AddPod / RemovePod rows as ADD_POD /
REMOVE_POD deltas (kgpu_apply_delta) followed by the same export."""
from gen_common import case
from st import DO_NOT_SCHEDULE as DNS, HOSTNAME, LS, N, P, SCHEDULE_ANYWAY as SA

FSRC = "pkg/scheduler/framework/plugins/podtopologyspread/filtering_test.go"
SSRC = "pkg/scheduler/framework/plugins/podtopologyspread/scoring_test.go"
REASON = "node(s) didn't match pod topology spread constraints"


def nz(name, zone, node_label=None, zone_key="zone"):
    n = N().name(name)
    if zone is not None:
        n.label(zone_key, zone)
    n.label("node", node_label or name)
    return n.obj()


def nh(name, zone=None, host_key=HOSTNAME):
    n = N().name(name)
    if zone is not None:
        n.label("zone", zone)
    n.label(host_key, name)
    return n.obj()


def ep(name, node, labels=(("foo", ""),), ns=None, terminating=False):
    p = P().name(name).node(node)
    if ns:
        p.namespace(ns)
    for k, v in labels:
        p.label(k, v)
    if terminating:
        p.terminating()
    return p.obj()


def foo():
    return LS().exists("foo").obj()


def bar():
    return LS().exists("bar").obj()


FOUR = lambda: [nz("node-a", "zone1"), nz("node-b", "zone1"), nz("node-x", "zone2"), nz("node-y", "zone2")]  # noqa


def spread_2103():
    """The tables' recurring 2/1/0/3 distribution."""
    return [ep("p-a1", "node-a"), ep("p-a2", "node-a"), ep("p-b1", "node-b"), ep("p-y1", "node-y"),
            ep("p-y2", "node-y"), ep("p-y3", "node-y")]


def filter_cases():
    out = []

    def fc(name, line, pod, nodes, existing, fits):
        exp = {n: ({"code": 0, "reasons": []} if ok else {"code": 2, "reasons": [REASON]}) for n, ok in fits.items()}
        out.append(case(name, FSRC + ":%d" % line, kind="filter", plugin="PodTopologySpread", args={}, pod=pod,
                        pods=existing, nodes=nodes, expect_filter=exp))

    A, B, X, Y = "node-a", "node-b", "node-x", "node-y"
    allfit = {A: True, B: True, X: True, Y: True}
    # ---- TestSingleConstraint
    fc("no existing pods", 1155, P().name("p").label("foo", "").spread(1, "zone", DNS, foo()).obj(), FOUR(), [],
       allfit)
    fc("no existing pods, incoming pod doesn't match itself", 1173,
       P().name("p").label("foo", "").spread(1, "zone", DNS, bar()).obj(), FOUR(), [], allfit)
    fc("existing pods in a different namespace do not count", 1191,
       P().name("p").label("foo", "").spread(1, "zone", DNS, foo()).obj(), FOUR(),
       [ep("p-a1", A, ns="ns1"), ep("p-b1", A, ns="ns2"), ep("p-x1", X), ep("p-y1", Y)],
       {A: True, B: True, X: False, Y: False})
    fc("pods spread across zones as 3/3, all nodes fit", 1215,
       P().name("p").label("foo", "").spread(1, "zone", DNS, foo()).obj(), FOUR(),
       [ep("p-a1", A), ep("p-a2", A), ep("p-b1", B), ep("p-y1", Y), ep("p-y2", Y), ep("p-y3", Y)], allfit)
    fc("pods spread across zones as 1/2 due to absence of label 'zone' on node-b", 1243,
       P().name("p").label("foo", "").spread(1, "zone", DNS, foo()).obj(),
       [nz(A, "zone1"), nz(B, "zone1", zone_key="zon"), nz(X, "zone2"), nz(Y, "zone2")],
       [ep("p-a1", A), ep("p-b1", B), ep("p-x1", X), ep("p-y1", Y)],
       {A: True, B: False, X: False, Y: False})
    fc("pods spread across nodes as 2/1/0/3, only node-x fits", 1267,
       P().name("p").label("foo", "").spread(1, "node", DNS, foo()).obj(), FOUR(), spread_2103(),
       {A: False, B: False, X: True, Y: False})
    fc("pods spread across nodes as 2/1/0/3, maxSkew is 2, node-b and node-x fit", 1293,
       P().name("p").label("foo", "").spread(2, "node", DNS, foo()).obj(), FOUR(), spread_2103(),
       {A: False, B: True, X: True, Y: False})
    fc("pods spread across nodes as 2/1/0/3, but pod doesn't match itself", 1323,
       P().name("p").label("bar", "").spread(1, "node", DNS, foo()).obj(), FOUR(), spread_2103(),
       {A: False, B: True, X: True, Y: False})
    fc("incoming pod has nodeAffinity, pods spread as 2/~1~/~0~/3, hence node-a fits", 1354,
       P().name("p").label("foo", "").node_affinity_in("node", [A, Y]).spread(1, "node", DNS, foo()).obj(),
       FOUR(), spread_2103(), {A: True, B: True, X: True, Y: False})
    fc("terminating Pods should be excluded", 1381,
       P().name("p").label("foo", "").spread(1, "node", DNS, foo()).obj(),
       [N().name(A).label("node", A).obj(), N().name(B).label("node", B).obj()],
       [ep("p-a", A, terminating=True), ep("p-b", B)], {A: True, B: False})
    # ---- TestMultipleConstraints
    two = lambda s1, s2: P().name("p").label("foo", "").spread(1, "zone", DNS, s1).spread(1, "node", DNS, s2)  # noqa
    fc("two Constraints on zone and node, spreads = [3/3, 2/1/0/3]", 1432, two(foo(), foo()).obj(), FOUR(),
       spread_2103(), {A: False, B: False, X: True, Y: False})
    fc("two Constraints on zone and node, spreads = [3/4, 2/1/0/4]", 1462, two(foo(), foo()).obj(), FOUR(),
       spread_2103() + [ep("p-y4", Y)], {A: False, B: False, X: False, Y: False})
    fc("Constraints hold different labelSelectors, spreads = [1/0, 1/0/0/1]", 1493,
       two(foo(), bar()).label("bar", "").obj(), FOUR(),
       [ep("p-a1", A), ep("p-y1", Y, labels=(("bar", ""),))], {A: False, B: False, X: True, Y: False})
    fc("Constraints hold different labelSelectors, spreads = [1/0, 0/0/1/1]", 1519,
       two(foo(), bar()).label("bar", "").obj(), FOUR(),
       [ep("p-a1", A), ep("p-x1", X, labels=(("bar", ""),)), ep("p-y1", Y, labels=(("bar", ""),))],
       {A: False, B: False, X: False, Y: False})
    fc("Constraints hold different labelSelectors, spreads = [2/3, 1/0/0/1]", 1546,
       two(foo(), bar()).label("bar", "").obj(), FOUR(),
       [ep("p-a1", A), ep("p-a2", A, labels=(("foo", ""), ("bar", ""))), ep("p-y1", Y),
        ep("p-y2", Y, labels=(("foo", ""), ("bar", ""))), ep("p-y3", Y)],
       {A: False, B: True, X: False, Y: False})
    fc("Constraints hold different labelSelectors but pod doesn't match itself on 'zone' constraint", 1575,
       P().name("p").label("bar", "").spread(1, "zone", DNS, foo()).spread(1, "node", DNS, bar()).obj(), FOUR(),
       [ep("p-a1", A), ep("p-x1", X, labels=(("bar", ""),)), ep("p-y1", Y, labels=(("bar", ""),))],
       {A: True, B: True, X: False, Y: False})
    return out


def score_cases():
    out = []

    def sc(name, line, pod, nodes, failed, existing, want):
        allnodes = nodes + failed
        out.append(case(name, SSRC + ":%d" % line, kind="score", plugin="PodTopologySpread", args={}, pod=pod,
                        pods=existing, nodes=allnodes, filtered=[n["metadata"]["name"] for n in nodes],
                        normalize=True, expect_scores=want))

    def host_pod(skew=1, key=HOSTNAME, sel=None):
        return P().name("p").label("foo", "").spread(skew, key, SA, sel or foo()).obj()

    A, B, C, D, X, Y = "node-a", "node-b", "node-c", "node-d", "node-x", "node-y"
    sc("one constraint on node, no existing pods", 237, host_pod(), [nh(A), nh(B)], [], [], {A: 100, B: 100})
    sc("one constraint on node, only one node is candidate", 252, host_pod(), [nh(A)], [nh(B)],
       [ep("p-a1", A), ep("p-a2", A), ep("p-b1", B)], {A: 100})
    sc("one constraint on node, all nodes have the same number of matching pods", 272, host_pod(),
       [nh(A), nh(B)], [], [ep("p-a1", A), ep("p-b1", B)], {A: 100, B: 100})
    e2103 = [ep("p-a1", A), ep("p-a2", A), ep("p-b1", B), ep("p-d1", D), ep("p-d2", D), ep("p-d3", D)]
    sc("one constraint on node, all 4 nodes are candidates", 291, host_pod(), [nh(A), nh(B), nh(C), nh(D)], [],
       e2103, {A: 40, B: 80, C: 100, D: 0})
    sc("one constraint on node, all 4 nodes are candidates, maxSkew=2", 320, host_pod(2),
       [nh(A), nh(B), nh(C), nh(D)], [], e2103, {A: 60, B: 100, C: 100, D: 20})
    e4321 = ([ep("p-a%d" % i, A) for i in range(1, 5)] + [ep("p-b%d" % i, B) for i in range(1, 4)] +
             [ep("p-c1", C), ep("p-c2", C), ep("p-d1", D)])
    sc("one constraint on node, all 4 nodes are candidates, maxSkew=3", 349, host_pod(3),
       [nh(A), nh(B), nh(C), nh(D)], [], e4321, {A: 42, B: 71, C: 100, D: 100})
    e4213 = ([ep("p-a%d" % i, A) for i in range(1, 5)] + [ep("p-b1", B), ep("p-b2", B), ep("p-x1", X)] +
             [ep("p-y%d" % i, Y) for i in range(1, 4)])
    sc("one constraint on node, 3 out of 4 nodes are candidates", 381, host_pod(), [nh(A), nh(B), nh(X)], [nh(Y)],
       e4213, {A: 16, B: 66, X: 100})
    sc("one constraint on node, 3 out of 4 nodes are candidates, one node doesn't match topology key", 413,
       host_pod(), [nh(A), nh(B, host_key="n"), nh(X)], [nh(Y)], e4213, {A: 20, B: 0, X: 100})
    sc("one constraint on zone, 3 out of 4 nodes are candidates", 445, host_pod(key="zone"),
       [nh(A, "zone1"), nh(B, "zone1"), nh(X, "zone2")], [nh(Y, "zone2")], e4213, {A: 62, B: 62, X: 100})
    twoc = lambda s2: P().name("p").label("foo", "").label("bar", "").spread(1, "zone", SA, foo()).spread(  # noqa
        1, HOSTNAME, SA, s2).obj()
    sc("two Constraints on zone and node, 2 out of 4 nodes are candidates", 477,
       P().name("p").label("foo", "").spread(1, "zone", SA, foo()).spread(1, HOSTNAME, SA, foo()).obj(),
       [nh(A, "zone1"), nh(X, "zone2")], [nh(B, "zone1"), nh(Y, "zone2")],
       [ep("p-a1", A), ep("p-a2", A), ep("p-b1", B), ep("p-x1", X), ep("p-x2", X)] +
       [ep("p-y%d" % i, Y) for i in range(1, 5)], {A: 100, X: 54})
    FB = (("foo", ""), ("bar", ""))
    sc("two Constraints on zone and node, with different labelSelectors", 517, twoc(bar()),
       [nh(A, "zone1"), nh(B, "zone1"), nh(X, "zone2"), nh(Y, "zone2")], [],
       [ep("p-a1", A), ep("p-b1", B, labels=FB), ep("p-y1", Y), ep("p-y2", Y, labels=(("bar", ""),))],
       {A: 75, B: 25, X: 100, Y: 50})
    sc("two Constraints on zone and node, with different labelSelectors, some nodes have 0 pods", 545, twoc(bar()),
       [nh(A, "zone1"), nh(B, "zone1"), nh(X, "zone2"), nh(Y, "zone2")], [],
       [ep("p-b1", B, labels=(("bar", ""),)), ep("p-x1", X), ep("p-y1", Y, labels=FB)],
       {A: 100, B: 75, X: 50, Y: 0})
    sc("two Constraints on zone and node, with different labelSelectors, 3 out of 4 nodes are candidates", 572,
       twoc(bar()), [nh(A, "zone1"), nh(B, "zone1"), nh(X, "zone2")], [nh(Y, "zone2")],
       [ep("p-a1", A), ep("p-b1", B, labels=FB), ep("p-y1", Y), ep("p-y2", Y, labels=(("bar", ""),))],
       {A: 75, B: 25, X: 100})
    sc("existing pods in a different namespace do not count", 598, host_pod(), [nh(A), nh(B)], [],
       [ep("p-a1", A, ns="ns1"), ep("p-a2", A), ep("p-b1", B), ep("p-b2", B)], {A: 100, B: 50})
    sc("terminating Pods should be excluded", 618, host_pod(), [nh(A), nh(B)], [],
       [ep("p-a", A, terminating=True), ep("p-b", B)], {A: 100, B: 0})
    return out


MAXI = 2 ** 31 - 1


def svc_obj(selector):
    return {"metadata": {"name": "svc", "namespace": ""}, "spec": {"selector": dict(selector)}}


def rs_obj(sel):
    return {"metadata": {"name": "rs", "namespace": ""}, "spec": {"selector": sel}}


def state_cases():
    out = []
    A, B, X, Y = "node-a", "node-b", "node-x", "node-y"

    def sc(name, line, pod, nodes, existing, want, op="prefilter", op_pod=None, op_node=None, default=(),
           services=(), rss=()):
        kw = dict(op=op)
        if op_pod is not None:
            kw.update(op_pod=op_pod, op_node=op_node)
        out.append(case(name, FSRC + ":%d" % line if op != "prescore" else SSRC + ":%d" % line, kind="pts_state",
                        plugin="PodTopologySpread", args={"default_constraints": list(default)}, pod=pod,
                        pods=existing, nodes=nodes, services=list(services), rss=list(rss), expect_state=want,
                        **kw))

    def want(cons, paths, pairs):
        return {"constraints": cons, "paths": {k: [list(a), list(b)] for k, (a, b) in paths.items()},
                "pairs": [list(x) for x in pairs]}

    zf, nf, nb = [1, "zone", foo()], [1, "node", foo()], [1, "node", bar()]
    pfoo = lambda: P().name("p").label("foo", "")  # noqa
    # ---- TestPreFilterState
    sc("clean cluster with one spreadConstraint", 70,
       pfoo().spread(5, "zone", DNS, LS().label("foo", "bar").obj()).obj(), FOUR(), [],
       want([[5, "zone", LS().label("foo", "bar").obj()]], {"zone": (("zone1", 0), ("zone2", 0))},
            [("zone", "zone1", 0), ("zone", "zone2", 0)]))
    five = [ep("p-a1", A), ep("p-a2", A), ep("p-b1", B), ep("p-y1", Y), ep("p-y2", Y)]
    sc("normal case with one spreadConstraint", 90, pfoo().spread(1, "zone", DNS, foo()).obj(), FOUR(), five,
       want([zf], {"zone": (("zone2", 2), ("zone1", 3))}, [("zone", "zone1", 3), ("zone", "zone2", 2)]))
    six = FOUR() + [nz("node-o", "zone3"), nz("node-p", "zone3")]
    sc("normal case with one spreadConstraint, on a 3-zone cluster", 117,
       pfoo().spread(1, "zone", DNS, LS().exists("foo").obj()).obj(), six, five,
       want([zf], {"zone": (("zone3", 0), ("zone2", 2))},
            [("zone", "zone1", 3), ("zone", "zone2", 2), ("zone", "zone3", 0)]))
    sc("namespace mismatch doesn't count", 147, pfoo().spread(1, "zone", DNS, foo()).obj(), FOUR(),
       [ep("p-a1", A), ep("p-a2", A, ns="ns1"), ep("p-b1", B), ep("p-y1", Y, ns="ns2"), ep("p-y2", Y)],
       want([zf], {"zone": (("zone2", 1), ("zone1", 2))}, [("zone", "zone1", 2), ("zone", "zone2", 1)]))
    seven = [ep("p-a1", A), ep("p-a2", A), ep("p-b1", B), ep("p-y1", Y), ep("p-y2", Y), ep("p-y3", Y), ep("p-y4", Y)]
    sc("normal case with two spreadConstraints", 174,
       pfoo().spread(1, "zone", DNS, foo()).spread(1, "node", DNS, foo()).obj(), FOUR(), seven,
       want([zf, nf], {"zone": (("zone1", 3), ("zone2", 4)), "node": (("node-x", 0), ("node-b", 1))},
            [("zone", "zone1", 3), ("zone", "zone2", 4), ("node", A, 2), ("node", B, 1), ("node", X, 0),
             ("node", Y, 4)]))
    three = [nz(A, "zone1"), nz(B, "zone1"), nz(Y, "zone2")]
    sc("soft spreadConstraints should be bypassed", 214,
       pfoo().spread(1, "zone", SA, foo()).spread(1, "zone", DNS, foo()).spread(1, "node", SA, foo())
       .spread(1, "node", DNS, foo()).obj(), three, seven,
       want([zf, nf], {"zone": (("zone1", 3), ("zone2", 4)), "node": (("node-b", 1), ("node-a", 2))},
            [("zone", "zone1", 3), ("zone", "zone2", 4), ("node", A, 2), ("node", B, 1), ("node", Y, 4)]))
    pfb = lambda: P().name("p").label("foo", "").label("bar", "").spread(1, "zone", DNS, foo()).spread(  # noqa
        1, "node", DNS, bar()).obj()
    sc("different labelSelectors - simple version", 254, pfb(), three,
       [ep("p-a", A), ep("p-b", B, labels=(("bar", ""),))],
       want([zf, nb], {"zone": (("zone2", 0), ("zone1", 1)), "node": (("node-a", 0), ("node-y", 0))},
            [("zone", "zone1", 1), ("zone", "zone2", 0), ("node", A, 0), ("node", B, 1), ("node", Y, 0)]))
    fb = (("foo", ""), ("bar", ""))
    sc("different labelSelectors - complex pods", 287, pfb(), three,
       [ep("p-a1", A), ep("p-a2", A, labels=fb), ep("p-b1", B), ep("p-y1", Y), ep("p-y2", Y, labels=fb),
        ep("p-y3", Y), ep("p-y4", Y, labels=fb)],
       want([zf, nb], {"zone": (("zone1", 3), ("zone2", 4)), "node": (("node-b", 0), ("node-a", 1))},
            [("zone", "zone1", 3), ("zone", "zone2", 4), ("node", A, 1), ("node", B, 0), ("node", Y, 2)]))
    sc("two spreadConstraints, and with podAffinity", 325,
       pfoo().node_affinity_not_in("node", ["node-x"]).spread(1, "zone", DNS, foo()).spread(1, "node", DNS, foo())
       .obj(), FOUR(), seven,
       want([zf, nf], {"zone": (("zone1", 3), ("zone2", 4)), "node": (("node-b", 1), ("node-a", 2))},
            [("zone", "zone1", 3), ("zone", "zone2", 4), ("node", A, 2), ("node", B, 1), ("node", Y, 4)]))
    fbar = LS().label("foo", "bar").obj()
    empty_paths = (("", MAXI), ("", MAXI))
    sc("default constraints and a service", 364, P().name("p").label("foo", "bar").label("baz", "kar").obj(), [], [],
       want([[3, "node", fbar], [5, "rack", fbar]], {"node": empty_paths, "rack": empty_paths}, []),
       default=[{"maxSkew": 3, "topologyKey": "node", "whenUnsatisfiable": DNS},
                {"maxSkew": 2, "topologyKey": "node", "whenUnsatisfiable": SA},
                {"maxSkew": 5, "topologyKey": "rack", "whenUnsatisfiable": DNS}],
       services=[svc_obj({"foo": "bar"})])
    sc("default constraints and a service that doesn't match", 393, P().name("p").label("foo", "bar").obj(), [], [],
       want([], {}, []), default=[{"maxSkew": 3, "topologyKey": "node", "whenUnsatisfiable": DNS}],
       services=[svc_obj({"baz": "kep"})])
    sc("default constraints and a service, but pod has constraints", 404,
       P().name("p").label("foo", "bar").label("baz", "tar").spread(1, "zone", DNS, LS().label("baz", "tar").obj())
       .spread(2, "planet", SA, LS().label("fot", "rok").obj()).obj(), [], [],
       want([[1, "zone", LS().label("baz", "tar").obj()]], {"zone": empty_paths}, []),
       default=[{"maxSkew": 2, "topologyKey": "node", "whenUnsatisfiable": DNS}],
       services=[svc_obj({"foo": "bar"})])
    sc("default soft constraints and a service", 428, P().name("p").label("foo", "bar").obj(), [], [],
       want([], {}, []), default=[{"maxSkew": 2, "topologyKey": "node", "whenUnsatisfiable": SA}],
       services=[svc_obj({"foo": "bar"})])

    # ---- TestPreFilterStateAddPod
    two = [nz(A, "zone1"), nz(B, "zone1")]
    ax = [nz(A, "zone1"), nz(X, "zone2")]
    abx = [nz(A, "zone1"), nz(B, "zone1"), nz(X, "zone2")]
    pn = lambda: pfoo().spread(1, "node", DNS, LS().exists("foo").obj()).obj()  # noqa
    pzn = lambda: pfoo().spread(1, "zone", DNS, foo()).spread(1, "node", DNS, foo()).obj()  # noqa

    def add(name, line, pod, added, existing, node_idx, nodes, w):
        sc(name, line, pod, nodes, existing, w, op="add", op_pod=added, op_node=nodes[node_idx]["metadata"]["name"])

    add("node a and b both impact current min match", 559, pn(), ep("p-a1", A), [], 0, two,
        want([nf], {"node": (("node-b", 0), ("node-a", 1))}, [("node", A, 1), ("node", B, 0)]))
    add("only node a impacts current min match", 581, pn(), ep("p-a1", A), [ep("p-b1", B)], 0, two,
        want([nf], {"node": (("node-a", 1), ("node-b", 1))}, [("node", A, 1), ("node", B, 1)]))
    add("add a pod in a different namespace doesn't change topologyKeyToMinPodsMap", 605, pn(),
        ep("p-a1", A, ns="ns1"), [ep("p-b1", B)], 0, two,
        want([nf], {"node": (("node-a", 0), ("node-b", 1))}, [("node", A, 0), ("node", B, 1)]))
    add("add pod on non-critical node won't trigger re-calculation", 629, pn(), ep("p-b2", B), [ep("p-b1", B)], 1,
        two, want([nf], {"node": (("node-a", 0), ("node-b", 2))}, [("node", A, 0), ("node", B, 2)]))
    add("node a and x both impact topologyKeyToMinPodsMap on zone and node", 653, pzn(), ep("p-a1", A), [], 0, ax,
        want([zf, nf], {"zone": (("zone2", 0), ("zone1", 1)), "node": (("node-x", 0), ("node-a", 1))},
             [("zone", "zone1", 1), ("zone", "zone2", 0), ("node", A, 1), ("node", X, 0)]))
    add("only node a impacts topologyKeyToMinPodsMap on zone and node", 678, pzn(), ep("p-a1", A), [ep("p-x1", X)],
        0, ax, want([zf, nf], {"zone": (("zone1", 1), ("zone2", 1)), "node": (("node-a", 1), ("node-x", 1))},
                    [("zone", "zone1", 1), ("zone", "zone2", 1), ("node", A, 1), ("node", X, 1)]))
    add("node a impacts topologyKeyToMinPodsMap on node, node x impacts topologyKeyToMinPodsMap on zone", 705,
        pzn(), ep("p-a1", A), [ep("p-b1", B), ep("p-b2", B), ep("p-x1", X)], 0, abx,
        want([zf, nf], {"zone": (("zone2", 1), ("zone1", 3)), "node": (("node-a", 1), ("node-x", 1))},
             [("zone", "zone1", 3), ("zone", "zone2", 1), ("node", A, 1), ("node", B, 2), ("node", X, 1)]))
    add("Constraints hold different labelSelectors, node a impacts topologyKeyToMinPodsMap on zone", 735, pfb(),
        ep("p-a1", A), [ep("p-b1", B, labels=fb), ep("p-x1", X, labels=fb), ep("p-x2", X, labels=(("bar", ""),))],
        0, abx, want([zf, nb], {"zone": (("zone2", 1), ("zone1", 2)), "node": (("node-a", 0), ("node-b", 1))},
                     [("zone", "zone1", 2), ("zone", "zone2", 1), ("node", A, 0), ("node", B, 1), ("node", X, 2)]))
    add("Constraints hold different labelSelectors, node a impacts topologyKeyToMinPodsMap on both zone and node", 773,
        pfb(), ep("p-a1", A, labels=fb),
        [ep("p-b1", B, labels=(("bar", ""),)), ep("p-x1", X, labels=fb), ep("p-x2", X, labels=(("bar", ""),))],
        0, abx, want([zf, nb], {"zone": (("zone1", 1), ("zone2", 1)), "node": (("node-a", 1), ("node-b", 1))},
                     [("zone", "zone1", 1), ("zone", "zone2", 1), ("node", A, 1), ("node", B, 1), ("node", X, 2)]))

    # ---- TestPreFilterStateRemovePod
    pz = lambda: pfoo().spread(1, "zone", DNS, foo()).obj()  # noqa

    def rm(name, line, pod, nodes, existing, deleted, node_idx, w):
        sc(name, line, pod, nodes, existing, w, op="remove", op_pod=deleted,
           op_node=nodes[node_idx]["metadata"]["name"])

    abxy = [nz(A, "zone1"), nz(B, "zone1"), nz(X, "zone2"), nz(Y, "zone2")]
    e3 = [ep("p-a1", A), ep("p-b1", B), ep("p-x1", X)]
    rm("one spreadConstraint on zone, topologyKeyToMinPodsMap unchanged", 876, pz(), abx, e3, e3[0], 0,
       want([zf], {"zone": (("zone1", 1), ("zone2", 1))}, [("zone", "zone1", 1), ("zone", "zone2", 1)]))
    e4 = [ep("p-a1", A), ep("p-b1", B), ep("p-x1", X), ep("p-y1", Y)]
    rm("one spreadConstraint on node, topologyKeyToMinPodsMap changed", 902, pz(), abxy, e4, e4[0], 0,
       want([zf], {"zone": (("zone1", 1), ("zone2", 2))}, [("zone", "zone1", 1), ("zone", "zone2", 2)]))
    e5 = [ep("p-a0", A, labels=(("bar", ""),))] + e4
    rm("delete an irrelevant pod won't help", 930, pz(), abxy, e5, e5[0], 0,
       want([zf], {"zone": (("zone1", 2), ("zone2", 2))}, [("zone", "zone1", 2), ("zone", "zone2", 2)]))
    rm("delete a non-existing pod won't help", 959, pz(), abxy, e4, ep("p-a0", A, labels=(("bar", ""),)), 0,
       want([zf], {"zone": (("zone1", 2), ("zone2", 2))}, [("zone", "zone1", 2), ("zone", "zone2", 2)]))
    e6 = [ep("p-a1", A), ep("p-a2", A), ep("p-b1", B), ep("p-x1", X), ep("p-x2", X)]
    rm("two spreadConstraints", 988, pzn(), abx, e6, e6[3], 2,
       want([zf, nf], {"zone": (("zone2", 1), ("zone1", 3)), "node": (("node-b", 1), ("node-x", 1))},
            [("zone", "zone1", 3), ("zone", "zone2", 1), ("node", A, 2), ("node", B, 1), ("node", X, 1)]))

    # ---- scoring_test.go TestPreScoreStateEmptyNodes
    def ps(name, line, pod, nodes, w, default=(), rss=()):
        sc(name, line, pod, nodes, [], w, op="prescore", default=default, rss=rss)

    H = HOSTNAME
    nzh = lambda n, z: N().name(n).label("zone", z).label(H, n).obj()  # noqa
    ps("normal case", 48, pfoo().spread(1, "zone", SA, foo()).spread(1, H, SA, foo()).obj(),
       [nzh(A, "zone1"), nzh(B, "zone1"), nzh(X, "zone2")],
       {"constraints": [[1, "zone", foo()], [1, H, foo()]], "ignored": [],
        "pairs": [["zone", "zone1", 0], ["zone", "zone2", 0]], "weight_sizes": [2, 3]})
    ps("node-x doesn't have label zone", 77, pfoo().spread(1, "zone", SA, foo()).spread(1, H, SA, bar()).obj(),
       [nzh(A, "zone1"), nzh(B, "zone1"), N().name(X).label(H, X).obj()],
       {"constraints": [[1, "zone", foo()], [1, H, bar()]], "ignored": [X],
        "pairs": [["zone", "zone1", 0]], "weight_sizes": [1, 2]})
    rs_foo = rs_obj(LS().exists("foo").obj())
    ps("defaults constraints and a replica set", 105, P().name("p").label("foo", "tar").label("baz", "sup").obj(),
       [N().name(A).label("rack", "rack1").label(H, A).label("planet", "mars").obj()],
       {"constraints": [[1, H, foo()], [2, "planet", foo()]], "ignored": [],
        "pairs": [["planet", "mars", 0]], "weight_sizes": [1, 1]},
       default=[{"maxSkew": 1, "topologyKey": H, "whenUnsatisfiable": SA},
                {"maxSkew": 2, "topologyKey": "rack", "whenUnsatisfiable": DNS},
                {"maxSkew": 2, "topologyKey": "planet", "whenUnsatisfiable": SA}], rss=[rs_foo])
    ps("defaults constraints and a replica set that doesn't match", 138,
       P().name("p").label("foo", "bar").label("baz", "sup").obj(), [N().name(A).label("planet", "mars").obj()],
       {"constraints": [], "ignored": [], "pairs": [], "weight_sizes": []},
       default=[{"maxSkew": 2, "topologyKey": "planet", "whenUnsatisfiable": SA}],
       rss=[rs_obj(LS().exists("tar").obj())])
    ps("defaults constraints and a replica set, but pod has constraints", 155,
       P().name("p").label("foo", "bar").label("baz", "sup").spread(1, "zone", DNS, LS().label("foo", "bar").obj())
       .spread(2, "planet", SA, LS().label("baz", "sup").obj()).obj(),
       [N().name(A).label("planet", "mars").label("galaxy", "andromeda").obj()],
       {"constraints": [[2, "planet", LS().label("baz", "sup").obj()]], "ignored": [],
        "pairs": [["planet", "mars", 0]], "weight_sizes": [1]},
       default=[{"maxSkew": 2, "topologyKey": "galaxy", "whenUnsatisfiable": SA}], rss=[rs_foo])
    return out


def all_cases():
    return filter_cases() + score_cases() + state_cases()

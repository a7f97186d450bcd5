"""Golden vectors transcribed from pkg/scheduler/framework/plugins/podtopologyspread/
{filtering_test.go (TestPreFilterState, TestSingleConstraint, TestMultipleConstraints),
scoring_test.go (TestPodTopologySpreadScore)}."""
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


def all_cases():
    return filter_cases() + score_cases()

"""Golden vectors transcribed from pkg/scheduler/framework/plugins/tainttoleration/taint_toleration_test.go."""
from gen_common import case, node, pod

SRC = "pkg/scheduler/framework/plugins/tainttoleration/taint_toleration_test.go"


def tol(key, value=None, effect=None, op=None):
    t = {"key": key}
    if op is not None:
        t["operator"] = op
    if value is not None:
        t["value"] = value
    if effect is not None:
        t["effect"] = effect
    return t


def taint(key, value, effect):
    return {"key": key, "value": value, "effect": effect}


def pwt(tols):
    return pod(name="pod1", tolerations=tols)


def nwt(name, taints):
    return node(name, {}, taints=taints)


PNS, NS = "PreferNoSchedule", "NoSchedule"


def score_cases():
    out = []

    def sc(name, line, p, nodes, exp):
        out.append(case(name, SRC + ":%d" % line, kind="score", plugin="TaintToleration", args={}, pod=p,
                        pods=[], nodes=nodes, normalize=True, expect_scores=exp))

    sc("node with taints tolerated by the pod, gets a higher score than those node with intolerable taints", 61,
       pwt([tol("foo", "bar", PNS, "Equal")]),
       [nwt("nodeA", [taint("foo", "bar", PNS)]), nwt("nodeB", [taint("foo", "blah", PNS)])],
       {"nodeA": 100, "nodeB": 0})
    sc("the nodes that all of their taints are tolerated by the pod, get the same score, no matter how many "
       "tolerable taints a node has", 87,
       pwt([tol("cpu-type", "arm64", PNS, "Equal"), tol("disk-type", "ssd", PNS, "Equal")]),
       [nwt("nodeA", []), nwt("nodeB", [taint("cpu-type", "arm64", PNS)]),
        nwt("nodeC", [taint("cpu-type", "arm64", PNS), taint("disk-type", "ssd", PNS)])],
       {"nodeA": 100, "nodeB": 100, "nodeC": 100})
    sc("the more intolerable taints a node has, the lower score it gets.", 130,
       pwt([tol("foo", "bar", PNS, "Equal")]),
       [nwt("nodeA", []), nwt("nodeB", [taint("cpu-type", "arm64", PNS)]),
        nwt("nodeC", [taint("cpu-type", "arm64", PNS), taint("disk-type", "ssd", PNS)])],
       {"nodeA": 100, "nodeB": 50, "nodeC": 0})
    sc("only taints and tolerations that have effect PreferNoSchedule are checked by taints-tolerations "
       "priority function", 166,
       pwt([tol("cpu-type", "arm64", NS, "Equal"), tol("disk-type", "ssd", NS, "Equal")]),
       [nwt("nodeA", []), nwt("nodeB", [taint("cpu-type", "arm64", NS)]),
        nwt("nodeC", [taint("cpu-type", "arm64", PNS), taint("disk-type", "ssd", PNS)])],
       {"nodeA": 100, "nodeB": 100, "nodeC": 0})
    sc("Default behaviour No taints and tolerations, lands on node with no taints", 208,
       pwt([]), [nwt("nodeA", []), nwt("nodeB", [taint("cpu-type", "arm64", PNS)])],
       {"nodeA": 100, "nodeB": 0})
    return out


def filter_cases():
    out = []
    U = 3  # UnschedulableAndUnresolvable

    def fc(name, line, p, n, code=0, reasons=()):
        out.append(case(name, SRC + ":%d" % line, kind="filter", plugin="TaintToleration", args={}, pod=p,
                        pods=[], nodes=[n], expect_filter={"nodeA": {"code": code, "reasons": list(reasons)}}))

    fc("A pod having no tolerations can't be scheduled onto a node with nonempty taints", 269, pwt([]),
       nwt("nodeA", [taint("dedicated", "user1", NS)]), U,
       ["node(s) had taint {dedicated: user1}, that the pod didn't tolerate"])
    fc("A pod which can be scheduled on a dedicated node assigned to user1 with effect NoSchedule", 276,
       pwt([tol("dedicated", "user1", NS)]), nwt("nodeA", [taint("dedicated", "user1", NS)]))
    fc("A pod which can't be scheduled on a dedicated node assigned to user2 with effect NoSchedule", 281,
       pwt([tol("dedicated", "user2", NS, "Equal")]), nwt("nodeA", [taint("dedicated", "user1", NS)]), U,
       ["node(s) had taint {dedicated: user1}, that the pod didn't tolerate"])
    fc("A pod can be scheduled onto the node, with a toleration uses operator Exists that tolerates the taints "
       "on the node", 288, pwt([tol("foo", None, NS, "Exists")]), nwt("nodeA", [taint("foo", "bar", NS)]))
    fc("A pod has multiple tolerations, node has multiple taints, all the taints are tolerated, pod can be "
       "scheduled onto the node", 293,
       pwt([tol("dedicated", "user2", NS, "Equal"), tol("foo", None, NS, "Exists")]),
       nwt("nodeA", [taint("dedicated", "user2", NS), taint("foo", "bar", NS)]))
    fc("toleration keys and values match the taint, but (non-empty) effect doesn't match", 304,
       pwt([tol("foo", "bar", PNS, "Equal")]), nwt("nodeA", [taint("foo", "bar", NS)]), U,
       ["node(s) had taint {foo: bar}, that the pod didn't tolerate"])
    fc("toleration keys and values match the taint, the effect of toleration is empty", 312,
       pwt([tol("foo", "bar", None, "Equal")]), nwt("nodeA", [taint("foo", "bar", NS)]))
    fc("toleration key and value don't match the taint, but the taint effect is PreferNoSchedule", 318,
       pwt([tol("dedicated", "user2", NS, "Equal")]), nwt("nodeA", [taint("dedicated", "user1", PNS)]))
    fc("no toleration, but the effect of taint on node is PreferNoSchedule", 324, pwt([]),
       nwt("nodeA", [taint("dedicated", "user1", PNS)]))
    return out


def all_cases():
    return score_cases() + filter_cases()

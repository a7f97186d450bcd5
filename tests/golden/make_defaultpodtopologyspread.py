"""Golden vectors transcribed from
pkg/scheduler/framework/plugins/defaultpodtopologyspread/default_pod_topology_spread_test.go
(TestDefaultPodTopologySpreadScore, TestZoneSelectorSpreadPriority).

controllerRef() in that file returns nil (its TODO), so no pod carries an owner reference; the
ReplicationController / ReplicaSet / StatefulSet listers still feed DefaultSelector."""
from gen_common import case, node, pod

SRC = "pkg/scheduler/framework/plugins/defaultpodtopologyspread/default_pod_topology_spread_test.go"
ZONE = "failure-domain.beta.kubernetes.io/zone"


def svc(selector, ns=""):
    return {"metadata": {"name": "svc", "namespace": ns}, "spec": {"selector": dict(selector)}}


def rc(selector):
    return {"metadata": {"name": "rc", "namespace": ""}, "spec": {"selector": dict(selector)}}


def rs(match_labels):
    return {"metadata": {"name": "rs", "namespace": ""}, "spec": {"selector": {"matchLabels": dict(match_labels)}}}


def ss(match_labels):
    return {"metadata": {"name": "ss", "namespace": ""}, "spec": {"selector": {"matchLabels": dict(match_labels)}}}


def p(node_name=None, labels=None, ns="", **spec):
    return pod(labels=labels, ns=ns, node_name=node_name, **spec)


def score_cases():
    labels1 = {"foo": "bar", "baz": "blah"}
    labels2 = {"bar": "foo", "baz": "blah"}
    out = []
    names = ["machine1", "machine2"]

    def sc(name, line, pod_, pods, exp, services=(), rcs=(), rss=(), sss=()):
        out.append(case(name, SRC + ":%d" % line, kind="score", plugin="DefaultPodTopologySpread", args={}, pod=pod_,
                        pods=list(pods), nodes=[node(n) for n in names], normalize=True,
                        services=list(services), rcs=list(rcs), rss=list(rss), sss=list(sss),
                        expect_scores=dict(zip(names, exp))))

    m1, m2 = "machine1", "machine2"
    sc("nothing scheduled", 73, p(), [], [100, 100])
    sc("no services", 80, p(labels=labels1), [p(m1)], [100, 100])
    sc("different services", 88, p(labels=labels1), [p(m1, labels2)], [100, 100], services=[svc({"key": "value"})])
    sc("two pods, one service pod", 99, p(labels=labels1), [p(m1, labels2), p(m2, labels1)], [100, 0],
       services=[svc(labels1)])
    sc("five pods, one service pod in no namespace", 113, p(labels=labels1),
       [p(m1, labels2), p(m1, labels1, "default"), p(m1, labels1, "ns1"), p(m2, labels1), p(m2, labels2)],
       [100, 0], services=[svc(labels1)])
    sc("four pods, one service pod in default namespace", 126, p(labels=labels1, ns="default"),
       [p(m1, labels1), p(m1, labels1, "ns1"), p(m2, labels1, "default"), p(m2, labels2)],
       [100, 0], services=[svc(labels1, "default")])
    sc("five pods, one service pod in specific namespace", 140, p(labels=labels1, ns="ns1"),
       [p(m1, labels1), p(m1, labels1, "default"), p(m1, labels1, "ns2"), p(m2, labels1, "ns1"), p(m2, labels2)],
       [100, 0], services=[svc(labels1, "ns1")])
    sc("three pods, two service pods on different machines", 152, p(labels=labels1),
       [p(m1, labels2), p(m1, labels1), p(m2, labels1)], [0, 0], services=[svc(labels1)])
    sc("four pods, three service pods", 164, p(labels=labels1),
       [p(m1, labels2), p(m1, labels1), p(m2, labels1), p(m2, labels1)], [50, 0], services=[svc(labels1)])
    sc("service with partial pod label matches", 175, p(labels=labels1),
       [p(m1, labels2), p(m1, labels1), p(m2, labels1)], [0, 50], services=[svc({"baz": "blah"})])
    three = [p(m1, labels2), p(m1, labels1), p(m2, labels1)]
    sc("service with partial pod label matches with service and replication controller", 189, p(labels=labels1), three,
       [0, 0], services=[svc({"baz": "blah"})], rcs=[rc({"foo": "bar"})])
    sc("service with partial pod label matches with service and replica set", 202, p(labels=labels1), three, [0, 0],
       services=[svc({"baz": "blah"})], rss=[rs({"foo": "bar"})])
    sc("service with partial pod label matches with service and stateful set", 214, p(labels=labels1), three, [0, 0],
       services=[svc({"baz": "blah"})], sss=[ss({"foo": "bar"})])
    both = {"foo": "bar", "bar": "foo"}
    sc("disjoined service and replication controller matches no pods", 227, p(labels=both), three, [100, 100],
       services=[svc({"bar": "foo"})], rcs=[rc({"foo": "bar"})])
    sc("disjoined service and replica set matches no pods", 240, p(labels=both), three, [100, 100],
       services=[svc({"bar": "foo"})], rss=[rs({"foo": "bar"})])
    sc("disjoined service and stateful set matches no pods", 252, p(labels=both), three, [100, 100],
       services=[svc({"bar": "foo"})], sss=[ss({"foo": "bar"})])
    sc("Replication controller with partial pod label matches", 265, p(labels=labels1), three, [0, 0],
       rcs=[rc({"foo": "bar"})])
    sc("Replica set with partial pod label matches", 278, p(labels=labels1), three, [0, 0], rss=[rs({"foo": "bar"})])
    sc("StatefulSet with partial pod label matches", 291, p(labels=labels1), three, [0, 0], sss=[ss({"foo": "bar"})])
    three2 = [p(m1, labels2), p(m1, labels1), p(m2, labels1)]
    sc("Another replication controller with partial pod label matches", 303, p(labels=labels1), three2, [0, 50],
       rcs=[rc({"baz": "blah"})])
    sc("Another replication set with partial pod label matches", 316, p(labels=labels1), three2, [0, 50],
       rss=[rs({"baz": "blah"})])
    sc("Another stateful set with partial pod label matches", 329, p(labels=labels1), three2, [0, 50],
       sss=[ss({"baz": "blah"})])
    tsc = [{"maxSkew": 1, "topologyKey": "foo", "whenUnsatisfiable": "DoNotSchedule"}]
    sc("Another stateful set with TopologySpreadConstraints set in pod", 353,
       p(labels=labels1, topologySpreadConstraints=tsc), three2, [0, 0], sss=[ss({"baz": "blah"})])
    return out


def zone_cases():
    labels1 = {"label1": "l1", "baz": "blah"}
    labels2 = {"label2": "l2", "baz": "blah"}
    z = {"machine1.zone1": "zone1", "machine1.zone2": "zone2", "machine2.zone2": "zone2",
         "machine1.zone3": "zone3", "machine2.zone3": "zone3", "machine3.zone3": "zone3"}
    nodes = [node(n, labels={ZONE: zz}) for n, zz in z.items()]
    order = list(z)
    out = []

    def sc(name, line, pod_, pods, exp, services=(), rcs=()):
        out.append(case(name, SRC + ":%d" % line, kind="score", plugin="DefaultPodTopologySpread", args={}, pod=pod_,
                        pods=list(pods), nodes=nodes, normalize=True, services=list(services), rcs=list(rcs),
                        expect_scores=dict(zip(order, exp))))

    m11, m12, m22, m13, m23, m33 = order
    sc("nothing scheduled", 475, p(), [], [100] * 6)
    sc("no services", 487, p(labels=labels1), [p(m11)], [100] * 6)
    sc("different services", 500, p(labels=labels1), [p(m11, labels2)], [100] * 6, services=[svc({"key": "value"})])
    sc("two pods, 0 matching", 516, p(labels=labels1), [p(m11, labels2), p(m12, labels2)], [100] * 6,
       services=[svc(labels1)])
    sc("two pods, 1 matching (in z2)", 532, p(labels=labels1), [p(m11, labels2), p(m12, labels1)],
       [100, 0, 33, 100, 100, 100], services=[svc(labels1)])
    sc("five pods, 3 matching (z2=2, z3=1)", 551, p(labels=labels1),
       [p(m11, labels2), p(m12, labels1), p(m22, labels1), p(m13, labels2), p(m23, labels1)],
       [100, 0, 0, 66, 33, 66], services=[svc(labels1)])
    sc("four pods, 3 matching (z1=1, z2=1, z3=1)", 569, p(labels=labels1),
       [p(m11, labels1), p(m12, labels1), p(m22, labels2), p(m13, labels1)],
       [0, 0, 33, 0, 33, 33], services=[svc(labels1)])
    sc("five pods, 4 matching (z1=1, z2=2, z3=1)", 588, p(labels=labels1),
       [p(m11, labels1), p(m12, labels1), p(m22, labels1), p(m22, labels2), p(m13, labels1)],
       [33, 0, 0, 33, 66, 66], services=[svc(labels1)])
    sc("Replication controller spreading (z1=0, z2=1, z3=2)", 613, p(labels=labels1),
       [p(m13, labels1), p(m12, labels1), p(m13, labels1)], [100, 50, 66, 0, 33, 33], rcs=[rc(labels1)])
    return out


def all_cases():
    return score_cases() + zone_cases()

"""Golden vectors transcribed from pkg/scheduler/framework/plugins/interpodaffinity/
{scoring_test.go (TestPreferredAffinity, TestPreferredAffinityWithHardPodAffinitySymmetricWeight),
filtering_test.go (TestRequiredAffinitySingleNode, TestRequiredAffinityMultipleNodes,
TestPreFilterStateAddRemovePod, TestGetTPMapMatchingIncomingAffinityAntiAffinity)}.

The two state tables (kind ipa_state, expect_ipa) compare preFilterState's maps: topologyToMatchedAffinityTerms
("aff") and topologyToMatchedAntiAffinityTerms ("anti") as sorted [key, value, count] triples.  Op
"add_remove" is TestPreFilterStateAddRemovePod: the expected maps hold after AddPod(added pod); the
state after AddPod must also equal the PreFilter state of a snapshot that already holds the pod, and
the state after RemovePod must equal the original."""
from gen_common import case

SSRC = "pkg/scheduler/framework/plugins/interpodaffinity/scoring_test.go"
FSRC = "pkg/scheduler/framework/plugins/interpodaffinity/filtering_test.go"


def req(key, op, vals=None):
    e = {"key": key, "operator": op}
    if vals is not None:
        e["values"] = list(vals)
    return e


def term(exprs, topo, ns=None, match_labels=None):
    sel = {}
    if exprs is not None:
        sel["matchExpressions"] = list(exprs)
    if match_labels is not None:
        sel["matchLabels"] = dict(match_labels)
    t = {"labelSelector": sel, "topologyKey": topo}
    if ns is not None:
        t["namespaces"] = list(ns)
    return t


def wterm(w, exprs, topo):
    return {"weight": w, "podAffinityTerm": term(exprs, topo)}


def pod(labels=None, node=None, affinity=None, name="", ns=""):
    m = {"name": name, "namespace": ns}
    if labels is not None:
        m["labels"] = dict(labels)
    s = {}
    if node:
        s["nodeName"] = node
    if affinity is not None:
        s["affinity"] = affinity
    return {"metadata": m, "spec": s}


def node(name, labels=None):
    m = {"name": name}
    if labels is not None:
        m["labels"] = dict(labels)
    return {"metadata": m, "spec": {}, "status": {"allocatable": {}}}


CHINA, INDIA = {"region": "China"}, {"region": "India"}
AZ1, AZ2 = {"az": "az1"}, {"az": "az2"}
CHINA_AZ1 = {"region": "China", "az": "az1"}
S1, S2 = {"security": "S1"}, {"security": "S2"}

STAY_S1_REGION = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    wterm(5, [req("security", "In", ["S1"])], "region")]}}
STAY_S2_REGION = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    wterm(6, [req("security", "In", ["S2"])], "region")]}}
AFFINITY3 = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    wterm(8, [req("security", "NotIn", ["S1"]), req("security", "In", ["S2"])], "region"),
    wterm(2, [req("security", "Exists"), req("wrongkey", "DoesNotExist")], "region")]}}
HARD_AFFINITY = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
    term([req("security", "In", ["S1", "value2"])], "region"),
    term([req("security", "Exists"), req("wrongkey", "DoesNotExist")], "region")]}}
AWAY_S1_AZ = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    wterm(5, [req("security", "In", ["S1"])], "az")]}}
AWAY_S2_AZ = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    wterm(5, [req("security", "In", ["S2"])], "az")]}}
STAY_S1_AWAY_S2 = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    wterm(8, [req("security", "In", ["S1"])], "region")]},
    "podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        wterm(5, [req("security", "In", ["S2"])], "az")]}}


def score_cases():
    out = []

    def sc(name, line, p, existing, nodes, want, hard_weight=1):
        out.append(case(name, SSRC + ":%d" % line, kind="score", plugin="InterPodAffinity",
                        args={"hard_pod_affinity_weight": hard_weight}, pod=p, pods=existing, nodes=nodes,
                        normalize=True, expect_scores=want))

    m = ["machine%d" % i for i in range(6)]
    sc("all machines are same priority as Affinity is nil", 262, pod(S1), [],
       [node(m[1], CHINA), node(m[2], INDIA), node(m[3], AZ1)], {m[1]: 0, m[2]: 0, m[3]: 0})
    sc("Affinity: pod that matches topology key & pods in nodes will get high score comparing to others"
       "which doesn't match either pods in nodes or in topology key", 275, pod(S1, affinity=STAY_S1_REGION),
       [pod(S1, m[1]), pod(S2, m[2]), pod(S1, m[3])], [node(m[1], CHINA), node(m[2], INDIA), node(m[3], AZ1)],
       {m[1]: 100, m[2]: 0, m[3]: 0})
    sc("All the nodes that have the same topology key & label value with one of them has an existing pod that "
       "match the affinity rules, have the same score", 295, pod(None, affinity=STAY_S1_REGION), [pod(S1, m[1])],
       [node(m[1], CHINA), node(m[2], CHINA_AZ1), node(m[3], INDIA)], {m[1]: 100, m[2]: 100, m[3]: 0})
    sc("Affinity: nodes in one region has more matching pods comparing to other reqion, so the region which has "
       "more macthes will get high score", 312, pod(S1, affinity=STAY_S2_REGION),
       [pod(S2, m[1]), pod(S2, m[1]), pod(S2, m[2]), pod(S2, m[3]), pod(S2, m[4]), pod(S2, m[5])],
       [node(m[1], CHINA), node(m[2], INDIA), node(m[3], CHINA), node(m[4], CHINA), node(m[5], INDIA)],
       {m[1]: 100, m[2]: 50, m[3]: 100, m[4]: 100, m[5]: 50})
    sc("Affinity: different Label operators and values for pod affinity scheduling preference, including some "
       "match failures ", 333, pod(S1, affinity=AFFINITY3), [pod(S1, m[1]), pod(S2, m[2]), pod(S1, m[3])],
       [node(m[1], CHINA), node(m[2], INDIA), node(m[3], AZ1)], {m[1]: 20, m[2]: 100, m[3]: 0})
    sc("Affinity symmetry: considered only the preferredDuringSchedulingIgnoredDuringExecution in pod affinity "
       "symmetry", 350, pod(S2), [pod(S1, m[1], STAY_S1_REGION), pod(S2, m[2], STAY_S2_REGION)],
       [node(m[1], CHINA), node(m[2], INDIA), node(m[3], AZ1)], {m[1]: 0, m[2]: 100, m[3]: 0})
    sc("Affinity symmetry: considered RequiredDuringSchedulingIgnoredDuringExecution in pod affinity symmetry", 364,
       pod(S1), [pod(S1, m[1], HARD_AFFINITY), pod(S2, m[2], HARD_AFFINITY)],
       [node(m[1], CHINA), node(m[2], INDIA), node(m[3], AZ1)], {m[1]: 100, m[2]: 100, m[3]: 0})
    sc("Anti Affinity: pod that doesnot match existing pods in node will get high score ", 385,
       pod(S1, affinity=AWAY_S1_AZ), [pod(S1, m[1]), pod(S2, m[2])], [node(m[1], AZ1), node(m[2], CHINA)],
       {m[1]: 0, m[2]: 100})
    sc("Anti Affinity: pod that does not matches topology key & matches the pods in nodes will get higher score "
       "comparing to others ", 398, pod(S1, affinity=AWAY_S1_AZ), [pod(S1, m[1]), pod(S1, m[2])],
       [node(m[1], AZ1), node(m[2], CHINA)], {m[1]: 0, m[2]: 100})
    sc("Anti Affinity: one node has more matching pods comparing to other node, so the node which has more "
       "unmacthes will get high score", 411, pod(S1, affinity=AWAY_S1_AZ),
       [pod(S1, m[1]), pod(S1, m[1]), pod(S2, m[2])], [node(m[1], AZ1), node(m[2], INDIA)], {m[1]: 0, m[2]: 100})
    sc("Anti Affinity symmetry: the existing pods in node which has anti affinity match will get high score", 426,
       pod(S2), [pod(S1, m[1], AWAY_S2_AZ), pod(S2, m[2], AWAY_S1_AZ)], [node(m[1], AZ1), node(m[2], AZ2)],
       {m[1]: 0, m[2]: 100})
    sc("Affinity and Anti Affinity: considered only preferredDuringSchedulingIgnoredDuringExecution in both pod "
       "affinity & anti affinity", 440, pod(S1, affinity=STAY_S1_AWAY_S2), [pod(S1, m[1]), pod(S1, m[2])],
       [node(m[1], CHINA), node(m[2], AZ1)], {m[1]: 100, m[2]: 0})
    sc("Affinity and Anti Affinity: considering both affinity and anti-affinity, the pod to schedule and existing "
       "pods have the same labels", 457, pod(S1, affinity=STAY_S1_AWAY_S2),
       [pod(S1, m[1]), pod(S1, m[1]), pod(S1, m[2]), pod(S1, m[3]), pod(S1, m[3]), pod(S1, m[4]), pod(S1, m[5])],
       [node(m[1], CHINA_AZ1), node(m[2], INDIA), node(m[3], CHINA), node(m[4], CHINA), node(m[5], INDIA)],
       {m[1]: 100, m[2]: 40, m[3]: 100, m[4]: 100, m[5]: 40})
    sc("Affinity and Anti Affinity and symmetry: considered only preferredDuringSchedulingIgnoredDuringExecution in "
       "both pod affinity & anti affinity & symmetry", 483, pod(S1, affinity=STAY_S1_AWAY_S2),
       [pod(S1, m[1]), pod(S2, m[2]), pod(None, m[3], STAY_S1_AWAY_S2), pod(None, m[4], AWAY_S1_AZ)],
       [node(m[1], CHINA), node(m[2], AZ1), node(m[3], INDIA), node(m[4], AZ2)],
       {m[1]: 100, m[2]: 0, m[3]: 100, m[4]: 0})
    sc("Avoid panic when partial nodes in a topology don't have pods with affinity", 503, pod(S1),
       [pod(S1, m[1]), pod(None, m[2], STAY_S1_AWAY_S2)], [node(m[1], CHINA), node(m[2], CHINA)],
       {m[1]: 100, m[2]: 100})
    # ---- TestPreferredAffinityWithHardPodAffinitySymmetricWeight
    hard = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        term([req("service", "In", ["S1"])], "region")]}}
    svc = {"service": "S1"}
    sc("Hard Pod Affinity symmetry: hard pod affinity symmetry weights 1 by default, then nodes that match the hard "
       "pod affinity symmetry rules, get a high score", 594, pod(svc),
       [pod(None, m[1], hard), pod(None, m[2], hard)], [node(m[1], CHINA), node(m[2], INDIA), node(m[3], AZ1)],
       {m[1]: 100, m[2]: 100, m[3]: 0}, hard_weight=1)
    sc("Hard Pod Affinity symmetry: hard pod affinity symmetry is closed(weights 0), then nodes that match the hard "
       "pod affinity symmetry rules, get same score with those not match", 609, pod(svc),
       [pod(None, m[1], hard), pod(None, m[2], hard)], [node(m[1], CHINA), node(m[2], INDIA), node(m[3], AZ1)],
       {m[1]: 0, m[2]: 0, m[3]: 0}, hard_weight=0)
    return out




def cpwat(ns, node_name, labels, aff, anti):
    """createPodWithAffinityTerms (filtering_test.go:34-53): both PodAffinity and PodAntiAffinity
    are non-nil, holding the given required terms."""
    a = {"podAffinity": {}, "podAntiAffinity": {}}
    if aff is not None:
        a["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"] = list(aff)
    if anti is not None:
        a["podAntiAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"] = list(anti)
    return pod(labels, node_name or None, a, ns=ns)


R_AFF = ["node(s) didn't match pod affinity/anti-affinity", "node(s) didn't match pod affinity rules"]
R_ANTI = ["node(s) didn't match pod affinity/anti-affinity", "node(s) didn't match pod anti-affinity rules"]
R_EXIST = ["node(s) didn't match pod affinity/anti-affinity", "node(s) didn't satisfy existing pods anti-affinity rules"]
U, UR = 2, 3


def single_node_cases():
    out = []
    SVC = {"service": "securityscan"}
    SEC = {"security": "S1"}
    n1 = node("machine1", {"region": "r1", "zone": "z11"})

    def fc(name, line, p, existing, code=0, reasons=()):
        out.append(case(name, FSRC + ":%d" % line, kind="filter", plugin="InterPodAffinity", args={}, pod=p,
                        pods=existing, nodes=[n1],
                        expect_filter={"machine1": {"code": code, "reasons": list(reasons)}}))

    in_ss = [req("service", "In", ["securityscan", "value2"])]
    in_av = [req("service", "In", ["antivirusscan", "value2"])]
    fc("A pod that has no required pod affinity scheduling rules can schedule onto a node with no existing pods", 71,
       pod(), [])
    fc("satisfies with requiredDuringSchedulingIgnoredDuringExecution in PodAffinity using In operator that matches "
       "the existing pod", 76, cpwat("", "", SEC, [term(in_ss, "region")], None), [pod(SVC, "machine1")])
    fc("satisfies the pod with requiredDuringSchedulingIgnoredDuringExecution in PodAffinity using not in operator "
       "in labelSelector that matches the existing pod", 96,
       cpwat("", "", SEC, [term([req("service", "NotIn", ["securityscan3", "value3"])], "region")], None),
       [pod(SVC, "machine1")])
    fc("Does not satisfy the PodAffinity with labelSelector because of diff Namespace", 116,
       cpwat("", "", SEC, [term(in_ss, "", ns=["DiffNameSpace"])], None), [pod(SVC, "machine1", ns="ns")], UR, R_AFF)
    fc("Doesn't satisfy the PodAffinity because of unmatching labelSelector with the existing pod", 141,
       cpwat("", "", SVC, [term(in_av, "")], None), [pod(SVC, "machine1")], UR, R_AFF)
    fc("satisfies the PodAffinity with different label Operators in multiple RequiredDuringSchedulingIgnoredDuring"
       "Execution ", 165,
       cpwat("", "", SEC, [term([req("service", "Exists"), req("wrongkey", "DoesNotExist")], "region"),
                           term([req("service", "In", ["securityscan"]), req("service", "NotIn", ["WrongValue"])],
                                "region")], None), [pod(SVC, "machine1")])
    fc("The labelSelector requirements(items of matchExpressions) are ANDed, the pod cannot schedule onto the node "
       "because one of the matchExpression item don't match.", 202,
       cpwat("", "", SEC, [term([req("service", "Exists"), req("wrongkey", "DoesNotExist")], "region"),
                           term([req("service", "In", ["securityscan2"]), req("service", "NotIn", ["WrongValue"])],
                                "region")], None), [pod(SVC, "machine1")], UR, R_AFF)
    fc("satisfies the PodAffinity and PodAntiAffinity with the existing pod", 244,
       cpwat("", "", SEC, [term(in_ss, "region")], [term(in_av, "node")]), [pod(SVC, "machine1")])
    fc("satisfies the PodAffinity and PodAntiAffinity and PodAntiAffinity symmetry with the existing pod", 278,
       cpwat("", "", SEC, [term(in_ss, "region")], [term(in_av, "node")]),
       [cpwat("", "machine1", SVC, None, [term(in_av, "node")])])
    fc("satisfies the PodAffinity but doesn't satisfy the PodAntiAffinity with the existing pod", 328,
       cpwat("", "", SEC, [term(in_ss, "region")], [term(in_ss, "zone")]), [pod(SVC, "machine1")], U, R_ANTI)
    fc("satisfies the PodAffinity and PodAntiAffinity but doesn't satisfy PodAntiAffinity symmetry with the existing "
       "pod", 367, cpwat("", "", SVC, [term(in_ss, "region")], [term(in_av, "node")]),
       [cpwat("", "machine1", SVC, None, [term(in_ss, "zone")])], U, R_EXIST)
    fc("pod matches its own Label in PodAffinity and that matches the existing pod Labels", 422,
       cpwat("", "", SVC, [term([req("service", "NotIn", ["securityscan", "value2"])], "region")], None),
       [pod(SVC, "machine2")], UR, R_AFF)
    fc("verify that PodAntiAffinity from existing pod is respected when pod has no AntiAffinity constraints. doesn't "
       "satisfy PodAntiAffinity symmetry with the existing pod", 447, pod(SVC),
       [cpwat("", "machine1", SVC, None, [term(in_ss, "zone")])], U, R_EXIST)
    fc("verify that PodAntiAffinity from existing pod is respected when pod has no AntiAffinity constraints. satisfy "
       "PodAntiAffinity symmetry with the existing pod", 478, pod(SVC),
       [cpwat("", "machine1", SVC, None, [term([req("service", "NotIn", ["securityscan", "value2"])], "zone")])])
    fc("satisfies the PodAntiAffinity with existing pod but doesn't satisfy PodAntiAffinity symmetry with incoming "
       "pod", 504, cpwat("", "", SVC, None, [term([req("service", "Exists")], "region"),
                                             term([req("security", "Exists")], "region")]),
       [cpwat("", "machine1", SEC, None, [term([req("security", "Exists")], "zone")])], U, R_ANTI)
    fc("PodAntiAffinity symmetry check a1: incoming pod and existing pod partially match each other on AffinityTerms",
       554, cpwat("", "", SVC, None, [term([req("service", "Exists")], "zone"),
                                      term([req("security", "Exists")], "zone")]),
       [cpwat("", "machine1", SEC, None, [term([req("security", "Exists")], "zone")])], U, R_ANTI)
    fc("PodAntiAffinity symmetry check a2: incoming pod and existing pod partially match each other on AffinityTerms",
       604, cpwat("", "", SEC, None, [term([req("security", "Exists")], "zone")]),
       [cpwat("", "machine1", SVC, None, [term([req("service", "Exists")], "zone"),
                                           term([req("security", "Exists")], "zone")])], U, R_EXIST)
    ab = [term([req("abc", "Exists")], "zone"), term([req("def", "Exists")], "zone")]
    fc("PodAntiAffinity symmetry check b1: incoming pod and existing pod partially match each other on AffinityTerms",
       654, cpwat("", "", {"abc": "", "xyz": ""}, None, ab),
       [cpwat("", "machine1", {"def": "", "xyz": ""}, None, ab)], U, R_ANTI)
    fc("PodAntiAffinity symmetry check b2: incoming pod and existing pod partially match each other on AffinityTerms",
       715, cpwat("", "", {"def": "", "xyz": ""}, None, ab),
       [cpwat("", "machine1", {"abc": "", "xyz": ""}, None, ab)], U, R_ANTI)
    return out


def multi_node_cases():
    """TestRequiredAffinityMultipleNodes (filtering_test.go:797-1683): every node of the table is
    filtered, and each has its own expected status."""
    out = []
    CN, CN_AZ1, IN = {"region": "China"}, {"region": "China", "az": "az1"}, {"region": "India"}

    def nd(name, **labels):
        return node(name, labels)

    def rzh(name, zone):
        return nd(name, region="r1", zone=zone, hostname=name)

    def fc(name, line, p, existing, nodes, want):
        exp = {}
        for n, w in zip(nodes, want):
            exp[n["metadata"]["name"]] = {"code": 0, "reasons": []} if w is None else {"code": w[0], "reasons": list(w[1])}
        out.append(case(name, FSRC + ":%d" % line, kind="filter", plugin="InterPodAffinity", args={}, pod=p,
                        pods=existing, nodes=nodes, expect_filter=exp))

    ex = lambda k: req(k, "Exists")
    aff_fail, anti_fail, exist_fail = (UR, R_AFF), (U, R_ANTI), (U, R_EXIST)
    fc("A pod can be scheduled onto all the nodes that have the same topology key & label value with one of them has "
       "an existing pod that matches the affinity rules", 852,
       cpwat("", "", None, [term([req("foo", "In", ["bar"])], "region")], None),
       [pod({"foo": "bar"}, "machine1", name="p1")],
       [node("machine1", CN), node("machine2", CN_AZ1), node("machine3", IN)], [None, None, aff_fail])
    two_zone = [term([req("foo", "In", ["bar"])], "zone"), term([req("service", "In", ["securityscan"])], "zone")]
    fc("The affinity rule is to schedule all of the pods of this collection to the same zone. The first pod of the "
       "collection should not be blocked from being scheduled onto any node, even there's no existing pod that "
       "matches the rule anywhere.", 888, cpwat("", "", {"foo": "bar", "service": "securityscan"}, two_zone, None),
       [pod({"foo": "bar"}, "nodeA", name="p1")],
       [nd("nodeA", zone="az1", hostname="h1"), nd("nodeB", zone="az2", hostname="h2")], [None, None])
    fc("The first pod of the collection can only be scheduled on nodes labelled with the requested topology keys", 936,
       cpwat("", "", {"foo": "bar", "service": "securityscan"}, two_zone, None),
       [pod({"foo": "bar"}, "nodeA", name="p1")],
       [nd("nodeA", zoneLabel="az1", hostname="h1"), nd("nodeB", zoneLabel="az2", hostname="h2")],
       [aff_fail, aff_fail])
    abc_region = [term([req("foo", "In", ["abc"])], "region")]
    fc("NodeA and nodeB have same topologyKey and label value. NodeA has an existing pod that matches the inter pod "
       "affinity rule. The pod can not be scheduled onto nodeA and nodeB.", 973,
       cpwat("", "", None, None, abc_region), [pod({"foo": "abc"}, "nodeA")],
       [nd("nodeA", region="r1", hostname="nodeA"), nd("nodeB", region="r1", hostname="nodeB")],
       [anti_fail, anti_fail])
    fc("This test ensures that anti-affinity matches a pod when any term of the anti-affinity rule matches a pod.",
       1022, cpwat("", "", None, None, [term([req("foo", "In", ["abc"])], "region"),
                                        term([req("service", "In", ["securityscan"])], "zone")]),
       [pod({"foo": "abc", "service": "securityscan"}, "nodeA")], [rzh("nodeA", "z1"), rzh("nodeB", "z2")],
       [anti_fail, anti_fail])
    fc("NodeA and nodeB have same topologyKey and label value. NodeA has an existing pod that matches the inter pod "
       "affinity rule. The pod can not be scheduled onto nodeA and nodeB but can be scheduled onto nodeC", 1061,
       cpwat("", "", None, None, abc_region), [pod({"foo": "abc"}, "nodeA")],
       [node("nodeA", CN), node("nodeB", CN_AZ1), node("nodeC", IN)], [anti_fail, anti_fail, None])
    fc("NodeA and nodeB have same topologyKey and label value. NodeA has an existing pod that matches the inter pod "
       "affinity rule. The pod can not be scheduled onto nodeA, nodeB, but can be scheduled onto nodeC (NodeC has an "
       "existing pod that match the inter pod affinity rule but in different namespace)", 1121,
       cpwat("NS1", "", {"foo": "123"}, None, [term([req("foo", "In", ["bar"])], "region")]),
       [pod({"foo": "bar"}, "nodeA", ns="NS1"),
        cpwat("NS2", "nodeC", None, None, [term([req("foo", "In", ["123"])], "region")])],
       [node("nodeA", CN), node("nodeB", CN_AZ1), node("nodeC", IN)], [anti_fail, anti_fail, None])
    z1 = [rzh("nodeA", "z1"), rzh("nodeB", "z1")]
    z12 = [rzh("nodeA", "z1"), rzh("nodeB", "z2")]
    fc("Test existing pod's anti-affinity: if an existing pod has a term with invalid topologyKey, labelSelector of "
       "the term is firstly checked, and then topologyKey of the term is also checked", 1148,
       pod({"foo": ""}), [cpwat("", "nodeA", None, None, [term([ex("foo")], "invalid-node-label")])], z1,
       [None, None])
    fc("Test incoming pod's anti-affinity: even if labelSelector matches, we still check if topologyKey matches", 1178,
       cpwat("", "", None, None, [term([ex("foo")], "invalid-node-label")]), [pod({"foo": ""}, "nodeA")], z1,
       [None, None])
    fc("Test existing pod's anti-affinity: incoming pod wouldn't considered as a fit as it violates each existingPod's "
       "terms on all nodes", 1230, pod({"foo": "", "bar": ""}),
       [cpwat("", "nodeA", None, None, [term([ex("foo")], "zone")]),
        cpwat("", "nodeA", None, None, [term([ex("bar")], "region")])], z12, [exist_fail, exist_fail])
    fc("Test incoming pod's anti-affinity: incoming pod wouldn't considered as a fit as it at least violates one "
       "anti-affinity rule of existingPod", 1288,
       cpwat("", "", None, None, [term([ex("foo")], "zone"), term([ex("bar")], "region")]),
       [pod({"foo": ""}, "nodeA"), pod({"bar": ""}, "nodeB")], z12, [anti_fail, anti_fail])
    fc("Test existing pod's anti-affinity: only when labelSelector and topologyKey both match, it's counted as a "
       "single term match - case when one term has invalid topologyKey", 1333, pod({"foo": "", "bar": ""}),
       [cpwat("", "nodeA", None, None, [term([ex("foo")], "invalid-node-label"), term([ex("bar")], "zone")])], z12,
       [exist_fail, None])
    fc("Test incoming pod's anti-affinity: only when labelSelector and topologyKey both match, it's counted as a "
       "single term match - case when one term has invalid topologyKey", 1381,
       cpwat("", "", None, None, [term([ex("foo")], "invalid-node-label"), term([ex("bar")], "zone")]),
       [pod({"foo": "", "bar": ""}, "nodeA", name="podA")], z12, [anti_fail, None])
    fc("Test existing pod's anti-affinity: only when labelSelector and topologyKey both match, it's counted as a "
       "single term match - case when all terms have valid topologyKey", 1430, pod({"foo": "", "bar": ""}),
       [cpwat("", "nodeA", None, None, [term([ex("foo")], "region"), term([ex("bar")], "zone")])], z12,
       [exist_fail, exist_fail])
    fc("Test incoming pod's anti-affinity: only when labelSelector and topologyKey both match, it's counted as a "
       "single term match - case when all terms have valid topologyKey", 1482,
       cpwat("", "", None, None, [term([ex("foo")], "region"), term([ex("bar")], "zone")]),
       [pod({"foo": "", "bar": ""}, "nodeA")], z12, [anti_fail, anti_fail])
    fc("Test existing pod's anti-affinity: existingPod on nodeA and nodeB has at least one anti-affinity term matches "
       "incoming pod, so incoming pod can only be scheduled to nodeC", 1558, pod({"foo": "", "bar": ""}),
       [cpwat("", "nodeA", None, None, [term([ex("foo")], "zone"), term([ex("labelA")], "zone")]),
        cpwat("", "nodeB", None, None, [term([ex("bar")], "zone"), term([ex("labelB")], "zone")])],
       [rzh("nodeA", "z1"), rzh("nodeB", "z2"), rzh("nodeC", "z3")], [exist_fail, exist_fail, None])
    fc("Test incoming pod's affinity: firstly check if all affinityTerms match, and then check if all topologyKeys "
       "match", 1599, cpwat("", "", None, [term([ex("foo")], "region"), term([ex("bar")], "zone")], None),
       [pod({"foo": "", "bar": ""}, "nodeA", name="pod1")], z1, [None, None])
    fc("Test incoming pod's affinity: firstly check if all affinityTerms match, and then check if all topologyKeys "
       "match, and the match logic should be satisfied on the same pod", 1657,
       cpwat("", "", None, [term([ex("foo")], "region"), term([ex("bar")], "zone")], None),
       [pod({"foo": ""}, "nodeA", name="pod1"), pod({"bar": ""}, "nodeB", name="pod2")], z12,
       [aff_fail, aff_fail])
    return out


def state_cases():
    out = []

    def sc(name, line, p, existing, nodes, aff, anti, added=None, services=()):
        kw = {}
        if added is not None:
            kw.update(op="add_remove", op_pod=added, op_node=added["spec"]["nodeName"])
        else:
            kw.update(op="prefilter")
        out.append(case(name, FSRC + ":%d" % line, kind="ipa_state", plugin="InterPodAffinity", args={}, pod=p,
                        pods=existing, nodes=nodes, services=list(services),
                        expect_ipa={"aff": sorted([list(x) for x in aff]), "anti": sorted([list(x) for x in anti])},
                        **kw))

    # ---- TestPreFilterStateAddRemovePod (filtering_test.go:1697)
    l1, l2, l3 = {"region": "r1", "zone": "z11"}, {"region": "r1", "zone": "z12"}, {"region": "r2", "zone": "z21"}
    sel1 = {"foo": "bar"}
    anti_foobar = {"requiredDuringSchedulingIgnoredDuringExecution": [term([req("foo", "In", ["bar"])], "region")]}
    complex_terms = [term([req("foo", "In", ["bar", "buzz"])], "region"),
                     term([req("service", "NotIn", ["bar", "security", "test"])], "zone")]
    anti_complex = {"requiredDuringSchedulingIgnoredDuringExecution": complex_terms}
    aff_complex = {"requiredDuringSchedulingIgnoredDuringExecution": [dict(t) for t in complex_terms]}
    abc = lambda: [node("nodeA", l1), node("nodeB", l2), node("nodeC", l3)]  # noqa: E731
    svc = [{"spec": {"selector": dict(sel1)}}]
    sc("no affinity exist", 1795, pod(sel1, name="pending"),
       [pod(sel1, "nodeA", name="p1"), pod(None, "nodeC", name="p2")], abc(), [], [],
       added=pod(sel1, "nodeB", name="addedPod"))
    sc("preFilterState anti-affinity terms are updated correctly after adding and removing a pod", 1820,
       pod(sel1, name="pending", affinity={"podAntiAffinity": anti_foobar}),
       [pod(sel1, "nodeA", name="p1"), pod(None, "nodeC", name="p2", affinity={"podAntiAffinity": anti_foobar})],
       abc(), [], [("region", "r1", 2)],
       added=pod(sel1, "nodeB", name="addedPod", affinity={"podAntiAffinity": anti_foobar}))
    sc("preFilterState anti-affinity terms are updated correctly after adding and removing a pod", 1862,
       pod(sel1, name="pending", affinity={"podAntiAffinity": anti_complex}),
       [pod(sel1, "nodeA", name="p1"), pod(None, "nodeC", name="p2", affinity={"podAntiAffinity": anti_foobar})],
       abc(), [], [("region", "r1", 2), ("zone", "z11", 2), ("zone", "z21", 1)],
       added=pod(sel1, "nodeA", name="addedPod", affinity={"podAntiAffinity": anti_complex}), services=svc)
    sc("preFilterState matching pod affinity and anti-affinity are updated correctly after adding and removing a pod",
       1907, pod(sel1, name="pending", affinity={"podAffinity": aff_complex}),
       [pod(sel1, "nodeA", name="p1"),
        pod(None, "nodeC", name="p2", affinity={"podAntiAffinity": anti_foobar, "podAffinity": aff_complex})],
       abc(), [("region", "r1", 2), ("zone", "z11", 2)], [],
       added=pod(sel1, "nodeA", name="addedPod", affinity={"podAntiAffinity": anti_complex}), services=svc)

    # ---- TestGetTPMapMatchingIncomingAffinityAntiAffinity (filtering_test.go:2045)
    def terms(*keys):
        return [term([req(k, "Exists")], "hostname") for k in keys]

    def normal(*labels):
        return pod({lb: "" for lb in labels}, "nodeA", name="normal")

    node_a = lambda: [node("nodeA", {"hostname": "nodeA"})]  # noqa: E731

    def both(aff_keys, anti_keys, name):
        return pod(None, name=name, affinity={"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": terms(*aff_keys)},
                                              "podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": terms(*anti_keys)}})

    hn = ("hostname", "nodeA")
    sc("nil test", 2087, pod(None, name="aaa-normal"), [], node_a(), [], [])
    sc("incoming pod without affinity/anti-affinity causes a no-op", 2096, pod(None, name="aaa-normal"),
       [normal("aaa")], node_a(), [], [])
    sc("no pod has label that violates incoming pod's affinity and anti-affinity", 2106,
       both(["aaa"], ["aaa"], "aaa-anti"), [normal("bbb")], node_a(), [], [])
    sc("existing pod matches incoming pod's affinity and anti-affinity - single term case", 2126,
       both(["aaa"], ["aaa"], "affi-antiaffi"), [normal("aaa")], node_a(), [hn + (1,)], [hn + (1,)])
    sc("existing pod matches incoming pod's affinity and anti-affinity - multiple terms case", 2150,
       both(["aaa", "bbb"], ["aaa"], "affi-antiaffi"), [normal("aaa", "bbb")], node_a(), [hn + (2,)], [hn + (1,)])
    sc("existing pod not match incoming pod's affinity but matches anti-affinity", 2174,
       both(["aaa", "bbb"], ["aaa", "bbb"], "affi-antiaffi"), [normal("aaa")], node_a(), [], [hn + (1,)])
    sc("incoming pod's anti-affinity has more than one term - existing pod violates partial term - case 1", 2196,
       both(["aaa", "ccc"], ["aaa", "ccc"], "anaffi-antiaffiti"), [normal("aaa", "bbb")], node_a(), [], [hn + (1,)])
    sc("incoming pod's anti-affinity has more than one term - existing pod violates partial term - case 2", 2218,
       both(["aaa", "bbb"], ["aaa", "bbb"], "affi-antiaffi"), [normal("bbb")], node_a(), [], [hn + (1,)])
    return out


def all_cases():
    return score_cases() + single_node_cases() + multi_node_cases() + state_cases()

"""Golden vectors transcribed from pkg/scheduler/framework/plugins/nodeaffinity/node_affinity_test.go."""
from gen_common import case, node, pod

SRC = "pkg/scheduler/framework/plugins/nodeaffinity/node_affinity_test.go"
U = 3  # UnschedulableAndUnresolvable
ERR = "node(s) didn't match node selector"


def req(key, op, values=None):
    r = {"key": key, "operator": op}
    if values is not None:
        r["values"] = list(values)
    return r


def required(*terms, nil_terms=False):
    sel = {} if nil_terms else {"nodeSelectorTerms": list(terms)}
    return {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": sel}}


def term(exprs=None, fields=None):
    t = {}
    if exprs is not None:
        t["matchExpressions"] = exprs
    if fields is not None:
        t["matchFields"] = fields
    return t


def filter_cases():
    out = []

    def fc(name, line, p, labels=None, node_name="", fail=False):
        out.append(case(name, SRC + ":%d" % line, kind="filter", plugin="NodeAffinity", args={}, pod=p, pods=[],
                        nodes=[node(node_name, {}, labels=labels)],
                        expect_filter={node_name: {"code": U if fail else 0, "reasons": [ERR] if fail else []}}))

    fc("no selector", 42, pod())
    fc("missing labels", 52, pod(nodeSelector={"foo": "bar"}), fail=True)
    fc("same labels", 66, pod(nodeSelector={"foo": "bar"}), {"foo": "bar"})
    fc("node labels are superset", 80, pod(nodeSelector={"foo": "bar"}), {"foo": "bar", "baz": "blah"})
    fc("node labels are subset", 94, pod(nodeSelector={"foo": "bar", "baz": "blah"}), {"foo": "bar"}, fail=True)
    fc("Pod with matchExpressions using In operator that matches the existing node", 122,
       pod(affinity=required(term([req("foo", "In", ["bar", "value2"])]))), {"foo": "bar"})
    fc("Pod with matchExpressions using Gt operator that matches the existing node", 150,
       pod(affinity=required(term([req("kernel-version", "Gt", ["0204"])]))), {"kernel-version": "0206"})
    fc("Pod with matchExpressions using NotIn operator that matches the existing node", 177,
       pod(affinity=required(term([req("mem-type", "NotIn", ["DDR", "DDR2"])]))), {"mem-type": "DDR3"})
    fc("Pod with matchExpressions using Exists operator that matches the existing node", 203,
       pod(affinity=required(term([req("GPU", "Exists")]))), {"GPU": "NVIDIA-GRID-K1"})
    fc("Pod with affinity that don't match node's labels won't schedule onto the node", 230,
       pod(affinity=required(term([req("foo", "In", ["value1", "value2"])]))), {"foo": "bar"}, fail=True)
    fc("Pod with a nil []NodeSelectorTerm in affinity, can't match the node's labels and won't schedule onto "
       "the node", 248, pod(affinity=required(nil_terms=True)), {"foo": "bar"}, fail=True)
    fc("Pod with an empty []NodeSelectorTerm in affinity, can't match the node's labels and won't schedule "
       "onto the node", 266, pod(affinity=required()), {"foo": "bar"}, fail=True)
    fc("Pod with empty MatchExpressions is not a valid value will match no objects and won't schedule onto "
       "the node", 288, pod(affinity=required(term([]))), {"foo": "bar"}, fail=True)
    fc("Pod with no Affinity will schedule onto a node", 296, pod(), {"foo": "bar"})
    fc("Pod with Affinity but nil NodeSelector will schedule onto a node", 311,
       pod(affinity={"nodeAffinity": {}}), {"foo": "bar"})
    fc("Pod with multiple matchExpressions ANDed that matches the existing node", 341,
       pod(affinity=required(term([req("GPU", "Exists"), req("GPU", "NotIn", ["AMD", "INTER"])]))),
       {"GPU": "NVIDIA-GRID-K1"})
    fc("Pod with multiple matchExpressions ANDed that doesn't match the existing node", 371,
       pod(affinity=required(term([req("GPU", "Exists"), req("GPU", "In", ["AMD", "INTER"])]))),
       {"GPU": "NVIDIA-GRID-K1"}, fail=True)
    fc("Pod with multiple NodeSelectorTerms ORed in affinity, matches the node's labels and will schedule onto "
       "the node", 408, pod(affinity=required(term([req("foo", "In", ["bar", "value2"])]),
                                              term([req("diffkey", "In", ["wrong", "value2"])]))), {"foo": "bar"})
    fc("Pod with an Affinity and a PodSpec.NodeSelector(the old thing that we are deprecating) both are "
       "satisfied, will schedule onto the node", 437,
       pod(nodeSelector={"foo": "bar"}, affinity=required(term([req("foo", "Exists")]))), {"foo": "bar"})
    fc("Pod with an Affinity matches node's labels but the PodSpec.NodeSelector(the old thing that we are "
       "deprecating) is not satisfied, won't schedule onto the node", 467,
       pod(nodeSelector={"foo": "bar"}, affinity=required(term([req("foo", "Exists")]))), {"foo": "barrrrrr"},
       fail=True)
    fc("Pod with an invalid value in Affinity term won't be scheduled onto the node", 496,
       pod(affinity=required(term([req("foo", "NotIn", ["invalid value: ___@#$%^"])]))), {"foo": "bar"}, fail=True)
    mf1 = [req("metadata.name", "In", ["node_1"])]
    fc("Pod with matchFields using In operator that matches the existing node", 522,
       pod(affinity=required(term(fields=mf1))), node_name="node_1")
    fc("Pod with matchFields using In operator that does not match the existing node", 547,
       pod(affinity=required(term(fields=mf1))), node_name="node_2", fail=True)
    fc("Pod with two terms: matchFields does not match, but matchExpressions matches", 583,
       pod(affinity=required(term(fields=mf1), term([req("foo", "In", ["bar"])]))), {"foo": "bar"}, "node_2")
    fc("Pod with one term: matchFields does not match, but matchExpressions matches", 616,
       pod(affinity=required(term([req("foo", "In", ["bar"])], mf1))), {"foo": "bar"}, "node_2", fail=True)
    fc("Pod with one term: both matchFields and matchExpressions match", 650,
       pod(affinity=required(term([req("foo", "In", ["bar"])], mf1))), {"foo": "bar"}, "node_1")
    fc("Pod with two terms: both matchFields and matchExpressions do not match", 685,
       pod(affinity=required(term(fields=mf1), term([req("foo", "In", ["not-match-to-bar"])]))), {"foo": "bar"},
       "node_2", fail=True)
    return out


def preferred(*terms):
    return {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": w, "preference": {"matchExpressions": exprs}} for w, exprs in terms]}}


def score_cases():
    l1, l2, l3 = {"foo": "bar"}, {"key": "value"}, {"az": "az1"}
    l4 = {"abc": "az11", "def": "az22"}
    l5 = {"foo": "bar", "key": "value", "az": "az1"}
    a1 = preferred((2, [req("foo", "In", ["bar"])]))
    a2 = preferred((2, [req("foo", "In", ["bar"])]), (4, [req("key", "In", ["value"])]),
                   (5, [req("foo", "In", ["bar"]), req("key", "In", ["value"]), req("az", "In", ["az1"])]))
    out = []

    def sc(name, line, p, nodes, exp):
        out.append(case(name, SRC + ":%d" % line, kind="score", plugin="NodeAffinity", args={}, pod=p, pods=[],
                        nodes=[node(n, {}, labels=lab) for n, lab in nodes], normalize=True, expect_scores=exp))

    sc("all machines are same priority as NodeAffinity is nil", 801, pod(),
       [("machine1", l1), ("machine2", l2), ("machine3", l3)], {"machine1": 0, "machine2": 0, "machine3": 0})
    sc("no machine macthes preferred scheduling requirements in NodeAffinity of pod so all machines' priority "
       "is zero", 815, pod(affinity=a1), [("machine1", l4), ("machine2", l2), ("machine3", l3)],
       {"machine1": 0, "machine2": 0, "machine3": 0})
    sc("only machine1 matches the preferred scheduling requirements of pod", 829, pod(affinity=a1),
       [("machine1", l1), ("machine2", l2), ("machine3", l3)], {"machine1": 100, "machine2": 0, "machine3": 0})
    sc("all machines matches the preferred scheduling requirements of pod but with different priorities ", 843,
       pod(affinity=a2), [("machine1", l1), ("machine5", l5), ("machine2", l2)],
       {"machine1": 18, "machine5": 100, "machine2": 36})
    return out


def all_cases():
    return filter_cases() + score_cases()

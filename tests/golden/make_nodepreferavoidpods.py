"""Golden vectors transcribed from
pkg/scheduler/framework/plugins/nodepreferavoidpods/node_prefer_avoid_pods_test.go (TestNodePreferAvoidPods).

The node annotation is kept as the JSON text the reference's test sets under
scheduler.alpha.kubernetes.io/preferAvoidPods."""
import json

from gen_common import case, node, pod

SRC = "pkg/scheduler/framework/plugins/nodepreferavoidpods/node_prefer_avoid_pods_test.go"
KEY = "scheduler.alpha.kubernetes.io/preferAvoidPods"


def avoid_annotation(kind, uid):
    doc = {"preferAvoidPods": [{"podSignature": {"podController": {
        "apiVersion": "v1", "kind": kind, "name": "foo", "uid": uid, "controller": True}},
        "reason": "some reason", "message": "some message"}]}
    return {KEY: json.dumps(doc, indent=4)}


def owned(kind, uid, controller):
    ref = {"kind": kind, "name": "foo", "uid": uid}
    if controller is not None:
        ref["controller"] = controller
    p = pod(ns="default")
    p["metadata"]["ownerReferences"] = [ref]
    return p


def all_cases():
    nodes = [node("machine1", {}, annotations=avoid_annotation("ReplicationController", "abcdef123456")),
             node("machine2", {}, annotations=avoid_annotation("ReplicaSet", "qwert12345")),
             node("machine3", {})]
    rows = [
        ("pod managed by ReplicationController should avoid a node, this node get lowest priority score", 102,
         owned("ReplicationController", "abcdef123456", True), [0, 100, 100]),
        ("ownership by random controller should be ignored", 115,
         owned("RandomController", "abcdef123456", True), [100, 100, 100]),
        ("owner without Controller field set should be ignored", 128,
         owned("ReplicationController", "abcdef123456", None), [100, 100, 100]),
        ("pod managed by ReplicaSet should avoid a node, this node get lowest priority score", 141,
         owned("ReplicaSet", "qwert12345", True), [100, 0, 100]),
    ]
    return [case(n, SRC + ":%d" % line, kind="score", plugin="NodePreferAvoidPods", args={}, pod=p, pods=[],
                 nodes=nodes, expect_scores={"machine%d" % (i + 1): s for i, s in enumerate(exp)})
            for n, line, p, exp in rows]

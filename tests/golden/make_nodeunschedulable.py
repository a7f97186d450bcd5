"""Golden vectors transcribed from
pkg/scheduler/framework/plugins/nodeunschedulable/node_unschedulable_test.go (TestNodeUnschedulable)."""
from gen_common import case, node, pod

SRC = "pkg/scheduler/framework/plugins/nodeunschedulable/node_unschedulable_test.go"
U = 3  # UnschedulableAndUnresolvable
ERR = "node(s) were unschedulable"


def all_cases():
    tol = [{"key": "node.kubernetes.io/unschedulable", "effect": "NoSchedule"}]
    rows = [("Does not schedule pod to unschedulable node (node.Spec.Unschedulable==true)", 36, pod(), True, True),
            ("Schedule pod to normal node", 45, pod(), False, False),
            ("Schedule pod with toleration to unschedulable node (node.Spec.Unschedulable==true)", 54,
             pod(tolerations=tol), True, False)]
    return [case(n, SRC + ":%d" % line, kind="filter", plugin="NodeUnschedulable", args={}, pod=p, pods=[],
                 nodes=[node("", {}, unschedulable=u)],
                 expect_filter={"": {"code": U if fail else 0, "reasons": [ERR] if fail else []}})
            for n, line, p, u, fail in rows]

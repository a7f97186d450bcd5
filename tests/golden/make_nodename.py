"""Golden vectors transcribed from pkg/scheduler/framework/plugins/nodename/node_name_test.go (TestNodeName)."""
from gen_common import case, node, pod

SRC = "pkg/scheduler/framework/plugins/nodename/node_name_test.go"
U = 3  # UnschedulableAndUnresolvable
ERR = "node(s) didn't match the requested hostname"


def all_cases():
    rows = [("no host specified", 39, pod(), "", False),
            ("host matches", 52, pod(node_name="foo"), "foo", False),
            ("host doesn't match", 64, pod(node_name="bar"), "foo", True)]
    return [case(n, SRC + ":%d" % line, kind="filter", plugin="NodeName", args={}, pod=p, pods=[],
                 nodes=[node(nn, {})],
                 expect_filter={nn: {"code": U if fail else 0, "reasons": [ERR] if fail else []}})
            for n, line, p, nn, fail in rows]

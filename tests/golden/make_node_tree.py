"""Golden vectors transcribed from pkg/scheduler/internal/cache/node_tree_test.go (TestNodeTree_Next).

Snapshot.List() order is the first numNodes outputs of nodeTree.next() (cache.go:278-301)."""
from gen_common import case, node

SRC = "pkg/scheduler/internal/cache/node_tree_test.go"
RG, ZN = "failure-domain.beta.kubernetes.io/region", "failure-domain.beta.kubernetes.io/zone"
RGS, ZNS = "topology.kubernetes.io/region", "topology.kubernetes.io/zone"

ALL = [  # node_tree_test.go:27-137 allNodes
    node("node-0", {}),
    node("node-1", {}, labels={RG: "region-1"}),
    node("node-2", {}, labels={ZN: "zone-2"}),
    node("node-3", {}, labels={RG: "region-1", ZN: "zone-2"}),
    node("node-4", {}, labels={RG: "region-1", ZN: "zone-2"}),
    node("node-5", {}, labels={RG: "region-1", ZN: "zone-3"}),
    node("node-6", {}, labels={RG: "region-2", ZN: "zone-2"}),
    node("node-7", {}, labels={RG: "region-2", ZN: "zone-2"}),
    node("node-8", {}, labels={RG: "region-2", ZN: "zone-2"}),
    node("node-9", {}, labels={RGS: "region-2", ZNS: "zone-2", RG: "region-2", ZN: "zone-2"}),
    node("node-10", {}, labels={RG: "region-2", ZN: "zone-3"}),
]


def all_cases():
    return [
        case("should go back to the first node after finishing a round", SRC + ":366", kind="node_tree",
             nodes=ALL[:1], expect_order=["node-0"]),
        case("should go back to the first node after going over all nodes", SRC + ":372", kind="node_tree",
             nodes=ALL[:4], expect_order=["node-0", "node-1", "node-2", "node-3"]),
        case("should go to all zones before going to the second nodes in the same zone", SRC + ":378",
             kind="node_tree", nodes=ALL[:9],
             expect_order=["node-0", "node-1", "node-2", "node-3", "node-5", "node-6", "node-4", "node-7", "node-8"]),
    ]

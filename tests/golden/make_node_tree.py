"""Golden vectors transcribed from pkg/scheduler/internal/cache/node_tree_test.go (TestNodeTree_AddNode,
_RemoveNode, _UpdateNode, _Next, TestNodeTreeMultiOperations).

Snapshot.List() order is numNodes outputs of nodeTree.next() (cache.go:278-301).  "node_tree"
cases hold a fresh tree's first pass; "node_tree_ops" cases replay add/remove/update/next
operations and compare the next() outputs, the zone arrays and the remove errors."""
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


def ops_cases():
    out = []

    def oc(name, line, initial, ops, output=None, tree=None, remove_errors=None):
        kw = {}
        if output is not None:
            kw["expect_output"] = output
        if tree is not None:
            kw["expect_tree"] = tree
        if remove_errors is not None:
            kw["expect_remove_errors"] = remove_errors
        out.append(case(name, SRC + ":%d" % line, kind="node_tree_ops", initial=list(initial), ops=ops, **kw))

    add = lambda ns: [["add", n] for n in ns]  # noqa
    rm = lambda ns: [["remove", n] for n in ns]  # noqa
    R1, Z2, R1Z2 = "region-1:\x00:", ":\x00:zone-2", "region-1:\x00:zone-2"
    R1Z3, R2Z2, R2Z3 = "region-1:\x00:zone-3", "region-2:\x00:zone-2", "region-2:\x00:zone-3"
    # ---- TestNodeTree_AddNode (:157)
    oc("single node no labels", 164, [], add(ALL[:1]), tree={"": ["node-0"]})
    oc("mix of nodes with and without proper labels", 169, [], add(ALL[:4]),
       tree={"": ["node-0"], R1: ["node-1"], Z2: ["node-2"], R1Z2: ["node-3"]})
    seven = {"": ["node-0"], R1: ["node-1"], Z2: ["node-2"], R1Z2: ["node-3", "node-4"], R1Z3: ["node-5"],
             R2Z2: ["node-6"]}
    oc("mix of nodes with and without proper labels and some zones with multiple nodes", 179, [], add(ALL[:7]),
       tree=seven)
    oc("nodes also using deprecated zone/region label", 191, [], add(ALL[9:]),
       tree={R2Z2: ["node-9"], R2Z3: ["node-10"]})
    # ---- TestNodeTree_RemoveNode (:211)
    oc("remove a single node with no labels", 220, ALL[:7], rm(ALL[:1]),
       tree={k: v for k, v in seven.items() if k != ""}, remove_errors=[False])
    oc("remove a few nodes including one from a zone with multiple nodes", 232, ALL[:7], rm(ALL[1:4]),
       tree={"": ["node-0"], R1Z2: ["node-4"], R1Z3: ["node-5"], R2Z2: ["node-6"]}, remove_errors=[False] * 3)
    oc("remove all nodes", 243, ALL[:7], rm(ALL[:7]), tree={}, remove_errors=[False] * 7)
    oc("remove non-existing node", 249, [], rm(ALL[:5]), tree={}, remove_errors=[True] * 5)
    # ---- TestNodeTree_UpdateNode (:271): the old object is allNodes' entry of the same name, else a
    # label-less "nonexisting-node"
    moved = node("node-0", {}, labels={RG: "region-1", ZN: "zone-2"})
    oc("update a node without label", 279, ALL[:7], [["update", ALL[0], moved]],
       tree={R1: ["node-1"], Z2: ["node-2"], R1Z2: ["node-3", "node-4", "node-0"], R1Z3: ["node-5"],
             R2Z2: ["node-6"]})
    oc("update the only existing node", 299, ALL[:1], [["update", ALL[0], moved]], tree={R1Z2: ["node-0"]})
    oc("update non-existing node", 315, ALL[:1],
       [["update", node("nonexisting-node", {}), node("node-new", {}, labels={RG: "region-1", ZN: "zone-2"})]],
       tree={"": ["node-0"], R1Z2: ["node-new"]})
    # ---- TestNodeTree_Next (:352)
    nx = lambda k: [["next"]] * k  # noqa
    oc("empty tree", 360, [], nx(2), output=["", ""])
    oc("should go back to the first node after finishing a round", 366, ALL[:1], nx(2), output=["node-0", "node-0"])
    oc("should go back to the first node after going over all nodes", 372, ALL[:4], nx(5),
       output=["node-0", "node-1", "node-2", "node-3", "node-0"])
    oc("should go to all zones before going to the second nodes in the same zone", 378, ALL[:9], nx(11),
       output=["node-0", "node-1", "node-2", "node-3", "node-5", "node-6", "node-4", "node-7", "node-8", "node-0",
               "node-1"])

    # ---- TestNodeTreeMultiOperations (:400)
    def multi(name, line, to_add, to_remove, ops, output):
        seq, ai, ri = [], 0, 0
        for o in ops:
            if o == "add":
                seq.append(["add", to_add[ai]])
                ai += 1
            elif o == "remove":
                seq.append(["remove", to_remove[ri]])
                ri += 1
            else:
                seq.append(["next"])
        oc(name, line, [], seq, output=output)

    # The table is built with append() on sub-slices of allNodes, which share its backing array:
    # append(allNodes[4:9], allNodes[3]) stores node-3 into allNodes[9], then
    # append(allNodes[3:5], allNodes[6:8]...) stores node-6, node-7 into allNodes[5], allNodes[6].
    # The tests run after the literal is built, so every allNodes[a:b] below reads the mutated array.
    mut = ALL[:5] + [ALL[6], ALL[7], ALL[7], ALL[8], ALL[3], ALL[10]]
    multi("add and remove all nodes between two Next operations", 409, mut[2:9], mut[2:9],
          ["add", "add", "next", "add", "remove", "remove", "remove", "next"], ["node-2", ""])
    multi("add and remove some nodes between two Next operations", 416, mut[2:9], mut[2:9],
          ["add", "add", "next", "add", "remove", "remove", "next"], ["node-2", "node-4"])
    multi("remove nodes already iterated on and add new nodes", 423, mut[2:9], mut[2:9],
          ["add", "add", "next", "next", "add", "remove", "remove", "next"], ["node-2", "node-3", "node-4"])
    multi("add more nodes to an exhausted zone", 430, mut[4:10], [],
          ["add"] * 5 + ["next"] * 4 + ["add"] + ["next"] * 3,
          ["node-4", "node-6", "node-7", "node-8", "node-3", "node-4", "node-6"])
    multi("remove zone and add new to ensure exhausted is reset correctly", 437, ALL[3:5] + ALL[6:8], ALL[3:5],
          ["add", "add", "next", "next", "remove", "add", "add", "next", "next", "remove", "next", "next"],
          ["node-3", "node-4", "node-6", "node-7", "node-6", "node-7"])
    return out


def all_cases():
    return ops_cases() + [
        case("should go back to the first node after finishing a round", SRC + ":366", kind="node_tree",
             nodes=ALL[:1], expect_order=["node-0"]),
        case("should go back to the first node after going over all nodes", SRC + ":372", kind="node_tree",
             nodes=ALL[:4], expect_order=["node-0", "node-1", "node-2", "node-3"]),
        case("should go to all zones before going to the second nodes in the same zone", SRC + ":378",
             kind="node_tree", nodes=ALL[:9],
             expect_order=["node-0", "node-1", "node-2", "node-3", "node-5", "node-6", "node-4", "node-7", "node-8"]),
    ]

"""Golden vectors transcribed from pkg/scheduler/framework/plugins/nodeports/node_ports_test.go (TestNodePorts).

The reference's NodeInfo there has no Node object; the fixture names its node "m1", the host every
pod of the table carries."""
from gen_common import case, container, node, pod

SRC = "pkg/scheduler/framework/plugins/nodeports/node_ports_test.go"
UNSCHED = 2
ERR = "node(s) didn't have free ports for the requested pod ports"


def new_pod(host, *infos):
    """node_ports_test.go:31 newPod: "PROTO/hostIP/hostPort" strings into one container's ports."""
    ports = []
    for s in infos:
        proto, ip, port = s.split("/")
        ports.append({"hostIP": ip, "hostPort": int(port), "protocol": proto})
    return pod(node_name=host, containers=[container(ports=ports)])


def all_cases():
    out = []

    def fc(name, line, p, existing, fail=False):
        out.append(case(name, SRC + ":%d" % line, kind="filter", plugin="NodePorts", args={}, pod=p,
                        pods=existing, nodes=[node("m1", {})],
                        expect_filter={"m1": {"code": UNSCHED if fail else 0, "reasons": [ERR] if fail else []}}))

    fc("nothing running", 65, pod(), [])
    fc("other port", 71, new_pod("m1", "UDP/127.0.0.1/8080"), [new_pod("m1", "UDP/127.0.0.1/9090")])
    fc("same udp port", 77, new_pod("m1", "UDP/127.0.0.1/8080"), [new_pod("m1", "UDP/127.0.0.1/8080")], True)
    fc("same tcp port", 84, new_pod("m1", "TCP/127.0.0.1/8080"), [new_pod("m1", "TCP/127.0.0.1/8080")], True)
    fc("different host ip", 91, new_pod("m1", "TCP/127.0.0.1/8080"), [new_pod("m1", "TCP/127.0.0.2/8080")])
    fc("different protocol", 97, new_pod("m1", "UDP/127.0.0.1/8080"), [new_pod("m1", "TCP/127.0.0.1/8080")])
    fc("second udp port conflict", 103, new_pod("m1", "UDP/127.0.0.1/8000", "UDP/127.0.0.1/8080"),
       [new_pod("m1", "UDP/127.0.0.1/8080")], True)
    fc("first tcp port conflict", 110, new_pod("m1", "TCP/127.0.0.1/8001", "UDP/127.0.0.1/8080"),
       [new_pod("m1", "TCP/127.0.0.1/8001", "UDP/127.0.0.1/8081")], True)
    fc("first tcp port conflict due to 0.0.0.0 hostIP", 117, new_pod("m1", "TCP/0.0.0.0/8001"),
       [new_pod("m1", "TCP/127.0.0.1/8001")], True)
    fc("TCP hostPort conflict due to 0.0.0.0 hostIP", 124, new_pod("m1", "TCP/10.0.10.10/8001", "TCP/0.0.0.0/8001"),
       [new_pod("m1", "TCP/127.0.0.1/8001")], True)
    fc("second tcp port conflict to 0.0.0.0 hostIP", 131, new_pod("m1", "TCP/127.0.0.1/8001"),
       [new_pod("m1", "TCP/0.0.0.0/8001")], True)
    fc("second different protocol", 138, new_pod("m1", "UDP/127.0.0.1/8001"), [new_pod("m1", "TCP/0.0.0.0/8001")])
    fc("UDP hostPort conflict due to 0.0.0.0 hostIP", 144, new_pod("m1", "UDP/127.0.0.1/8001"),
       [new_pod("m1", "TCP/0.0.0.0/8001", "UDP/0.0.0.0/8001")], True)
    return out

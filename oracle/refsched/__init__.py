"""ORACLE -- test infrastructure only.

A pure-Python restatement of the reference kube-scheduler hot path (lpastura/kubernetes-1,
Kubernetes 1.19-dev, pkg/scheduler/...) operating on k8s-v1-shaped dicts.  It is the
semantic checker for the MI355X path: pinned by golden vectors transcribed from the
reference's own table-driven unit tests (tests/golden/), and used by tests/ to check the HIP
path and the C restatement (oracle/c) on the same inputs.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import anything
under oracle/.  The product (kubernetes-1_amd/) never imports it.
"""
from . import quantity, labels, nodeinfo, plugins, framework, tiebreak, golog  # noqa: F401

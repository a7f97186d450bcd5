"""Helpers for transcribing the reference's table-driven unit tests into golden fixtures.

The fixture files (tests/golden/*.json) are DATA: inputs (k8s-v1-shaped pod/node dicts)
and the expected outputs the reference's own tests assert.  Every case carries "src", the
reference file:line of the table entry it was transcribed from.  Regenerate with
    python tests/golden/make_golden.py
"""
import copy


def rl_from_resource(milli_cpu=0, memory=0, eph=0, allowed_pods=0, scalars=None):
    """framework.Resource{...}.ResourceList() (types.go:307-323): always lists cpu, memory,
    pods and ephemeral-storage, plus every scalar."""
    out = {"cpu": "%dm" % milli_cpu, "memory": str(memory), "pods": str(allowed_pods),
           "ephemeral-storage": str(eph)}
    for k, v in (scalars or {}).items():
        out[k] = str(v)
    return out


def container(requests=None, image=None, ports=None, name=None):
    c = {}
    if name:
        c["name"] = name
    if requests is not None:
        c["resources"] = {"requests": dict(requests)}
    if image is not None:
        c["image"] = image
    if ports is not None:
        c["ports"] = list(ports)
    return c


def pod(name="", ns="", labels=None, node_name=None, containers=None, init_containers=None,
        overhead=None, uid=None, **spec):
    m = {"name": name, "namespace": ns}
    if labels is not None:
        m["labels"] = dict(labels)
    if uid is not None:
        m["uid"] = uid
    s = dict(spec)
    if node_name is not None:
        s["nodeName"] = node_name
    if containers is not None:
        s["containers"] = copy.deepcopy(containers)
    if init_containers is not None:
        s["initContainers"] = copy.deepcopy(init_containers)
    if overhead is not None:
        s["overhead"] = dict(overhead)
    return {"metadata": m, "spec": s}


def resource_pod(*usages, **kw):
    """fit_test.go newResourcePod: one container per framework.Resource."""
    return pod(containers=[container(rl_from_resource(**u)) for u in usages], **kw)


def node(name, allocatable=None, labels=None, taints=None, unschedulable=None, images=None,
         annotations=None):
    m = {"name": name}
    if labels is not None:
        m["labels"] = dict(labels)
    if annotations is not None:
        m["annotations"] = annotations
    spec = {}
    if taints is not None:
        spec["taints"] = list(taints)
    if unschedulable is not None:
        spec["unschedulable"] = unschedulable
    st = {"allocatable": dict(allocatable or {})}
    if images is not None:
        st["images"] = images
    return {"metadata": m, "spec": spec, "status": st}


def make_node_cpu_mem(name, milli_cpu, memory, **kw):
    """noderesources/test_util.go:25 makeNode."""
    return node(name, {"cpu": "%dm" % milli_cpu, "memory": str(memory)}, **kw)


def case(name, src, **kw):
    d = {"name": name, "src": src}
    d.update(kw)
    return d

"""Scheduler-extender front-end (kgpu/extender.py) against the reference wire format and the oracle.

The scheduler side of the protocol is `HTTPExtender` (core/extender.go:273-438): JSON POSTs of
`ExtenderArgs` to `<urlPrefix>/filter|prioritize|bind`, decoded as `ExtenderFilterResult`,
`HostPriorityList`, `ExtenderBindingResult` (extender/v1/types.go).  The tests drive the real HTTP
server on 127.0.0.1 exactly that way.

  * CPU: routing, status codes, error results, argument validation (no engine call).
  * GPU: a seeded scheduleOne loop through filter -> prioritize -> bind, each cycle compared with
    the Python oracle run from scratch on the same cluster state: the NodeNames that pass, the
    FailedNodes reasons, the prioritize winner (select mode) and weighted totals (total mode), and
    the cluster the binds leave behind.
"""
import json
import random
import urllib.error
import urllib.request

import pytest

from oracle.refsched import framework as F
from oracle.refsched import tiebreak as TB
from kgpu import cluster as K
from kgpu.cache import SchedulerCache
from kgpu.compile import Cluster, Profile
from kgpu.extender import GpuExtender, serve

from test_delta import Stream, _cluster


def _post(url, verb, obj, raw=None):
    data = raw if raw is not None else json.dumps(obj).encode()
    req = urllib.request.Request(url + "/" + verb, data=data, headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=30) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read() or b"{}")


class _Stub:
    def __init__(self):
        self.calls = []

    def filter(self, a):
        self.calls.append(("filter", a))
        return {"Nodes": None, "NodeNames": a.get("NodeNames"), "FailedNodes": {}, "Error": ""}

    def prioritize(self, a):
        self.calls.append(("prioritize", a))
        return [{"Host": n, "Score": 1} for n in a.get("NodeNames") or []]

    def bind(self, a):
        self.calls.append(("bind", a))
        return {"Error": ""}


def test_http_routing_and_status_codes():
    stub = _Stub()
    srv, url = serve(stub, prefix="/scheduler")
    try:
        args = {"Pod": {"metadata": {"name": "p", "uid": "u1"}}, "Nodes": None, "NodeNames": ["a", "b"]}
        assert _post(url, "filter", args) == (200, {"Nodes": None, "NodeNames": ["a", "b"], "FailedNodes": {},
                                                     "Error": ""})
        assert _post(url, "prioritize", args) == (200, [{"Host": "a", "Score": 1}, {"Host": "b", "Score": 1}])
        bind = {"PodName": "p", "PodNamespace": "default", "PodUID": "u1", "Node": "a"}
        assert _post(url, "bind", bind) == (200, {"Error": ""})
        assert [c[0] for c in stub.calls] == ["filter", "prioritize", "bind"]
        assert _post(url, "preempt", args)[0] == 404
        assert _post(url, "filter", None, raw=b"{not json")[0] == 400
    finally:
        srv.shutdown()


def test_argument_errors_without_engine():
    nodes = [K.node("n%d" % i, "4", "8Gi") for i in range(3)]
    c = SchedulerCache(Profile(), nodes, create_engine=False)
    ext = GpuExtender(c)
    with pytest.raises(ValueError):
        GpuExtender(c, mode="sum")
    # the scheduler cuts the candidate list itself: a second cut in the extender is refused
    with pytest.raises(ValueError):
        GpuExtender(SchedulerCache(Profile(percentage_of_nodes_to_score=50), nodes, create_engine=False))
    pod = K.pod("p", "100m", "128Mi")
    pod["metadata"]["uid"] = "u1"
    out = ext.filter({"Pod": pod, "Nodes": None, "NodeNames": ["n0", "nX"]})
    assert out["Error"] and "nX" in out["Error"] and out["NodeNames"] is None
    out = ext.filter({"Pod": pod, "Nodes": None, "NodeNames": None})
    assert "neither" in out["Error"]
    # a bind for a pod this extender never filtered
    assert "not filtered" in ext.bind({"PodName": "p", "PodNamespace": "default", "PodUID": "u9", "Node": "n0"})["Error"]


def _oracle(c, s, pod, seq):
    return F.schedule_sequence(c.ordered_nodes(), c.listed_pods(), [pod], F.Profile(), services=s.services,
                               rss=s.rss, first_seq=seq, order="given", image_nodes=list(c.nodes.values()))[0]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(2))
def test_extender_cycles_match_oracle(seed):
    nodes, existing, services, rss = _cluster(seed, 40)
    c = SchedulerCache(Profile(), nodes, existing, cluster=Cluster(services, rss=rss))
    ext = GpuExtender(c)
    srv, url = serve(ext)
    r = random.Random(seed)
    try:
        s = Stream(seed, c, nodes, services, rss, gpu=True)
        placed = subset_checked = 0
        for i in range(40):
            if i % 5 == 4:
                s.step()       # informer events between cycles reach the device as deltas
                c.sync()
            pod = s.fresh_pod()
            names = list(dict.fromkeys(c.list))
            if i % 3 == 2:
                names = r.sample(names, max(1, len(names) // 2))  # the scheduler's own filters removed some
            seq = ext.seq
            want = _oracle(c, s, pod, seq)
            code, out = _post(url, "filter", {"Pod": pod, "Nodes": None, "NodeNames": names})
            assert code == 200 and out["Error"] == "", out
            if isinstance(want, F.ScheduleError) and not isinstance(want, F.FitError):
                assert out["NodeNames"] == []   # PreFilter rejected the pod: no node passes
                continue
            statuses = want.statuses if isinstance(want, (F.Result, F.FitError)) else {}
            feas = set(want.feasible_names) if isinstance(want, F.Result) else set()
            assert out["NodeNames"] == [n for n in names if n in feas]
            for n in names:
                if n in feas:
                    continue
                assert n in out["FailedNodes"], n
                plugin, st = statuses[n]
                assert out["FailedNodes"][n] == (", ".join(st.reasons) if st.reasons else plugin), n
            if not out["NodeNames"]:
                continue
            code, prio = _post(url, "prioritize", {"Pod": pod, "Nodes": None, "NodeNames": out["NodeNames"]})
            assert code == 200
            top = [h["Host"] for h in prio if h["Score"] == 10]
            assert len(top) <= 1
            if want.host in out["NodeNames"]:
                assert top == [want.host]
            else:
                # the scheduler sent a strict subset without the overall winner (its own cut or
                # filters): select mode ranks the candidates it sent, by the oracle's totals
                # and the build's tie-break key
                idx = {}
                for k, n in enumerate(c.list):
                    idx.setdefault(n, k)
                tot = dict(want.totals) if want.totals else {n: 1 for n in out["NodeNames"]}
                exp = max(out["NodeNames"], key=lambda n: TB.key(tot[n], idx[n], seq, 0x7B))
                assert top == [exp], (i, top, exp)
                subset_checked += 1
            if not top:
                continue
            code, b = _post(url, "bind", {"PodName": pod["metadata"]["name"], "PodNamespace": "default",
                                          "PodUID": pod["metadata"]["uid"], "Node": top[0]})
            assert code == 200 and b["Error"] == ""
            assert pod["metadata"]["uid"] in c.states and c.states[pod["metadata"]["uid"]]["assumed"]
            placed += 1
            s.seq = ext.seq
        assert placed >= 10
        c.sync()
        s.check_rows()   # the binds are on the device rows exactly as the oracle's NodeInfos
    finally:
        srv.shutdown()
        c.close()


@pytest.mark.gpu
def test_extender_total_mode_and_node_objects():
    """mode "total": each feasible candidate's weighted total equals the oracle's; Nodes (not
    NodeNames) in and out, as for an extender the scheduler does not treat as node-cache capable."""
    nodes, existing, services, rss = _cluster(5, 30)
    c = SchedulerCache(Profile(), nodes, existing, cluster=Cluster(services, rss=rss))
    ext = GpuExtender(c, mode="total")
    srv, url = serve(ext)
    try:
        s = Stream(5, c, nodes, services, rss, gpu=True)
        checked = 0
        for _ in range(20):
            pod = s.fresh_pod()
            items = [c.nodes[n] for n in dict.fromkeys(c.list)]
            seq = ext.seq
            want = _oracle(c, s, pod, seq)
            code, out = _post(url, "filter", {"Pod": pod, "Nodes": {"metadata": {}, "items": items},
                                              "NodeNames": None})
            assert code == 200 and out["Error"] == "" and out["NodeNames"] is None
            got = [n["metadata"]["name"] for n in out["Nodes"]["items"]]
            feas = want.feasible_names if isinstance(want, F.Result) else []
            assert sorted(got) == sorted(feas)
            if not isinstance(want, F.Result) or want.feasible < 2:
                continue
            code, prio = _post(url, "prioritize", {"Pod": pod, "Nodes": out["Nodes"], "NodeNames": None})
            assert code == 200
            assert {h["Host"]: h["Score"] for h in prio} == {n: t for n, t in want.totals}
            checked += 1
        assert checked >= 5
    finally:
        srv.shutdown()
        c.close()


def test_pending_pods_are_bounded():
    """Pods filtered but never bound here (unschedulable, bound by another path, deleted) expire from
    the extender's pending map: bounded by count and by age."""
    from kgpu import extender as E
    nodes = [K.node("n%d" % i, "4", "8Gi") for i in range(2)]
    now = [0.0]
    c = SchedulerCache(Profile(), nodes, create_engine=False)
    ext = GpuExtender(c, clock=lambda: now[0])
    for i in range(E.PENDING_MAX + 50):
        ext._remember("u%d" % i, {"metadata": {"uid": "u%d" % i}})
    assert len(ext._pending) == E.PENDING_MAX
    assert "u0" not in ext._pending and "u%d" % (E.PENDING_MAX + 49) in ext._pending
    now[0] = E.PENDING_TTL + 1.0
    ext._remember("fresh", {"metadata": {"uid": "fresh"}})
    assert list(ext._pending) == ["fresh"]

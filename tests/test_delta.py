"""Delta stream (kgpu_apply_delta, kgpu/cache.py) against the reference cache semantics.

A seeded stream of informer / scheduler events (schedule + assume, confirm, forget, expire, pod
add / update / delete, node add / update / delete, pods on not-yet-known nodes) drives the host
mirror of the scheduler cache.  After every event the mirror syncs the device (UpdateSnapshot) and:

  * CPU: the mirror's list order must equal an independent replay of the node events on the
    oracle's nodeTree (oracle/refsched/nodeinfo.py NodeTreeRef), and the pods it keeps on device
    rows must equal the NodeInfo pod sets of the listed nodes;
  * GPU: a probe pod scheduled on the delta-maintained device mirror must get the placement,
    feasible count and score the Python oracle computes from scratch on the same cluster state,
    and every node row (requested, non-zero requested, pod count) must equal the oracle's NodeInfo.
"""
import copy
import random

import numpy as np
import pytest

import gen_random
from oracle.refsched import framework as F
from oracle.refsched import nodeinfo as NI
from kgpu.cache import CacheError, SchedulerCache
from kgpu.compile import Cluster, Profile


def _cluster(seed, n_nodes):
    nodes, existing, _, services, rss = gen_random.topo_cluster(seed, n_nodes=n_nodes, n_existing=2 * n_nodes,
                                                                n_pods=0)
    return nodes, existing, services, rss


class Stream:
    """Random cache events over a SchedulerCache, recording the node events for a nodeTree replay."""

    def __init__(self, seed, cache, nodes, services, rss, gpu):
        self.r = random.Random(seed)
        self.c = cache
        self.gpu = gpu
        self.services, self.rss = services, rss
        self.assumed = {}     # uid -> pod
        self.added = {}       # uid -> pod
        self.node_events = [("add", n) for n in nodes]
        self.next_pod = 0
        self.next_node = len(nodes)
        self.t = 0.0
        self.seq = 0

    def fresh_pod(self, bound_to=None):
        r = self.r
        names = list(self.c.nodes)
        p = gen_random.rpod(r, 50000 + self.next_pod, names, allow_node_name=False)
        gen_random._topo_spec(r, p["spec"], p["metadata"], p_tsc=0.4, p_aff=0.4)
        p["metadata"]["uid"] = "s%d" % self.next_pod
        p["metadata"]["name"] = "s%d" % self.next_pod
        self.next_pod += 1
        if bound_to is not None:
            p["spec"]["nodeName"] = bound_to
        return p

    def step(self):
        r, c = self.r, self.c
        op = r.choices(["sched", "confirm", "forget", "expire", "add", "remove", "update", "node_update",
                        "node_add", "node_remove", "ghost"],
                       weights=[6, 3, 2, 1, 3, 3, 2, 3, 1, 1, 1])[0]
        if op == "sched":
            p = self.fresh_pod()
            host = self.schedule_probe(p) if self.gpu else r.choice(list(c.nodes))
            if host is None:
                return op
            p["spec"]["nodeName"] = host
            c.assume_pod(p)
            self.assumed[p["metadata"]["uid"]] = p
        elif op == "confirm" and self.assumed:
            uid = r.choice(sorted(self.assumed))
            p = self.assumed.pop(uid)
            if r.random() < 0.2 and c.nodes:
                p = copy.deepcopy(p)
                p["spec"]["nodeName"] = r.choice(sorted(c.nodes))   # bound elsewhere (cache.go:470-477)
            c.add_pod(p)
            self.added[uid] = p
        elif op == "forget" and self.assumed:
            uid = r.choice(sorted(self.assumed))
            c.forget_pod(self.assumed.pop(uid))
        elif op == "expire" and self.assumed:
            uid = r.choice(sorted(self.assumed))
            c.finish_binding(self.assumed[uid], self.t)
            self.t += c.ttl + 1
            c.cleanup_assumed(self.t)
            self.assumed = {u: p for u, p in self.assumed.items() if u in c.states}
        elif op == "add" and c.nodes:
            p = self.fresh_pod(bound_to=r.choice(sorted(c.nodes)))
            c.add_pod(p)
            self.added[p["metadata"]["uid"]] = p
        elif op == "ghost":
            p = self.fresh_pod(bound_to="ghost%d" % r.randrange(3))
            c.add_pod(p)
            self.added[p["metadata"]["uid"]] = p
        elif op == "remove" and self.added:
            uid = r.choice(sorted(self.added))
            p = self.added.pop(uid)
            try:
                c.remove_pod(p)
            except CacheError:
                pass  # the pod's node was deleted and re-added: NodeInfo.RemovePod fails, as in the reference
        elif op == "update" and self.added:
            uid = r.choice(sorted(self.added))
            old = self.added[uid]
            new = copy.deepcopy(old)
            new["metadata"]["labels"] = {"app": r.choice(gen_random.APPS)}
            cont = new["spec"]["containers"][0]
            cont.setdefault("resources", {}).setdefault("requests", {})["cpu"] = "%dm" % r.choice([10, 700])
            try:
                c.update_pod(old, new)
                self.added[uid] = new
            except CacheError:
                pass
        elif op == "node_update" and c.nodes:
            nm = r.choice(sorted(c.nodes))
            old = c.nodes[nm]
            new = copy.deepcopy(old)
            lab = new["metadata"]["labels"]
            if r.random() < 0.5:
                lab[gen_random.ZONE] = "z%d" % r.randrange(4)          # may be a new value (dictionary growth)
            if r.random() < 0.3:
                lab["disk"] = r.choice(["ssd", "hdd", "nvme"])
            if r.random() < 0.3 and "disk" in lab:
                del lab["disk"]
            new["status"]["allocatable"]["cpu"] = "%dm" % r.choice([500, 4000, 64000])
            new["spec"]["unschedulable"] = r.random() < 0.1
            if r.random() < 0.3:
                new["spec"]["taints"] = [{"key": "spot", "value": "true", "effect": "PreferNoSchedule"}]
            c.update_node(old, new)
            self.node_events.append(("update", old, new))
        elif op == "node_add":
            if r.random() < 0.5:
                nm = "ghost%d" % r.randrange(3)
                if nm in c.nodes:
                    return op
                n = gen_random.rnode(r, 0)
                n["metadata"]["name"] = nm
                n["metadata"]["labels"][gen_random.HOST] = nm
            else:
                n = gen_random.rnode(r, self.next_node)
                self.next_node += 1
            n["status"]["allocatable"].update({"cpu": "64", "memory": "256Gi", "pods": "110"})
            c.add_node(n)
            self.node_events.append(("add", n))
        elif op == "node_remove" and len(c.nodes) > 4:
            nm = r.choice(sorted(c.nodes))
            n = c.nodes[nm]
            c.remove_node(n)
            self.node_events.append(("remove", n))
        return op

    def schedule_probe(self, pod):
        host, res = self.c.schedule(pod, seq=self.seq)
        want = F.schedule_sequence(self.c.ordered_nodes(), self.c.listed_pods(), [pod], F.Profile(),
                                   services=self.services, rss=self.rss, first_seq=self.seq, order="given",
                                   image_nodes=list(self.c.nodes.values()))[0]
        self.seq += 1
        if isinstance(want, F.ScheduleError):
            assert int(res["node"]) < 0, "oracle: %s, device placed on %s" % (want, host)
            return None
        assert host == want.host, "device %s vs oracle %s" % (host, want.host)
        assert int(res["feasible"]) == want.feasible
        if want.feasible > 1:
            assert int(res["score"]) == dict(want.totals)[want.host]
        return host

    def check_rows(self):
        c = self.c
        snap = NI.Snapshot(c.ordered_nodes(), c.listed_pods(), order="given")
        rows = c.engine.read_nodes(len(c.list))
        for i, ni in enumerate(snap.list):
            got = (int(rows["req_cpu"][i]), int(rows["req_mem"][i]), int(rows["nz_cpu"][i]), int(rows["nz_mem"][i]),
                   int(rows["num_pods"][i]))
            want = (ni.requested.milli_cpu, ni.requested.memory, ni.non_zero.milli_cpu, ni.non_zero.memory,
                    len(ni.pods))
            assert got == want, "node %s row %r vs oracle %r" % (c.list[i], got, want)


def _tree_replay(events):
    t = NI.NodeTreeRef()
    for ev in events:
        if ev[0] == "add":
            t.add_node(ev[1])
        elif ev[0] == "remove":
            t.remove_node(ev[1])
        else:
            t.update_node(ev[1], ev[2])
    return t


@pytest.mark.parametrize("seed", range(4))
def test_cache_mirror_host_bookkeeping(seed):
    nodes, existing, services, rss = _cluster(seed, 24)
    c = SchedulerCache(Profile(), nodes, existing, cluster=Cluster(services, rss=rss), create_engine=False)
    s = Stream(seed, c, nodes, services, rss, gpu=False)
    tree = _tree_replay(s.node_events)
    want_list = [tree.next() for _ in range(tree.num_nodes)]
    assert c.list == want_list
    for _ in range(120):
        before = len(s.node_events)
        s.step()
        changed = any(ev[0] in ("add", "remove") for ev in s.node_events[before:])
        for ev in s.node_events[before:]:
            if ev[0] == "add":
                tree.add_node(ev[1])
            elif ev[0] == "remove":
                tree.remove_node(ev[1])
            else:
                tree.update_node(ev[1], ev[2])
        c.sync()
        if changed:
            # updateAllLists: the list is the next numNodes outputs of the (stateful) nodeTree
            want_list = [tree.next() for _ in range(tree.num_nodes)]
        assert c.list == want_list
        want_dev = {u: nm for nm in dict.fromkeys(c.list) for u in c.node_pods.get(nm, {})}
        assert c.dev_pods == want_dev


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_delta_stream_matches_oracle(seed):
    nodes, existing, services, rss = _cluster(seed, 40)
    c = SchedulerCache(Profile(), nodes, existing, cluster=Cluster(services, rss=rss))
    try:
        s = Stream(seed, c, nodes, services, rss, gpu=True)
        s.check_rows()
        for _ in range(60):
            s.step()
            c.sync()
            s.check_rows()
            s.schedule_probe(s.fresh_pod())
        assert c.uploads >= 1
    finally:
        c.close()


@pytest.mark.gpu
def test_forget_snapshot_and_assumed_pods():
    """kgpu_forget_pod on batch-assumed pods (one k_delta op) and REMOVE_POD of snapshot pods bring
    the rows back to the oracle's NodeInfos."""
    from kgpu.framework import GpuFramework
    nodes, existing, pods = gen_random.cluster(7, n_nodes=30, n_existing=40, n_pods=20)
    fw = GpuFramework(Profile(), nodes, existing, pods_hint=pods)
    try:
        res = fw.schedule(pods)
        placed = [i for i in range(len(pods)) if res[i]["node"] >= 0]
        assert placed
        slot0 = fw.snap.n_pods
        # forget every other assumed pod
        kept = []
        for k, i in enumerate(placed):
            if k % 2 == 0:
                fw.engine.forget(slot0 + k)
            else:
                p = copy.deepcopy(pods[i])
                p["spec"]["nodeName"] = fw.order[int(res[i]["node"])]
                kept.append(p)
        snap = NI.Snapshot([fw.nodes[nm] for nm in fw.order], list(existing) + kept, order="given")
        rows = fw.engine.read_nodes(len(fw.order))
        for j, ni in enumerate(snap.list):
            assert int(rows["req_cpu"][j]) == ni.requested.milli_cpu
            assert int(rows["num_pods"][j]) == len(ni.pods)
    finally:
        fw.engine.close()


@pytest.mark.gpu
def test_host_ports_beyond_initial_slots():
    """More distinct host-port pods on one node than the snapshot's port slots: every UsedPorts entry
    is kept (the slot table grows), so NodePorts keeps rejecting each taken port."""
    from kgpu.framework import GpuFramework
    node = {"metadata": {"name": "solo", "labels": {"kubernetes.io/hostname": "solo"}}, "spec": {},
            "status": {"allocatable": {"cpu": "64", "memory": "64Gi", "pods": "110"}}}

    def port_pod(i, port):
        return {"metadata": {"name": "pp%d" % i, "namespace": "default", "uid": "pp%d" % i},
                "spec": {"containers": [{"name": "c", "ports": [{"containerPort": 80, "hostPort": port,
                                                                 "protocol": "TCP"}]}]}}

    pods = [port_pod(i, 20000 + i) for i in range(12)] + [port_pod(100 + i, 20000 + i) for i in range(12)]
    fw = GpuFramework(Profile(), [node], [], pods_hint=pods)
    try:
        res = fw.schedule(pods)
        assert all(int(r["node"]) == 0 for r in res[:12])
        assert all(int(r["node"]) == -1 for r in res[12:]), [int(r["node"]) for r in res]
    finally:
        fw.engine.close()

"""KGPU_OPT_TOPO_RESIDENT: a persistent topology run starts from the histograms, pair
registrations and eligibility bitmaps the previous run with the same tables left on the device
(k_tbatch writes its final bins back), instead of a k_tbatch_init pass over every node.

The resident state is only valid while nothing else changed the mirror: kgpu_forget_pod, deltas,
uploads and the other evaluation paths' assumes must drop it.  Two engines on the same cluster --
resident state on and off -- run the same sequence of kgpu_schedule_one cycles with assume,
interleaved with forgets of earlier pods, short batches and (in the mixed profile) pods that take
the non-topology paths; every cycle's record, status words and per-plugin scores, and the final node
rows, must agree.  The off engine is the init-per-run path the rest of the suite pins against the C
restatement; the on engine must have started runs from the resident state (the state is kept for one
set of tables: a run of pods of one template reuses it, a template change recomputes it, starting
from the spare buffer the previous run zeroed)."""
import json

import numpy as np
import pytest

import gen_random
from kgpu import abi, cluster
from kgpu.compile import Cluster, Profile
from kgpu.framework import GpuFramework

ROW_KEYS = ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")


def _case(name):
    if name == "spread":
        return cluster.taints_affinity_spread(n_nodes=400, n_pods=90) + (None,)
    if name == "affinity":
        # InterPodAffinity pods grouped by template (a deployment's pods arrive together): the
        # resident state serves the runs of one template and is recomputed at each template change
        nodes, existing, pods, prof = cluster.pod_affinity(n_nodes=300, n_existing=300, n_pods=90)
        pods = sorted(pods, key=lambda p: json.dumps(p["spec"].get("affinity"), sort_keys=True))
        return nodes, existing, pods, prof, None
    if name == "cycling":
        # config (d)'s arrival order: consecutive pods bring other tables, so every run misses and starts
        # from the spare buffer the previous run zeroed (no memset)
        return cluster.pod_affinity(n_nodes=300, n_existing=300, n_pods=60) + (None,)
    nodes, existing, pods, services, rss = gen_random.topo_cluster(11, n_nodes=120, n_existing=240, n_pods=90)
    return nodes, existing, pods, Profile(), Cluster(services=services, rss=rss)


class _Oracle:
    """The C restatement (oracle/c) run from scratch on the cluster as the device should hold it:
    the initial pods, plus every pod placed since, minus the forgotten ones."""

    def __init__(self, fw, nodes, existing, pods, prof, cl):
        self.nodes, self.pods, self.prof, self.cl = nodes, pods, prof, cl
        self.existing = list(existing)
        self.order = fw.order

    def run(self, idx, seq):
        from oracle.cref import RefEngine
        ref_fw = GpuFramework(self.prof, self.nodes, self.existing, cluster=self.cl, pods_hint=self.pods,
                              create_engine=False)
        assert ref_fw.order == self.order
        q, pc, _, errs = ref_fw.compile_pods([self.pods[i] for i in idx])
        assert not errs
        ref = RefEngine(ref_fw.config, ref_fw.snap, threads=4)
        out = ref.schedule(q, pc, first_seq=seq, diag=True)
        ref.close()
        return out

    def place(self, i, node):
        p = json.loads(json.dumps(self.pods[i]))
        p["spec"]["nodeName"] = self.order[node]
        self.existing.append(p)
        return p

    def forget(self, p):
        self.existing.remove(p)


def _drive(fw, q, pc, resident, oracle=None):
    e = fw.engine
    e.upload(fw.snap, fw.arrays)
    e.set_option(abi.OPT_TOPO_RESIDENT, 1 if resident else 0)
    n = fw.snap.n_nodes
    out = []
    slots = []
    i = 0
    while i < len(q):
        if i % 23 == 11:  # a short batch of four pods
            res, _ = e.schedule_batch(q[i:i + 4], pc, first_seq=i)
            out.append(("batch", res.copy()))
            if oracle is not None:
                want = oracle.run(range(i, min(i + 4, len(q))), i)[0]
                for f in ("node", "feasible", "scored", "score"):
                    np.testing.assert_array_equal(res[f], want[f], err_msg="batch at %d: %s vs oracle/c" % (i, f))
                for k, r in enumerate(res):
                    if r["node"] >= 0:
                        oracle.place(i + k, int(r["node"]))
            i += 4
            continue
        if i % 17 == 9 and slots:  # forget a pod placed earlier (NodeInfo.RemovePod through k_delta)
            slot, placed = slots.pop(0)
            e.forget(slot)
            if oracle is not None:
                oracle.forget(placed)
        res, slot = e.schedule_one(q[i], pc, seq=i, assume=True)
        words = e.filter_words(n).copy()
        scores = [e.scores(s, n) for s in range(abi.NUM_SCORES)]
        placed = None
        if oracle is not None:
            w, st, raw, norm = oracle.run([i], i)
            for f in ("node", "feasible", "scored", "score"):
                assert res[f] == w[0][f], "cycle %d: %s %s vs oracle/c %s" % (i, f, res[f], w[0][f])
            np.testing.assert_array_equal(words, st, err_msg="cycle %d: status words vs oracle/c" % i)
            feas = st == 0
            # one feasible node is returned unscored (generic_scheduler.go:184-191): the reference has no
            # scores then, the device's diagnostic rows are not compared
            for s in range(abi.NUM_SCORES if res["feasible"] > 1 else 0):
                np.testing.assert_array_equal(scores[s][1][feas], norm[s][feas],
                                              err_msg="cycle %d: normalized score %d vs oracle/c" % (i, s))
            if res["node"] >= 0:
                placed = oracle.place(i, int(res["node"]))
        if res["node"] >= 0:
            slots.append((slot, placed))
        out.append(("one", res.copy(), words, scores))
        i += 1
    rows = e.read_nodes(n)
    return out, rows, e.topo_resident()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["spread", "affinity", "cycling", "mixed"])
def test_resident_topology_state_matches_init(name):
    nodes, existing, pods, prof, cl = _case(name)
    fw_on = GpuFramework(prof, nodes, existing, cluster=cl, pods_hint=pods)
    fw_off = GpuFramework(prof, nodes, existing, cluster=cl, pods_hint=pods)
    q, pc, _, errs = fw_on.compile_pods(pods)
    assert not errs
    q2, pc2, _, _ = fw_off.compile_pods(pods)
    # the resident engine is checked against oracle/c at every cycle and batch, the init-per-run engine
    # against the resident one
    got_on, rows_on, (hits_on, _) = _drive(fw_on, q, pc, True,
                                           oracle=_Oracle(fw_on, nodes, existing, pods, prof, cl))
    got_off, rows_off, (hits_off, _) = _drive(fw_off, q2, pc2, False)
    assert hits_off == 0
    if name not in ("mixed", "cycling"):  # random pods: consecutive cycles rarely share a template
        assert hits_on > 0, "no run started from the resident state"
    assert len(got_on) == len(got_off)
    for k, (a, b) in enumerate(zip(got_on, got_off)):
        assert a[0] == b[0]
        for f in ("node", "feasible", "scored", "score"):
            np.testing.assert_array_equal(a[1][f], b[1][f], err_msg="%s step %d: %s" % (name, k, f))
        if a[0] == "one":
            np.testing.assert_array_equal(a[2], b[2], err_msg="%s step %d: status words" % (name, k))
            for s in range(abi.NUM_SCORES):
                np.testing.assert_array_equal(a[3][s][0], b[3][s][0], err_msg="%s step %d: raw %d" % (name, k, s))
                np.testing.assert_array_equal(a[3][s][1], b[3][s][1], err_msg="%s step %d: norm %d" % (name, k, s))
    for k in ROW_KEYS:
        np.testing.assert_array_equal(rows_on[k], rows_off[k], err_msg="%s: %s" % (name, k))
    fw_on.engine.close()
    fw_off.engine.close()


@pytest.mark.gpu
@pytest.mark.parametrize("resident", [0, 1])
def test_resident_state_dropped_by_deltas(resident):
    """Every delta batch drops the resident state: a node removal is an order-only batch
    (rows move, no op is sent), a node update a SET_NODE, a node add a list rebuild with a seeded row.
    Pods of one template (same tables) are scheduled between those events on the SchedulerCache's
    delta-maintained mirror; every cycle is checked against the Python oracle run from scratch on the
    same cluster state, so a run that started from bitmaps of the old row order would show."""
    import copy
    import random
    from kgpu.cache import SchedulerCache
    from oracle.refsched import framework as F
    nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=48, n_pods=4)
    template = pods[0]
    c = SchedulerCache(prof, nodes, existing, pods_hint=pods)
    r = random.Random(7)
    try:
        c.engine.set_option(abi.OPT_TOPO_RESIDENT, resident)
        placed = 0
        for step in range(28):
            kind = step % 4
            names = sorted(c.nodes)
            if kind == 1:    # node removal: an order-only delta batch
                c.remove_node(c.nodes[r.choice(names)])
            elif kind == 2:  # node update: SET_NODE with the list order unchanged
                old = c.nodes[r.choice(names)]
                new = copy.deepcopy(old)
                new["status"]["allocatable"]["cpu"] = r.choice(["2", "8", "64"])
                c.update_node(old, new)
            elif kind == 3:  # node add: list rebuild
                n = cluster.node("extra%d" % step, "16", "64Gi", 110, "100Gi",
                                 labels={cluster.ZONE: "zone%d" % r.randrange(1, 4), cluster.HOSTNAME: "extra%d" % step})
                c.add_node(n)
            p = copy.deepcopy(template)
            p["metadata"]["name"] = p["metadata"]["uid"] = "t%d" % step
            host, res = c.schedule(p, seq=step)
            want = F.schedule_sequence(c.ordered_nodes(), c.listed_pods(), [p], F.Profile(), first_seq=step,
                                       order="given", image_nodes=list(c.nodes.values()))[0]
            if isinstance(want, F.ScheduleError):
                assert int(res["node"]) < 0, "step %d: oracle %s, device placed on %s" % (step, want, host)
                continue
            assert host == want.host, "step %d: device %s vs oracle %s" % (step, host, want.host)
            assert int(res["feasible"]) == want.feasible
            if kind == 0 and step % 8 == 0:  # place some of them, so the spread counts move
                p["spec"]["nodeName"] = host
                c.assume_pod(p)
                placed += 1
        hits, _ = c.engine.topo_resident()
        assert placed > 0
        if resident:
            assert hits > 0, "no cycle started from the resident state"
        else:
            assert hits == 0
    finally:
        c.close()

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


def _drive(fw, q, pc, resident):
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
            i += 4
            continue
        if i % 17 == 9 and slots:  # forget a pod placed earlier (NodeInfo.RemovePod through k_delta)
            e.forget(slots.pop(0))
        res, slot = e.schedule_one(q[i], pc, seq=i, assume=True)
        if res["node"] >= 0:
            slots.append(slot)
        words = e.filter_words(n).copy()
        scores = [e.scores(s, n) for s in range(abi.NUM_SCORES)]
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
    got_on, rows_on, (hits_on, _) = _drive(fw_on, q, pc, True)
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

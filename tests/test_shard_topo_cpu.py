"""Node sharding with topology plugins on the CPU: world_size-2 and -4 gloo ranks.

tests/test_shard_cpu.py pins the combine rule for pods whose only cross-node state is the
DefaultNormalizeScore maxima.  This file pins the rule for PodTopologySpread, InterPodAffinity and
DefaultPodTopologySpread, whose PreFilter / PreScore state is a function of EVERY node of the cluster:

* every rank holds a Snapshot, but reads only its contiguous shard of Snapshot.List() (a stale copy
  of the other rank's nodes is never touched: only the owning rank applies an assume, so any read of a
  foreign node would diverge from the unsharded result);
* PodTopologySpread PreFilter (podtopologyspread/filtering.go:146-273): each rank sends the pairs its
  eligible nodes register and the matching-pod count of every pair its nodes carry; the cluster's
  TpPairToMatchNum is the SUM over ranks, restricted to the UNION of the registrations, and
  criticalPaths are rebuilt from it (the MIN the device takes over the summed histograms);
* PodTopologySpread PreScore (scoring.go:59-132): ignored nodes and the distinct pairs of the
  filtered nodes are unions (topologyNormalizingWeight counts the union), the hostname size is
  SUM(filtered) - SUM(ignored), and the pair counts are SUMs;
* InterPodAffinity PreFilter / PreScore (interpodaffinity/filtering.go:166-271, scoring.go:160-224):
  the three filter maps and topologyScore are SUMs of the shard maps;
* NormalizeScore: TaintToleration / NodeAffinity MAX, PodTopologySpread MIN / MAX over non-ignored
  nodes, InterPodAffinity MIN / MAX, DefaultPodTopologySpread MAX per node and SUM per zone;
* selectHost: the max packed key over the ranks' best keys (global node index) with the SUMmed
  feasible count must be the unsharded scheduleOne's choice, pod after pod.

The expected side is the unsharded Python oracle (oracle/refsched framework.schedule_sequence) and,
for the world-4 runs, the C restatement (oracle/c) over the whole cluster as well: its placements are
the device's parity anchor, so the combine rule is pinned against both restatements."""
import copy
import os

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kgpu import cluster


def _rendezvous_file():
    """A fresh path for torch.distributed's FileStore (the file must not exist yet)."""
    import tempfile
    return os.path.join(tempfile.mkdtemp(prefix="kgpu_rdv_"), "store")


def _workload(name):
    if name == "spread":  # config (c) shape
        nodes, existing, pods, _ = cluster.taints_affinity_spread(n_nodes=90, n_pods=36)
    elif name == "interpod":  # config (d) shape
        nodes, existing, pods, _ = cluster.pod_affinity(n_nodes=48, n_existing=48, n_pods=32)
    elif name == "sharded_spread":  # config (e) generator, small: zone = i % 16, NodeAffinity admits zone1..zone4
        nodes, existing, pods, _ = cluster.sharded_spread(n_nodes=160, n_pods=36, n_zones=16)
    elif name == "sharded_spread_e4":  # config (e) shape over four shards: zone = i % 64 as the bench's 125k shards
        nodes, existing, pods, _ = cluster.sharded_spread(n_nodes=256, n_pods=40, n_zones=64)
    else:
        nodes, existing, pods, _ = cluster.uneven_zones()
    return nodes, existing, pods


class _ShardView:
    """A Snapshot seen through one rank's shard: List() is the shard; Get() and NumNodes() are the
    cluster's (ImageLocality's spread divides by the cluster's node count, as n_total_nodes does)."""

    def __init__(self, snap, base, cnt):
        self.full = snap
        self.list = snap.list[base:base + cnt]
        self.map = snap.map

    def num_nodes_listed(self):
        return self.full.num_nodes_listed()

    def get(self, n):
        return self.full.map[n]

    def have_pods_with_affinity(self):
        return [ni for ni in self.list if ni.pods_with_affinity]


def _gather(obj, world):
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def _sum_maps(parts):
    m = {}
    for p in parts:
        for k, v in p.items():
            m[k] = m.get(k, 0) + v
    return {k: v for k, v in m.items() if v != 0}


def _rank_main(rank, world, port, name, out):
    # a rendezvous file, not a port: a free-port probe can race another process for the port
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        from oracle.refsched import framework as F
        from oracle.refsched import nodeinfo as NI
        from oracle.refsched import plugins as P
        from oracle.refsched import tiebreak

        nodes, existing, pods = _workload(name)
        prof = F.Profile()
        want = F.schedule_sequence(nodes, existing, pods, prof)
        want_c = None
        if world > 2:
            # the C restatement over the whole cluster (default provider profile, like F.Profile())
            from kgpu.compile import Profile
            from kgpu.framework import GpuFramework
            from oracle.cref import RefEngine
            full = GpuFramework(Profile(), nodes, existing, pods_hint=pods, create_engine=False)
            q, pc, _, errs = full.compile_pods(pods)
            assert not errs, errs
            ref = RefEngine(full.config, full.snap)
            rc = ref.schedule(q, pc)
            ref.close()
            want_c = [full.order[int(x)] if int(x) >= 0 else None for x in rc["node"]]

        snap = NI.Snapshot(nodes, existing)
        N = len(snap.list)
        base, cnt = rank * N // world, (rank + 1) * N // world - rank * N // world
        view = _ShardView(snap, base, cnt)
        mine = {NI.name(ni.node) for ni in view.list}
        gidx = {NI.name(ni.node): base + i for i, ni in enumerate(view.list)}
        fw = F.Framework(prof, F.Handle(view))
        pts = fw.plugins.get("PodTopologySpread")
        ipa = fw.plugins.get("InterPodAffinity")
        scored = {pl.name for pl, _ in fw.scores if hasattr(pl, "normalize")}
        assert scored <= {"TaintToleration", "NodeAffinity", "PodTopologySpread", "InterPodAffinity",
                          "DefaultPodTopologySpread"}, scored
        n_topo = 0
        for k, pod in enumerate(pods):
            ns = NI.namespace(pod)
            state = {}
            assert P.is_success(fw.run_prefilter(state, pod))  # per-pod prefilters; topology ones redone below
            # ---- PodTopologySpread PreFilter, sharded (filtering.go:146-273)
            cons = pts._constraints(pod, "DoNotSchedule")
            reg, cnts = set(), {}
            for ni in view.list:
                nl = NI.labels_of(ni.node)
                if cons and P.pod_matches_node_selector_and_affinity_terms(pod, ni.node) and \
                        P.node_labels_match_spread(nl, cons):
                    for c in cons:
                        reg.add((c[1], nl[c[1]]))
                for c in cons:
                    pair = (c[1], nl.get(c[1], ""))
                    cnts[pair] = cnts.get(pair, 0) + P.count_pods_match_selector(ni.pods, c[2], ns)
            parts = _gather((reg, cnts), world)
            pairs = {}
            for p in set().union(*[r for r, _ in parts]):
                pairs[p] = sum(c.get(p, 0) for _, c in parts)
            paths = {c[1]: P.CriticalPaths() for c in cons}
            for (key, v), num in sorted(pairs.items()):
                paths[key].update(v, num)
            state["PreFilterPodTopologySpread"] = {"constraints": cons, "pairs": pairs, "paths": paths}
            n_topo += bool(cons) or bool(NI.has_pod_affinity_fields(pod))
            # ---- InterPodAffinity PreFilter: the shard maps, summed
            ipa.prefilter(state, pod)
            s = state["PreFilterInterPodAffinity"]
            parts = _gather((s["existing_anti"], s["aff"], s["anti"]), world)
            for j, key in enumerate(("existing_anti", "aff", "anti")):
                s[key] = _sum_maps([p[j] for p in parts])
            # ---- Filter this rank's nodes (percentageOfNodesToScore = 100)
            feasible = []
            for ni in view.list:
                plugin, st = fw.run_filters(state, pod, ni)
                assert st is None or st.code != P.ERROR, (k, plugin, st)
                if st is None:
                    feasible.append(ni.node)
            counts = _gather((len(feasible), [NI.name(n) for n in feasible[:1]]), world)
            total = sum(c for c, _ in counts)
            w = want[k]
            if total == 0:
                assert isinstance(w, F.FitError), "pod %d: shards found no node, unsharded %r" % (k, w)
                assert want_c is None or want_c[k] is None, "pod %d: oracle/c placed it on %s" % (k, want_c[k])
                continue
            assert not isinstance(w, F.ScheduleError), "pod %d: unsharded failed: %r" % (k, w)
            assert total == w.feasible, "pod %d: feasible %d vs %d" % (k, total, w.feasible)
            if total == 1:  # generic_scheduler.go:184-191: no scoring
                host = next(h[0] for c, h in counts if c)
            else:
                # ---- PreScore: per-pod plugins on the shard; the two cluster-wide states redone
                fw.run_prescore(state, pod, [ni.node for ni in view.list])
                soft = pts._constraints(pod, "ScheduleAnyway")
                ignored, fpairs, call = set(), set(), {}
                if soft:
                    for node in feasible:
                        nl = NI.labels_of(node)
                        if not P.node_labels_match_spread(nl, soft):
                            ignored.add(NI.name(node))
                            continue
                        for c in soft:
                            if c[1] != NI.LABEL_HOSTNAME:
                                fpairs.add((c[1], nl[c[1]]))
                    for ni in view.list:
                        nl = NI.labels_of(ni.node)
                        if not P.pod_matches_node_selector_and_affinity_terms(pod, ni.node) or \
                                not P.node_labels_match_spread(nl, soft):
                            continue
                        for c in soft:
                            pair = (c[1], nl[c[1]])
                            call[pair] = call.get(pair, 0) + P.count_pods_match_selector(ni.pods, c[2], ns)
                parts = _gather((len(ignored), fpairs, call), world)
                n_ign = sum(p[0] for p in parts)
                upairs = set().union(*[p[1] for p in parts])
                pst = {"constraints": soft, "ignored": ignored, "weights": [],
                       "counts": {p: sum(q[2].get(p, 0) for q in parts) for p in upairs}}
                for c in soft:
                    sz = total - n_ign if c[1] == NI.LABEL_HOSTNAME else sum(1 for p in upairs if p[0] == c[1])
                    pst["weights"].append(P.go_log(float(sz + 2)))
                state["PreScorePodTopologySpread"] = pst
                if "PreScoreInterPodAffinity" in state:
                    parts = _gather(state["PreScoreInterPodAffinity"], world)
                    topo = {}
                    for p in parts:
                        for key, vals in p.items():
                            d = topo.setdefault(key, {})
                            for v, x in vals.items():
                                d[v] = d.get(v, 0) + x
                    state["PreScoreInterPodAffinity"] = topo
                # ---- raw scores of the shard's feasible nodes, then the cluster-wide normalize stats
                raw = {}
                for pl, _ in fw.scores:
                    raw[pl.name] = [pl.score(state, pod, NI.name(n))[0] for n in feasible]
                loc = {}
                for nm, vals in raw.items():
                    if nm == "PodTopologySpread":
                        kept = [v for n, v in zip(feasible, vals) if NI.name(n) not in ignored]
                        loc[nm] = (min(kept, default=2 ** 63 - 1), max(kept, default=0))
                    elif nm == "InterPodAffinity":
                        loc[nm] = (min(vals, default=0), max(vals, default=0))
                    elif nm == "DefaultPodTopologySpread":
                        zs = {}
                        for n, v in zip(feasible, vals):
                            z = NI.get_zone_key(n)
                            if z != "":
                                zs[z] = zs.get(z, 0) + v
                        loc[nm] = (max(vals, default=0), zs)
                    else:
                        loc[nm] = max(vals, default=0)
                parts = _gather(loc, world)
                stat = {}
                for nm in loc:
                    ps = [p[nm] for p in parts]
                    if nm in ("PodTopologySpread", "InterPodAffinity"):
                        stat[nm] = (min(p[0] for p in ps), max(p[1] for p in ps))
                    elif nm == "DefaultPodTopologySpread":
                        zones = {}  # zones with a zero sum still count toward haveZones
                        for p in ps:
                            for z, x in p[1].items():
                                zones[z] = zones.get(z, 0) + x
                        stat[nm] = (max(p[0] for p in ps), zones)
                    else:
                        stat[nm] = max(ps)
                best, host = -1, None
                tk_seq = k
                for i, n in enumerate(feasible):
                    nm_n = NI.name(n)
                    tot = 0
                    for pl, wt in fw.scores:
                        v = raw[pl.name][i]
                        if pl.name in ("TaintToleration", "NodeAffinity"):  # helper/normalize_score.go:26-54
                            mx = stat[pl.name]
                            rev = pl.name == "TaintToleration"
                            if mx == 0:
                                v = P.MAX_NODE_SCORE if rev else v
                            else:
                                v = P.go_div(P.MAX_NODE_SCORE * v, mx)
                                v = P.MAX_NODE_SCORE - v if rev else v
                        elif pl.name == "PodTopologySpread":  # scoring.go:211-257
                            mn, mx = stat[pl.name]
                            if nm_n in ignored:
                                v = 0
                            elif mx == 0:
                                v = P.MAX_NODE_SCORE
                            else:
                                v = P.go_div(P.MAX_NODE_SCORE * (mx + mn - v), mx)
                        elif pl.name == "InterPodAffinity" and state["PreScoreInterPodAffinity"]:
                            mn, mx = stat[pl.name]
                            mn, mx = min(mn, 0), max(mx, 0)  # scoring.go:239-272 starts both at 0
                            v = int(float(P.MAX_NODE_SCORE) * (float(v - mn) / float(mx - mn))) if mx > mn else 0
                        elif pl.name == "DefaultPodTopologySpread" and not pl._skip(pod):
                            mnode, zones = stat[pl.name]
                            f = float(P.MAX_NODE_SCORE)
                            if mnode > 0:
                                f = float(P.MAX_NODE_SCORE) * (float(mnode - v) / float(mnode))
                            z = NI.get_zone_key(n)
                            if zones and z != "":
                                mz = max(zones.values())
                                zsc = float(P.MAX_NODE_SCORE)
                                if mz > 0:
                                    zsc = float(P.MAX_NODE_SCORE) * (float(mz - zones.get(z, 0)) / float(mz))
                                f = (f * (1.0 - P.ZONE_WEIGHTING)) + (P.ZONE_WEIGHTING * zsc)
                            v = int(f)
                        assert P.MIN_NODE_SCORE <= v <= P.MAX_NODE_SCORE, (k, pl.name, v)
                        tot += v * wt
                    key = tiebreak.key(tot, gidx[nm_n], tk_seq, prof.seed, prof.tie_break_mode)
                    if key > best:
                        best, host = key, nm_n
                recs = _gather((best, host), world)
                host = max(recs)[1]
            assert host == w.host, "pod %d: shards chose %s, unsharded %s" % (k, host, w.host)
            assert want_c is None or host == want_c[k], "pod %d: shards chose %s, oracle/c %s" % (k, host, want_c[k])
            if host in mine:  # only the owning rank applies the assume (cache.go AssumePod)
                placed = copy.deepcopy(pod)
                placed["spec"]["nodeName"] = host
                snap.get(host).add_pod(placed)
        assert n_topo > 0
        out.put((rank, "ok"))
    except Exception as e:  # surfaced by the parent
        out.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _run(name, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous_file()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    got = dict(q.get(timeout=5) for _ in range(world))
    assert got == {r: "ok" for r in range(world)}, got
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("name", ["spread", "interpod", "sharded_spread", "uneven"])
def test_shard_topology_combine_gloo_world2(name):
    _run(name, 2)


@pytest.mark.parametrize("name", ["sharded_spread_e4", "spread", "interpod"])
def test_shard_topology_combine_gloo_world4(name):
    """Four ranks (the combine's associativity beyond a pair; the (e) shape with 64 zones over four
    shards), checked against the Python oracle and oracle/c on the whole cluster."""
    _run(name, 4)

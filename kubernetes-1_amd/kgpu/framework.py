"""The plugin-side mirror of the reference framework for the GPU path.

`GpuFramework` plays the role of the out-of-tree plugin set the Go shim registers:
it holds the compiled, device-resident snapshot (cache.UpdateSnapshot), compiles each pod once
(the PreFilter-time work), and runs the scheduling cycle on libkgpu:

  cycle(pod)      -> per-node filter statuses (RunFilterPlugins + PluginToStatus.Merge,
                     framework/v1alpha1/framework.go:477-502) and per-plugin raw / normalized
                     scores (RunScorePlugins, framework.go:579-656) + the selected host
  schedule(pods)  -> the scheduleOne loop (scheduler.go:509-593) with on-device assume

Status reasons are rebuilt from the device's status word by libkgpu's kgpu_filter_reasons, exactly
as the plugins format them (file:line at each message in csrc/kgpu_reasons.h).
"""
import numpy as np

from . import abi
from . import api
from .compile import CompileError, Compiler, Pools
from . import native
from .native import Engine

def node_taints(compiler, node):
    """A node's Spec.Taints in spec order as kgpu_filter_reasons takes them: (key, value, effect,
    taint dictionary id)."""
    out = []
    if node is None:
        return out
    for t in api.spec(node).get("taints") or []:
        k, v, e = t.get("key", "") or "", t.get("value", "") or "", t.get("effect", "") or ""
        out.append((k, v, e, compiler.taints.get((k, v, e))))
    return out


def status_reasons(filters, compiler, nodes, pod, node_name, word, handle=None, node=-1, compiled=None,
                   scalar_names=None):
    """(code, plugin, reasons) of a node's device status word, None for a feasible node.  The reasons
    come from libkgpu's kgpu_filter_reasons, the formatter the Go shim's Filter calls too, which
    writes them exactly as the failing plugin does (file:line at each message in kgpu_reasons.h).
    filters: the profile's filter plugins in order; nodes: name -> v1.Node; handle: the engine that
    produced the word (None: pure formatting); node: the word's local node index; compiled: the pod's
    (query, pools) when the caller holds them; scalar_names: compiler.scalar_names(pod) when the caller
    holds them (a cycle formats many nodes' reasons for one pod)."""
    pos = word & 0xFF
    if pos == 0 or word == abi.STATUS_NOT_EVALUATED:
        return None
    plugin = filters[pos - 1]
    code = (word >> 8) & 3
    if compiled is None:
        pools = Pools()
        q = compiler.compile_pod(pod, pools)
        pc, _ = pools.finalize()
    else:
        q, pc = compiled
    if scalar_names is None:
        scalar_names = compiler.scalar_names(pod)
    reasons = native.filter_reasons(handle, q, pc, node, word, node_taints(compiler, nodes.get(node_name)),
                                    scalar_names,
                                    filters=None if handle else [abi.FILTER_IDS[f] for f in filters])
    return code, plugin, reasons


class CycleResult:
    def __init__(self, host, result, statuses, scores, plugin_statuses=None):
        self.host = host            # node name or None
        self.result = result        # kgpu_result record
        self.statuses = statuses    # {node: (code, plugin, reasons)} for infeasible nodes
        self.scores = scores        # {plugin: {node: (raw, normalized)}} over feasible nodes
        # runAllFilters: {node: {plugin: (code, reasons)}} -- RunFilterPlugins' PluginToStatus, whose
        # Merge is `statuses` (code merged, reasons of every failing plugin in profile order; the plugin
        # named there is the first failing one)
        self.plugin_statuses = plugin_statuses


def nodes_where_preemption_might_help(order, codes):
    """nodesWherePreemptionMightHelp (generic_scheduler.go:1041-1056): every node of `order` whose
    filter status in `codes` ({node: status code}; absent = success) is not
    UnschedulableAndUnresolvable -- removing pods cannot fix such a node."""
    return [nn for nn in order if codes.get(nn, abi.CODE_SUCCESS) != abi.CODE_UNRESOLVABLE]


class GpuFramework:
    def __init__(self, profile, nodes, existing=(), cluster=None, pods_hint=(), device=0, create_engine=True,
                 shard=None, compiled=None):
        """shard=(rank, world): keep only this rank's contiguous slice of Snapshot.List() on the
        device (native.shard_range); join the communicator with init_comm before scheduling.
        compiled=(compiler, (snap, arrays, order)): a snapshot compiled elsewhere (a columnar
        generator such as cluster.sharded_spread_compiled, already sliced to this rank's shard);
        `nodes` may then be None (status reasons that name a node's taints need the node objects)."""
        self.profile = profile
        if compiled is None:
            self.compiler = Compiler(profile, cluster)
            self.compiler.register(nodes, existing, pods_hint)
            self.shard = None if shard is None else native.shard_range(len(nodes), shard[1], shard[0])
            self.snap, self.arrays, self.order = self.compiler.compile_snapshot(nodes, existing, shard=self.shard)
        else:
            self.compiler, (self.snap, self.arrays, self.order) = compiled
            n_total = len(self.order)
            self.shard = None if shard is None else native.shard_range(n_total, shard[1], shard[0])
            want = (0, n_total) if self.shard is None else self.shard
            if (self.snap.node_base, self.snap.n_nodes) != want:
                raise ValueError("compiled snapshot holds rows [%d, +%d), the shard is [%d, +%d)"
                                 % (self.snap.node_base, self.snap.n_nodes, want[0], want[1]))
        self.config = self.compiler.config(device)
        self.nodes = {api.name_of(n): n for n in nodes or ()}
        self.filters = [f for f in profile.filters if f in abi.FILTER_IDS]
        self.seq = 0
        # NodeInfo.Pods of every listed node, in order, with each pod's pod-table slot (snapshot pods
        # in compile order, then the pods this framework assumes); the potential victims of preemption
        self.node_pods = {}
        slot = 0
        for p in existing:
            nn = api.spec(p).get("nodeName", "") or ""
            if nn in self.nodes:
                self.node_pods.setdefault(nn, []).append((p, slot))
                slot += 1
        self.next_slot = slot
        self.nominated = []   # [(pod, node name)] -- framework.PodNominator, in nomination order
        self.engine = None
        if create_engine:
            self.engine = Engine(self.config)
            if getattr(profile, "run_all_filters", False):
                self.engine.set_option(abi.OPT_RUN_ALL_FILTERS, 1)
            self.engine.upload(self.snap, self.arrays)

    def init_comm(self, rank, world, uid):
        """Node sharding over RCCL (kgpu_comm_init): uid from native.comm_unique_id() on rank 0."""
        self.engine.comm_init(world, rank, uid)

    # ------------------------------------------------------------------ compile
    def compile_pods(self, pods):
        """Returns (queries, pools_ctypes, pools_np, errors) -- errors: {index: message}."""
        pools = Pools()
        qs, errors = [], {}
        for i, p in enumerate(pods):
            try:
                qs.append(self.compiler.compile_pod(p, pools))
            except CompileError as e:
                errors[i] = str(e)
                qs.append(np.zeros((), abi.QUERY))
        pc, pnp = pools.finalize()
        q = np.array(qs, dtype=abi.QUERY) if qs else np.zeros(0, abi.QUERY)
        return q, pc, pnp, errors

    # ------------------------------------------------------------------ reasons
    def reasons(self, pod, node_name, word, compiled=None, node=-1):
        h = self.engine.h if self.engine is not None else None
        return status_reasons(self.filters, self.compiler, self.nodes, pod, node_name, word, handle=h, node=node,
                              compiled=compiled)

    # ------------------------------------------------------------------ cycles
    def cycle(self, pod, assume=False, seq=None):
        """One diagnostic scheduling cycle (kgpu_schedule_one)."""
        q, pc, pnp, errors = self.compile_pods([pod])
        if errors:
            raise CompileError(errors[0])
        s = self.seq if seq is None else seq
        res, _ = self.engine.schedule_one(q[0], pc, seq=s, assume=assume)
        self.seq = s + 1
        n = self.snap.n_nodes
        words = self.engine.filter_words(n)
        run_all = getattr(self.profile, "run_all_filters", False)
        every = self.engine.filter_words_all(len(self.filters), n) if run_all else None
        statuses, plugin_statuses = {}, ({} if run_all else None)
        for i in np.nonzero(words)[0]:
            if int(words[i]) == abi.STATUS_NOT_EVALUATED:
                continue  # never examined: percentageOfNodesToScore stopped the search before it
            nm = self.order[self.snap.node_base + int(i)]
            if not run_all:
                statuses[nm] = self.reasons(pod, nm, int(words[i]), compiled=(q[0], pc), node=int(i))
                continue
            per = {}
            for p in range(len(self.filters)):
                wp = int(every[p, i])
                if wp:
                    code, plugin, rs = self.reasons(pod, nm, wp, compiled=(q[0], pc), node=int(i))
                    per[plugin] = (code, rs)
            plugin_statuses[nm] = per
            w = int(words[i])
            statuses[nm] = ((w >> 8) & 3, self.filters[(w & 0xFF) - 1], [r for _, rs in per.values() for r in rs])
        scores = {}
        feas = np.nonzero(words == 0)[0]
        for name, w in self.profile.scores:
            raw, norm = self.engine.scores(abi.SCORE_IDS[name], n)
            scores[name] = {self.order[self.snap.node_base + int(i)]: (int(raw[i]), int(norm[i])) for i in feas}
        host = self.order[res["node"]] if res["node"] >= 0 else None
        if assume and host is not None:
            self._placed(pod, host)
        return CycleResult(host, res, statuses, scores, plugin_statuses)

    def _placed(self, pod, host):
        """Record an assumed pod on its node (NodeInfo.AddPod) and drop it from the nominator
        (scheduler.assume, scheduler.go:448)."""
        placed = dict(pod)
        placed["spec"] = dict(api.spec(pod))
        placed["spec"]["nodeName"] = host
        self.node_pods.setdefault(host, []).append((placed, self.next_slot))
        self.next_slot += 1
        key = _pod_key(pod)
        self.nominated = [(p, n) for p, n in self.nominated if _pod_key(p) != key]

    def schedule(self, pods, first_seq=None, stats=None):
        """scheduleOne loop over pods; returns kgpu_result records (node index -1: FitError,
        -2: scoring error, -3: compile error)."""
        q, pc, pnp, errors = self.compile_pods(pods)
        s0 = self.seq if first_seq is None else first_seq
        out = np.zeros(len(pods), abi.RESULT)
        i = 0
        while i < len(pods):
            j = i
            while j < len(pods) and j not in errors:
                j += 1
            if j > i:
                res, stats = self.engine.schedule_batch(q[i:j], pc, first_seq=s0 + i, stats=stats)
                out[i:j] = res
                for k in range(i, j):
                    if out[k]["node"] >= 0:
                        self._placed(pods[k], self.order[out[k]["node"]])
            if j < len(pods):
                out[j]["node"] = -3
                j += 1
            i = j
        self.seq = s0 + len(pods)
        return out

    def host_of(self, node_index):
        return self.order[node_index] if node_index >= 0 else None

    # ------------------------------------------------------------------ nominated pods / preemption
    def set_nominated(self, nominated):
        """framework.PodNominator contents: [(pod, nominated node name)] in nomination order
        (kgpu_set_nominated).  Every later cycle filters those nodes twice (podPassesFiltersOnNode)."""
        self.nominated = list(nominated)
        q, pc, pnp, errors = self.compile_pods([p for p, _ in self.nominated])
        if errors:
            raise CompileError(errors[min(errors)])
        index = {nn: i for i, nn in enumerate(self.order)}
        noms = np.zeros(len(self.nominated), abi.NOMINATED)
        for i, (_, nn) in enumerate(self.nominated):
            noms[i] = (index[nn], i)
        self.engine.set_nominated(noms, q, pc)

    def select_nodes_for_preemption(self, pod, pdbs=(), now=0, nodes=None):
        """selectNodesForPreemption + pickOneNodeForPreemption (generic_scheduler.go:718-1012) on the
        device over `nodes` (default: every node).  Returns ({node name: (victim pods,
        numPDBViolations)} in Snapshot.List() order, the picked node name or "").

        A node outside `nodes` gets no potential victims, so the engine re-filters it as it stands --
        it failed this cycle's filters, so it fails again and is never a candidate: the result is the
        reference's selection over potentialNodes only (generic_scheduler.go:279-289)."""
        prio = _priority(pod)
        keep = None if nodes is None else set(nodes)
        cand = []
        for nn in self.order:
            if keep is not None and nn not in keep:
                continue
            for p, slot in self.node_pods.get(nn, []):
                if _priority(p) < prio:
                    cand.append((nn, p, slot))
        q, pc, pnp, errors = self.compile_pods([pod] + [p for _, p, _ in cand])
        if errors:
            raise CompileError(errors[min(errors)])
        index = {nn: i for i, nn in enumerate(self.order)}
        # Preempt passes every PDB of the cluster; filterPodsWithPDBViolation only touches those that
        # select a potential victim, in order: the engine gets that subset, renumbered (64-bit masks)
        sel = [_pdbs_of(p, pdbs) for _, p, _ in cand]
        used = sorted({j for js in sel for j in js})
        if len(used) > 64:
            raise ValueError("%d PodDisruptionBudgets select potential victims (the engine takes 64)" % len(used))
        renum = {j: k for k, j in enumerate(used)}
        vic = np.zeros(len(cand), abi.VICTIM)
        for i, (nn, p, slot) in enumerate(cand):
            m = 0
            for j in sel[i]:
                m |= 1 << renum[j]
            vic[i] = (index[nn], slot, i, 0, _start_time(p, now), m)
        allowed = np.array([int(pdbs[j].get("disruptionsAllowed", 0)) for j in used], np.int32)
        out, vout, chosen = self.engine.select_victims(q[0], pc, vic, q[1:], allowed, self.snap.n_nodes)
        res = {}
        for n in range(self.snap.n_nodes):
            o = out[n]
            if not o["fits"]:
                continue
            nn = self.order[self.snap.node_base + n]
            vs = [cand[int(vout[o["first"] + k])][1] for k in range(o["n_victims"])]
            res[nn] = (vs, int(o["num_pdb_violations"]))
        return res, (self.order[chosen] if chosen >= 0 else "")

    def preempt(self, pod, statuses, pdbs=(), now=0, extenders=()):
        """genericScheduler.Preempt (generic_scheduler.go:252-315) after a FitError whose per-node
        statuses are `statuses` ({node: (code, plugin, reasons)}, CycleResult.statuses).
        extenders: the profile's scheduler extenders, objects with supports_preemption() /
        is_interested(pod) / is_ignorable() / process_preemption(pod, {node: (victims,
        numPDBViolations)}, node_of) (processPreemptionWithExtenders, :317-351).
        Returns (node name or "", victim pods, nominated pods whose nomination is cleared)."""
        if not self._eligible_to_preempt(pod):
            return "", [], []
        potential = nodes_where_preemption_might_help(
            self.order, {nn: st[0] for nn, st in statuses.items() if st})
        if not potential:
            return "", [], [pod]
        n2v, node = self.select_nodes_for_preemption(pod, pdbs, now, nodes=potential)
        if extenders and n2v:
            n2v = process_preemption_with_extenders(pod, n2v, extenders, self.nodes.get)
            node = pick_one_node_for_preemption(n2v, now, self.order)
        if not node:
            return "", [], []
        prio = _priority(pod)
        lower = [p for p, nn in self.nominated if nn == node and _priority(p) < prio]
        return node, n2v[node][0], lower

    def _eligible_to_preempt(self, pod):
        """podEligibleToPreemptOthers (generic_scheduler.go:1030-1056)."""
        if api.spec(pod).get("preemptionPolicy") == "Never":
            return False
        nom = (pod.get("status") or {}).get("nominatedNodeName") or ""
        if nom and nom in self.nodes:
            prio = _priority(pod)
            for p, _ in self.node_pods.get(nom, []):
                if api.meta(p).get("deletionTimestamp") is not None and _priority(p) < prio:
                    return False
        return True


def process_preemption_with_extenders(pod, n2v, extenders, node_of):
    """processPreemptionWithExtenders (generic_scheduler.go:317-351): each extender that supports
    preemption and is interested in the pod replaces the candidate map in turn; an ignorable
    extender's error is skipped, any other is raised; an empty map ends the walk."""
    for ext in extenders:
        if not (ext.supports_preemption() and ext.is_interested(pod)):
            continue
        try:
            new = ext.process_preemption(pod, n2v, node_of)
        except Exception:
            if ext.is_ignorable():
                continue
            raise
        n2v = new
        if not n2v:
            break
    return n2v


def pick_one_node_for_preemption(n2v, now, order):
    """pickOneNodeForPreemption (generic_scheduler.go:718-843) on the host over an extender-edited
    candidate map ({node: (victim pods, numPDBViolations)}), walked in Snapshot.List() order: the
    device's own pick (kgpu_select_victims) covers the map before any extender edits it."""
    if not n2v:
        return ""
    max_i32 = (1 << 31) - 1
    rank = {nn: i for i, nn in enumerate(order)}
    nodes = sorted(n2v, key=lambda nn: rank.get(nn, len(rank)))
    for nn in nodes:
        if not n2v[nn][0]:
            return nn
    lo = min(n2v[nn][1] for nn in nodes)
    cand = [nn for nn in nodes if n2v[nn][1] == lo]
    # victims are sorted MoreImportantPod first: the first one has the highest priority
    for key in (lambda nn: _priority(n2v[nn][0][0]),
                lambda nn: sum(_priority(p) + max_i32 + 1 for p in n2v[nn][0]),
                lambda nn: len(n2v[nn][0])):
        if len(cand) == 1:
            return cand[0]
        lo = min(key(nn) for nn in cand)
        cand = [nn for nn in cand if key(nn) == lo]
    if len(cand) == 1:
        return cand[0]
    # the latest "earliest start time" among the victims of each node (GetEarliestPodStartTime)
    def earliest(nn):
        vs = n2v[nn][0]
        hp = max(_priority(p) for p in vs)
        return min(_start_time(p, now) for p in vs if _priority(p) == hp)
    best = cand[0]
    for nn in cand[1:]:
        if earliest(nn) > earliest(best):
            best = nn
    return best


def _pod_key(pod):
    return api.meta(pod).get("uid", "") or "%s/%s" % (api.ns_of(pod), api.name_of(pod))


def _priority(pod):
    """podutil.GetPodPriority."""
    p = api.spec(pod).get("priority")
    return 0 if p is None else int(p)


def _start_time(pod, now):
    """util.GetPodStartTime (utils.go:38-44) in ns; pods that have not started: `now`."""
    import datetime
    s = (pod.get("status") or {}).get("startTime")
    if s is None:
        return now
    if not isinstance(s, str):
        return int(s)
    t = datetime.datetime.strptime(s.replace("Z", "+0000"), "%Y-%m-%dT%H:%M:%S%z")
    return int(t.timestamp()) * 1_000_000_000


def _pdbs_of(pod, pdbs):
    """Indices of the PodDisruptionBudgets selecting the pod, in order."""
    m = _pdb_mask(pod, pdbs)
    return [j for j in range(len(pdbs)) if (m >> j) & 1]


def _pdb_mask(pod, pdbs):
    """PodDisruptionBudgets selecting the pod (filterPodsWithPDBViolation, generic_scheduler.go:878-919):
    same namespace, a non-empty selector matching the pod's labels; label-less pods match none.
    A Python int: bit j for PDB j, any number of PDBs."""
    from .compile import label_selector_matches
    labels = api.labels_of(pod)
    m = 0
    if not labels:
        return 0
    for j, b in enumerate(pdbs):
        if (b.get("namespace", "") or "") != api.ns_of(pod):
            continue
        sel = b.get("selector")
        if sel is None or (not (sel.get("matchLabels") or {}) and not (sel.get("matchExpressions") or [])):
            continue  # Selector.Empty(): matches nothing
        if any(e.get("operator") not in ("In", "NotIn", "Exists", "DoesNotExist") for e in sel.get("matchExpressions") or []):
            continue  # LabelSelectorAsSelector error: the PDB is skipped
        if label_selector_matches(sel, labels):
            m |= 1 << j
    return m

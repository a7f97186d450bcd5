"""ORACLE (test infrastructure only) -- nominated-pod two-pass filter and preemption.

Follows:
  pkg/scheduler/core/generic_scheduler.go:526-551   addNominatedPods
  pkg/scheduler/core/generic_scheduler.go:553-615   podPassesFiltersOnNode (two passes)
  pkg/scheduler/core/generic_scheduler.go:252-315   Preempt
  pkg/scheduler/core/generic_scheduler.go:335-355   getLowerPriorityNominatedPods
  pkg/scheduler/core/generic_scheduler.go:718-843   pickOneNodeForPreemption
  pkg/scheduler/core/generic_scheduler.go:845-876   selectNodesForPreemption
  pkg/scheduler/core/generic_scheduler.go:878-919   filterPodsWithPDBViolation
  pkg/scheduler/core/generic_scheduler.go:921-1012  selectVictimsOnNode
  pkg/scheduler/core/generic_scheduler.go:1014-1028 nodesWherePreemptionMightHelp
  pkg/scheduler/core/generic_scheduler.go:1030-1056 podEligibleToPreemptOthers
  pkg/scheduler/util/utils.go:38-83                  GetPodStartTime, GetEarliestPodStartTime,
                                                     MoreImportantPod
  pkg/scheduler/internal/queue/scheduling_queue.go   nominatedPodMap (add / delete / podsForNode)

Determinism contract: the reference builds nodeNameToVictims in a map and walks it in
Go's random map order, so pickOneNodeForPreemption's "first node" among ties (and the early return
for a node without victims) is not reproducible; this restatement walks candidate nodes in
Snapshot.List() order, the rule the HIP path implements.  sort.Slice of the potential victims is
stable here (Go 1.13 uses insertion sort for up to 12 elements, which is stable; longer lists of
equally important pods have no defined order in the reference).
"""
import copy
import datetime

from . import labels as L
from . import nodeinfo as NI
from . import plugins as P

MAX_INT32 = 2 ** 31 - 1


def pod_priority(pod):
    """podutil.GetPodPriority: spec.priority, 0 when unset."""
    p = (pod.get("spec") or {}).get("priority")
    return 0 if p is None else int(p)


def _parse_time(s):
    t = datetime.datetime.strptime(s.replace("Z", "+0000"), "%Y-%m-%dT%H:%M:%S%z")
    return int(t.timestamp()) * 1_000_000_000


def pod_start_time(pod, now):
    """utils.go:38-44 GetPodStartTime: status.startTime, else time.Now() (`now`, ns)."""
    s = (pod.get("status") or {}).get("startTime")
    return now if s is None else (_parse_time(s) if isinstance(s, str) else int(s))


def more_important_pod(p1, p2, now):
    """utils.go:76-83."""
    a, b = pod_priority(p1), pod_priority(p2)
    if a != b:
        return a > b
    return pod_start_time(p1, now) < pod_start_time(p2, now)


def earliest_pod_start_time(victims, now):
    """utils.go:48-70 GetEarliestPodStartTime over victims.Pods in list order."""
    if not victims:
        return None
    earliest = pod_start_time(victims[0], now)
    maxp = pod_priority(victims[0])
    for p in victims:
        pr = pod_priority(p)
        if pr == maxp:
            if pod_start_time(p, now) < earliest:
                earliest = pod_start_time(p, now)
        elif pr > maxp:
            maxp = pr
            earliest = pod_start_time(p, now)
    return earliest


class Nominator:
    """framework.PodNominator backed by nominatedPodMap (scheduling_queue.go): pods nominated to a
    node, in nomination order; re-nominating a pod (by UID) moves it."""

    def __init__(self):
        self.by_node = {}
        self.node_of = {}

    def add(self, pod, node_name):
        self.delete(pod)
        uid = NI.pod_key(pod)
        self.node_of[uid] = node_name
        self.by_node.setdefault(node_name, []).append(pod)

    def delete(self, pod):
        uid = NI.pod_key(pod)
        nn = self.node_of.pop(uid, None)
        if nn is None:
            return
        lst = [p for p in self.by_node.get(nn, []) if NI.pod_key(p) != uid]
        if lst:
            self.by_node[nn] = lst
        else:
            self.by_node.pop(nn, None)

    def pods_for_node(self, node_name):
        return list(self.by_node.get(node_name, []))


# ------------------------------------------------------------------ cycle-state / NodeInfo clones
def clone_state(state):
    """CycleState.Clone (cycle_state.go:76-88): every plugin state's Clone().  The PTS and IPA
    states deep-copy the maps AddPod / RemovePod mutate."""
    out = dict(state)
    s = state.get("PreFilterPodTopologySpread")
    if s is not None:
        paths = {}
        for k, cp in s["paths"].items():
            n = P.CriticalPaths()
            n.p = [list(cp.p[0]), list(cp.p[1])]
            paths[k] = n
        out["PreFilterPodTopologySpread"] = {"constraints": s["constraints"], "pairs": dict(s["pairs"]),
                                             "paths": paths}
    s = state.get("PreFilterInterPodAffinity")
    if s is not None:
        out["PreFilterInterPodAffinity"] = {"existing_anti": dict(s["existing_anti"]), "aff": dict(s["aff"]),
                                            "anti": dict(s["anti"]), "pi": s["pi"]}
    return out


def clone_node_info(ni):
    """NodeInfo.Clone (types.go:407-444)."""
    out = NI.NodeInfo()
    out.node = ni.node
    out.pods = list(ni.pods)
    out.pods_with_affinity = list(ni.pods_with_affinity)
    out.used_ports = {ip: set(s) for ip, s in ni.used_ports.items()}
    out.requested = copy.deepcopy(ni.requested)
    out.non_zero = copy.deepcopy(ni.non_zero)
    out.allocatable = ni.allocatable
    out.image_states = ni.image_states
    return out


def run_prefilter_extension_add_pod(fw, state, pod, pod_to_add, ni):
    """framework.go:391-411 RunPreFilterExtensionAddPod over the PreFilter plugins with extensions."""
    for pl in fw.prefilters:
        if hasattr(pl, "add_pod"):
            pl.add_pod(state, pod, pod_to_add, ni)


def run_prefilter_extension_remove_pod(fw, state, pod, pod_to_remove, ni):
    """framework.go:413-433 RunPreFilterExtensionRemovePod."""
    for pl in fw.prefilters:
        if hasattr(pl, "remove_pod"):
            pl.remove_pod(state, pod, pod_to_remove, ni)


# ------------------------------------------------------------------ two-pass filter
def add_nominated_pods(fw, nominator, pod, state, ni):
    """generic_scheduler.go:526-551.  Returns (pods_added, state, node_info)."""
    if nominator is None or ni is None or ni.node is None:
        return False, state, ni
    noms = nominator.pods_for_node(NI.name(ni.node))
    if not noms:
        return False, state, ni
    ni_out = clone_node_info(ni)
    st_out = clone_state(state)
    added = False
    for p in noms:
        if pod_priority(p) >= pod_priority(pod) and NI.pod_key(p) != NI.pod_key(pod):
            ni_out.add_pod(p)
            run_prefilter_extension_add_pod(fw, st_out, pod, p, ni_out)
            added = True
    return added, st_out, ni_out


def pod_passes_filters_on_node(fw, nominator, state, pod, ni):
    """generic_scheduler.go:553-615.  Returns (fits, plugin, status); an Error status raises."""
    status, plugin = None, None
    added = False
    for i in range(2):
        st_use, ni_use = state, ni
        if i == 0:
            added, st_use, ni_use = add_nominated_pods(fw, nominator, pod, state, ni)
        elif not added or status is not None:
            break
        plugin, status = fw.run_filters(st_use, pod, ni_use)
        if status is not None and status.code == P.ERROR:
            from .framework import ScheduleError
            raise ScheduleError(repr(status))
    return status is None, plugin, status


# ------------------------------------------------------------------ preemption
def nodes_where_preemption_might_help(nodes, statuses):
    """generic_scheduler.go:1014-1028: every node whose status is not UnschedulableAndUnresolvable
    (a node with no status -- not evaluated -- qualifies)."""
    out = []
    for ni in nodes:
        st = statuses.get(NI.name(ni.node))
        code = st[1].code if isinstance(st, tuple) else (st.code if st is not None else P.SUCCESS)
        if code == P.UNRESOLVABLE:
            continue
        out.append(ni)
    return out


def pod_eligible_to_preempt_others(pod, snapshot):
    """generic_scheduler.go:1030-1056."""
    if (pod.get("spec") or {}).get("preemptionPolicy") == "Never":
        return False
    nom = (pod.get("status") or {}).get("nominatedNodeName") or ""
    if nom and nom in snapshot.map:
        pp = pod_priority(pod)
        for pi in snapshot.map[nom].pods:
            if (pi.pod.get("metadata") or {}).get("deletionTimestamp") is not None and pod_priority(pi.pod) < pp:
                return False
    return True


def filter_pods_with_pdb_violation(pods, pdbs):
    """generic_scheduler.go:878-919 (stable: preserves the order of `pods`).  pdbs: list of
    {"namespace", "selector" (LabelSelector), "disruptionsAllowed"}."""
    allowed = [int(p.get("disruptionsAllowed", 0)) for p in pdbs]
    violating, non_violating = [], []
    for pod in pods:
        violated = False
        plabels = NI.labels_of(pod)
        if len(plabels) != 0:
            for i, pdb in enumerate(pdbs):
                if pdb.get("namespace", "") != NI.namespace(pod):
                    continue
                try:
                    sel = L.label_selector_as_selector(pdb.get("selector"))
                except L.SelectorError:
                    continue
                if sel.empty() or not sel.matches(plabels):
                    continue
                if allowed[i] <= 0:
                    violated = True
                    break
                allowed[i] -= 1
        (violating if violated else non_violating).append(pod)
    return violating, non_violating


def select_victims_on_node(fw, nominator, state, pod, ni, pdbs, now):
    """generic_scheduler.go:921-1012 on a cloned state / NodeInfo.  Returns (victims,
    num_pdb_violations, fits)."""
    pp = pod_priority(pod)
    potential = []
    # the reference ranges over nodeInfo.Pods while RemovePod swap-deletes from it; every original
    # element is still visited once, in the original order
    for pi in list(ni.pods):
        if pod_priority(pi.pod) < pp:
            potential.append(pi.pod)
            ni.remove_pod(pi.pod)
            run_prefilter_extension_remove_pod(fw, state, pod, pi.pod, ni)
    fits, _, _ = pod_passes_filters_on_node(fw, nominator, state, pod, ni)
    if not fits:
        return None, 0, False
    # sort.Slice(potentialVictims, MoreImportantPod) -- stable here (module docstring)
    import functools
    potential.sort(key=functools.cmp_to_key(
        lambda a, b: -1 if more_important_pod(a, b, now) else (1 if more_important_pod(b, a, now) else 0)))
    violating, non_violating = filter_pods_with_pdb_violation(potential, pdbs)
    victims = []
    n_viol = 0

    def reprieve(p):
        ni.add_pod(p)
        run_prefilter_extension_add_pod(fw, state, pod, p, ni)
        ok, _, _ = pod_passes_filters_on_node(fw, nominator, state, pod, ni)
        if not ok:
            ni.remove_pod(p)
            run_prefilter_extension_remove_pod(fw, state, pod, p, ni)
            victims.append(p)
        return ok

    for p in violating:
        if not reprieve(p):
            n_viol += 1
    for p in non_violating:
        reprieve(p)
    return victims, n_viol, True


def select_nodes_for_preemption(fw, nominator, state, pod, potential_nodes, pdbs, now):
    """generic_scheduler.go:845-876: {node name: (victims, num_pdb_violations)} for the nodes where
    the pod fits after preemption, in potential_nodes order."""
    out = {}
    for ni in potential_nodes:
        v, nv, fits = select_victims_on_node(fw, nominator, clone_state(state), pod, clone_node_info(ni), pdbs, now)
        if fits:
            out[NI.name(ni.node)] = (v, nv)
    return out


def pick_one_node_for_preemption(nodes_to_victims, now):
    """generic_scheduler.go:718-843, walking nodes_to_victims in insertion (Snapshot.List()) order."""
    if not nodes_to_victims:
        return ""
    min_pdb = MAX_INT32
    min1 = []
    for node, (victims, nv) in nodes_to_victims.items():
        if len(victims) == 0:
            return node
        if nv < min_pdb:
            min_pdb = nv
            min1 = []
        if nv == min_pdb:
            min1.append(node)
    if len(min1) == 1:
        return min1[0]
    min_hp = MAX_INT32
    min2 = []
    for node in min1:
        hp = pod_priority(nodes_to_victims[node][0][0])
        if hp < min_hp:
            min_hp = hp
            min2 = []
        if hp == min_hp:
            min2.append(node)
    if len(min2) == 1:
        return min2[0]
    min_sum = 2 ** 63 - 1
    min1 = []
    for node in min2:
        s = sum(pod_priority(p) + MAX_INT32 + 1 for p in nodes_to_victims[node][0])
        if s < min_sum:
            min_sum = s
            min1 = []
        if s == min_sum:
            min1.append(node)
    if len(min1) == 1:
        return min1[0]
    min_pods = MAX_INT32
    min2 = []
    for node in min1:
        n = len(nodes_to_victims[node][0])
        if n < min_pods:
            min_pods = n
            min2 = []
        if n == min_pods:
            min2.append(node)
    if len(min2) == 1:
        return min2[0]
    latest = earliest_pod_start_time(nodes_to_victims[min2[0]][0], now)
    ret = min2[0]
    for node in min2[1:]:
        t = earliest_pod_start_time(nodes_to_victims[node][0], now)
        if t > latest:
            latest, ret = t, node
    return ret


def lower_priority_nominated_pods(nominator, pod, node_name):
    """generic_scheduler.go:335-355."""
    if nominator is None:
        return []
    pp = pod_priority(pod)
    return [p for p in nominator.pods_for_node(node_name) if pod_priority(p) < pp]


def process_preemption_with_extenders(pod, n2v, extenders, node_of):
    """generic_scheduler.go:317-351: every extender that supports preemption and is interested in the
    pod narrows (or extends) the candidates in turn; an ignorable extender's error is skipped, any
    other aborts Preempt.  extenders: objects with supports_preemption / is_interested /
    is_ignorable / process_preemption(pod, n2v, node_of) (tests/fake_plugins.FakeExtender)."""
    if not n2v:
        return n2v
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


def preempt(gs, pod, fit_error, pdbs=(), nominator=None, now=0, extenders=()):
    """generic_scheduler.go:252-315 Preempt.  Returns (node, victims, nominated pods to clear); node
    "" when preemption cannot help."""
    from .framework import FitError, ScheduleError
    if not isinstance(fit_error, FitError):
        return "", [], []
    snap = gs.fw.handle.snapshot
    if not pod_eligible_to_preempt_others(pod, snap):
        return "", [], []
    if len(snap.list) == 0:
        raise ScheduleError("no nodes available to schedule pods")
    potential = nodes_where_preemption_might_help(snap.list, fit_error.statuses)
    if not potential:
        return "", [], [pod]
    state = {}
    st = gs.fw.run_prefilter(state, pod)
    if st is not None:
        raise ScheduleError(repr(st))
    n2v = select_nodes_for_preemption(gs.fw, nominator, state, pod, potential, list(pdbs), now)
    n2v = process_preemption_with_extenders(pod, n2v, extenders, lambda nn: snap.map[nn].node)
    cand = pick_one_node_for_preemption(n2v, now)
    if not cand:
        return "", [], []
    return cand, n2v[cand][0], lower_priority_nominated_pods(nominator, pod, cand)

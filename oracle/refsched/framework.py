"""ORACLE (test infrastructure only) -- framework runner + generic scheduler restatement.

Follows:
  pkg/scheduler/framework/v1alpha1/framework.go:369-389  RunPreFilterPlugins
  pkg/scheduler/framework/v1alpha1/framework.go:477-502  RunFilterPlugins (early exit)
  pkg/scheduler/framework/v1alpha1/framework.go:543-563  RunPreScorePlugins
  pkg/scheduler/framework/v1alpha1/framework.go:579-656  RunScorePlugins (score, normalize,
                                                         [0,100] check, weights)
  pkg/scheduler/framework/v1alpha1/interface.go:158-191  PluginToStatus.Merge
  pkg/scheduler/core/generic_scheduler.go:146-238,379-495,565-716  Schedule, selectHost,
                                                         numFeasibleNodesToFind, filters, prioritize
  pkg/scheduler/algorithmprovider/registry.go:77-172     default / ClusterAutoscaler profiles
  pkg/scheduler/scheduler.go:509-593                     scheduleOne -> assume

Determinism contract: the reference appends feasible nodes through an atomic
counter from 16 goroutines and breaks score ties with math/rand reservoir sampling, so its
placements are not reproducible.  This restatement scans nodes in Snapshot.List() order and
breaks ties with the deterministic packed key of tiebreak.py -- the same contract the HIP
path implements.
"""
from . import nodeinfo as NI
from . import plugins as P
from . import tiebreak

MAX_TOTAL_SCORE = 2 ** 63 - 1
MIN_FEASIBLE_NODES_TO_FIND = 100
MIN_FEASIBLE_NODES_PERCENTAGE_TO_FIND = 5

DEFAULT_FILTERS = ["NodeUnschedulable", "NodeResourcesFit", "NodeName", "NodePorts", "NodeAffinity",
                   "VolumeRestrictions", "TaintToleration", "EBSLimits", "GCEPDLimits",
                   "NodeVolumeLimits", "AzureDiskLimits", "VolumeBinding", "VolumeZone",
                   "PodTopologySpread", "InterPodAffinity"]
DEFAULT_PREFILTERS = ["NodeResourcesFit", "NodePorts", "PodTopologySpread", "InterPodAffinity"]
DEFAULT_PRESCORES = ["InterPodAffinity", "PodTopologySpread", "DefaultPodTopologySpread", "TaintToleration"]
DEFAULT_SCORES = [("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1), ("InterPodAffinity", 1),
                  ("NodeResourcesLeastAllocated", 1), ("NodeAffinity", 1), ("NodePreferAvoidPods", 10000),
                  ("PodTopologySpread", 2), ("DefaultPodTopologySpread", 1), ("TaintToleration", 1)]
# volume plugins return Success for volume-less pods; they are modelled as no-ops.
VOLUME_FILTERS = {"VolumeRestrictions", "EBSLimits", "GCEPDLimits", "NodeVolumeLimits", "AzureDiskLimits",
                  "VolumeBinding", "VolumeZone"}


class Profile:
    def __init__(self, filters=None, prefilters=None, prescores=None, scores=None,
                 least_resources=(("cpu", 1), ("memory", 1)), most_resources=(("cpu", 1), ("memory", 1)),
                 hard_pod_affinity_weight=1, ignored_resources=(), pts_default_constraints=(),
                 percentage_of_nodes_to_score=100, tie_break_mode=tiebreak.MODE_HASH, seed=0x7B,
                 plugin_factories=None, run_all_filters=False):
        self.filters = list(DEFAULT_FILTERS if filters is None else filters)
        self.prefilters = list(DEFAULT_PREFILTERS if prefilters is None else prefilters)
        self.prescores = list(DEFAULT_PRESCORES if prescores is None else prescores)
        self.scores = list(DEFAULT_SCORES if scores is None else scores)
        self.least_resources = list(least_resources)
        self.most_resources = list(most_resources)
        self.hard_pod_affinity_weight = hard_pod_affinity_weight
        self.ignored_resources = list(ignored_resources)
        self.pts_default_constraints = list(pts_default_constraints)
        self.percentage_of_nodes_to_score = percentage_of_nodes_to_score
        self.tie_break_mode = tie_break_mode
        self.seed = seed
        # extra plugin constructors, name -> factory(handle): the fake plugins of the reference's
        # generic_scheduler_test.go (tests/fake_plugins.py)
        self.plugin_factories = dict(plugin_factories or {})
        # WithRunAllFilters (framework.go:155-160), set from the legacy Policy's AlwaysCheckAllPredicates
        # (factory.go:107,278-281)
        self.run_all_filters = bool(run_all_filters)


def cluster_autoscaler_profile(**kw):
    scores = [("NodeResourcesMostAllocated" if n == "NodeResourcesLeastAllocated" else n, w)
              for n, w in DEFAULT_SCORES]
    return Profile(scores=scores, **kw)


class Handle:
    """FrameworkHandle: snapshot lister + informer-backed listers used by DefaultSelector."""

    def __init__(self, snapshot, services=(), rcs=(), rss=(), sss=(), pvcs=()):
        self.snapshot = snapshot
        self.services, self.rcs, self.rss, self.sss = list(services), list(rcs), list(rss), list(sss)
        self.pvcs = list(pvcs)


class ScheduleError(Exception):
    pass


class FitError(ScheduleError):
    def __init__(self, statuses):
        super().__init__("0/%d nodes are available" % len(statuses))
        self.statuses = statuses


class Framework:
    def __init__(self, profile, handle):
        self.profile = profile
        self.handle = handle
        h = handle
        reg = {
            "NodeUnschedulable": lambda: P.NodeUnschedulable(),
            "NodeName": lambda: P.NodeName(),
            "NodePorts": lambda: P.NodePorts(),
            "NodeResourcesFit": lambda: P.Fit(profile.ignored_resources),
            "NodeResourcesLeastAllocated": lambda: P.LeastAllocated(h, profile.least_resources),
            "NodeResourcesMostAllocated": lambda: P.MostAllocated(h, profile.most_resources),
            "NodeResourcesBalancedAllocation": lambda: P.BalancedAllocation(h),
            "TaintToleration": lambda: P.TaintToleration(h),
            "NodeAffinity": lambda: P.NodeAffinity(h),
            "ImageLocality": lambda: P.ImageLocality(h),
            "NodePreferAvoidPods": lambda: P.NodePreferAvoidPods(h),
            "PodTopologySpread": lambda: P.PodTopologySpread(h, profile.pts_default_constraints),
            "DefaultPodTopologySpread": lambda: P.DefaultPodTopologySpread(h),
            "InterPodAffinity": lambda: P.InterPodAffinity(h, profile.hard_pod_affinity_weight),
        }
        for n, f in profile.plugin_factories.items():
            reg[n] = (lambda f: lambda: f(h))(f)
        self.plugins = {}

        def get(n):
            if n not in self.plugins:
                self.plugins[n] = reg[n]()
            return self.plugins[n]

        self.filters = [get(n) for n in profile.filters if n not in VOLUME_FILTERS]
        self.prefilters = [get(n) for n in profile.prefilters]
        self.prescores = [get(n) for n in profile.prescores]
        self.scores = []
        total = 0
        for n, w in profile.scores:
            w = w or 1
            if w * P.MAX_NODE_SCORE > MAX_TOTAL_SCORE - total:
                raise ValueError("total score of Score plugins could overflow")
            total += w * P.MAX_NODE_SCORE
            self.scores.append((get(n), w))

    # ---------------------------------------------------------------- runner
    def run_prefilter(self, state, pod):
        for pl in self.prefilters:
            st = pl.prefilter(state, pod)
            if not P.is_success(st):
                if st.code in (P.UNSCHEDULABLE, P.UNRESOLVABLE):
                    return P.Status(st.code, 'rejected by "%s" at prefilter' % pl.name)
                return P.Status(P.ERROR, "error while running %s prefilter" % pl.name)
        return None

    def run_filters(self, state, pod, ni):
        """Returns (plugin_name or None, status): RunFilterPlugins + PluginToStatus.Merge.  Without
        runAllFilters the first failure (early exit); with it the Merge of every failing plugin's
        status, named after the first (merge_statuses)."""
        if self.profile.run_all_filters:
            statuses = self.run_filter_plugins(state, pod, ni, run_all_filters=True)
            if not statuses:
                return None, None
            return next(iter(statuses)), merge_statuses(statuses)
        for pl in self.filters:
            st = pl.filter(state, pod, ni)
            if not P.is_success(st):
                if st.code not in (P.UNSCHEDULABLE, P.UNRESOLVABLE):
                    return pl.name, P.Status(P.ERROR, "running %s filter plugin: %r" % (pl.name, st.reasons))
                return pl.name, st
        return None, None

    def run_filter_plugins(self, state, pod, ni, run_all_filters=False):
        """framework.go:477-502 RunFilterPlugins: PluginToStatus {plugin name: Status}, the first
        non-Unschedulable failure becoming the only entry, as an Error."""
        statuses = {}
        for pl in self.filters:
            st = pl.filter(state, pod, ni)
            if P.is_success(st):
                continue
            if st.code not in (P.UNSCHEDULABLE, P.UNRESOLVABLE):
                return {pl.name: P.Status(P.ERROR, 'running "%s" filter plugin for pod "%s": %s'
                                          % (pl.name, NI.name(pod), ", ".join(st.reasons)))}
            statuses[pl.name] = st
            if not run_all_filters:
                return statuses
        return statuses

    def run_score_plugins(self, state, pod, nodes):
        """framework.go:579-656 RunScorePlugins: ({plugin: [[node, score], ...]}, None) or (None, Error status)."""
        out = {}
        for pl, _ in self.scores:
            lst = []
            for n in nodes:
                sc, st = pl.score(state, pod, NI.name(n))
                if not P.is_success(st):
                    return None, P.Status(P.ERROR, 'error while running score plugin for pod "%s": %s'
                                          % (NI.name(pod), ", ".join(st.reasons)))
                lst.append([NI.name(n), sc])
            out[pl.name] = lst
        for pl, _ in self.scores:
            if hasattr(pl, "normalize"):
                st = pl.normalize(state, pod, out[pl.name])
                if not P.is_success(st):
                    return None, P.Status(P.ERROR, 'error while running normalize score plugin for pod "%s": '
                                          'normalize score plugin "%s" failed with error %s'
                                          % (NI.name(pod), pl.name, ", ".join(st.reasons)))
        for pl, w in self.scores:
            for sc in out[pl.name]:
                if sc[1] > P.MAX_NODE_SCORE or sc[1] < P.MIN_NODE_SCORE:
                    return None, P.Status(P.ERROR, 'error while applying score defaultWeights for pod "%s": score '
                                          'plugin "%s" returns an invalid score %d, it should in the range of '
                                          '[%d, %d] after normalizing' % (NI.name(pod), pl.name, sc[1],
                                                                          P.MIN_NODE_SCORE, P.MAX_NODE_SCORE))
                sc[1] = sc[1] * w
        return out, None

    def run_prescore(self, state, pod, nodes):
        for pl in self.prescores:
            st = pl.prescore(state, pod, nodes)
            if not P.is_success(st):
                return P.Status(P.ERROR, "error while running %s prescore plugin" % pl.name)
        return None

    def run_scores(self, state, pod, nodes):
        """Returns {plugin name: [[node name, score], ...]} after normalize and weights."""
        out = {}
        for pl, w in self.scores:
            lst = []
            for n in nodes:
                s, st = pl.score(state, pod, NI.name(n))
                if not P.is_success(st):
                    # framework.go:603-607 -> generic_scheduler.go:640-642
                    raise ScheduleError('error while running score plugin for pod "%s": %s'
                                        % (NI.name(pod), "; ".join(st.reasons)))
                lst.append([NI.name(n), s])
            out[pl.name] = lst
        for pl, w in self.scores:
            if hasattr(pl, "normalize"):
                st = pl.normalize(state, pod, out[pl.name])
                if not P.is_success(st):
                    raise ScheduleError("normalize %s: %r" % (pl.name, st))
        for pl, w in self.scores:
            for sc in out[pl.name]:
                if sc[1] > P.MAX_NODE_SCORE or sc[1] < P.MIN_NODE_SCORE:
                    raise ScheduleError("score plugin %s returns an invalid score %d" % (pl.name, sc[1]))
                sc[1] = sc[1] * w
        return out


def merge_statuses(statuses):
    """PluginToStatus.Merge (framework/v1alpha1/interface.go:161-191): precedence Error >
    UnschedulableAndUnresolvable > Unschedulable, every reason appended (Go iterates the map in
    random order; here in plugin order)."""
    if not statuses:
        return None
    final = P.Status(P.SUCCESS)
    codes = set()
    for st in statuses.values():
        codes.add(st.code)
        final.code = st.code
        final.reasons.extend(st.reasons)
    for c in (P.ERROR, P.UNRESOLVABLE, P.UNSCHEDULABLE):
        if c in codes:
            final.code = c
            break
    return final


class Result:
    def __init__(self, host=None, host_index=-1, evaluated=0, feasible=0, statuses=None, scores=None,
                 totals=None, feasible_names=None):
        self.host, self.host_index = host, host_index
        self.evaluated, self.feasible = evaluated, feasible
        self.statuses = statuses or {}
        self.scores = scores or {}
        self.totals = totals or []
        self.feasible_names = feasible_names or []


class GenericScheduler:
    """core/generic_scheduler.go with the determinism contract described above."""

    def __init__(self, fw, nominator=None):
        self.fw = fw
        self.next_start = 0
        self.nominator = nominator  # framework.PodNominator (preemption.Nominator), None: no pods nominated

    def num_feasible_nodes_to_find(self, n):
        pct = self.fw.profile.percentage_of_nodes_to_score
        if n < MIN_FEASIBLE_NODES_TO_FIND or pct >= 100:
            return n
        adaptive = pct
        if adaptive <= 0:
            adaptive = 50 - n // 125
            if adaptive < MIN_FEASIBLE_NODES_PERCENTAGE_TO_FIND:
                adaptive = MIN_FEASIBLE_NODES_PERCENTAGE_TO_FIND
        num = n * adaptive // 100
        if num < MIN_FEASIBLE_NODES_TO_FIND:
            return MIN_FEASIBLE_NODES_TO_FIND
        return num

    def schedule(self, pod, pod_seq):
        pod_passes_basic_checks(pod, self.fw.handle.pvcs)
        snap = self.fw.handle.snapshot
        state = {}
        all_nodes = snap.list
        if len(all_nodes) == 0:
            raise ScheduleError("no nodes available to schedule pods")
        st = self.fw.run_prefilter(state, pod)
        if not P.is_success(st):
            raise ScheduleError(repr(st))
        index = {NI.name(ni.node): i for i, ni in enumerate(all_nodes)}
        to_find = self.num_feasible_nodes_to_find(len(all_nodes))
        feasible, statuses = [], {}
        if not self.fw.filters:
            # no filter plugins: the first numNodesToFind nodes, not rotated (generic_scheduler.go:438-444)
            feasible = [ni.node for ni in all_nodes[:to_find]]
        else:
            # checkNode (generic_scheduler.go:451-471) run by one worker: after to_find nodes fit, the
            # next node that fits cancels the search and is dropped (length > numNodesToFind); failures
            # seen before it are recorded
            for i in range(len(all_nodes)):
                ni = all_nodes[(self.next_start + i) % len(all_nodes)]
                if self.nominator is not None:
                    # podPassesFiltersOnNode (generic_scheduler.go:553-615): a second pass with the
                    # node's nominated pods of equal or higher priority added
                    from .preemption import pod_passes_filters_on_node
                    _, plugin, fst = pod_passes_filters_on_node(self.fw, self.nominator, state, pod, ni)
                else:
                    plugin, fst = self.fw.run_filters(state, pod, ni)
                if fst is not None and fst.code == P.ERROR:
                    raise ScheduleError(repr(fst))
                if fst is None:
                    if len(feasible) >= to_find:
                        break
                    feasible.append(ni.node)
                else:
                    statuses[NI.name(ni.node)] = (plugin, fst)
        processed = len(feasible) + len(statuses)
        self.next_start = (self.next_start + processed) % len(all_nodes)
        if not feasible:
            raise FitError(statuses)
        if len(feasible) == 1:
            n = NI.name(feasible[0])
            return Result(n, index[n], 1 + len(statuses), 1, statuses, {}, [], [n])
        pst = self.fw.run_prescore(state, pod, feasible)
        if not P.is_success(pst):
            raise ScheduleError(repr(pst))
        if len(self.fw.scores) == 0:
            totals = [[NI.name(n), 1] for n in feasible]
            scores = {}
        else:
            scores = self.fw.run_scores(state, pod, feasible)
            totals = []
            for i, n in enumerate(feasible):
                totals.append([NI.name(n), sum(scores[k][i][1] for k in scores)])
        host, hidx = select_host(totals, index, self.fw.profile, pod_seq)
        return Result(host, hidx, len(feasible) + len(statuses), len(feasible), statuses, scores, totals,
                      [NI.name(n) for n in feasible])


def pod_passes_basic_checks(pod, pvcs):
    """generic_scheduler.go:1084-1107: every PVC volume must exist in the pod's namespace and not
    be terminating."""
    ns = NI.namespace(pod)
    for v in (pod.get("spec") or {}).get("volumes") or []:
        claim = (v.get("persistentVolumeClaim") or {}).get("claimName") if v.get("persistentVolumeClaim") else None
        if claim is None:
            continue
        pvc = next((c for c in pvcs if NI.name(c) == claim and NI.namespace(c) == ns), None)
        if pvc is None:
            raise ScheduleError('persistentvolumeclaim "%s" not found' % claim)
        if (pvc.get("metadata") or {}).get("deletionTimestamp") is not None:
            raise ScheduleError('persistentvolumeclaim "%s" is being deleted' % claim)


def select_host(totals, index, profile, pod_seq):
    """selectHost (generic_scheduler.go:217-238) with the deterministic packed-key tie-break."""
    if not totals:
        raise ScheduleError("empty priorityList")
    best_key, best = -1, None
    for name, score in totals:
        k = tiebreak.key(score, index[name], pod_seq, profile.seed, profile.tie_break_mode)
        if k > best_key:
            best_key, best = k, name
    return best, index[best]


def schedule_sequence(nodes, existing_pods, pods, profile, services=(), rcs=(), rss=(), sss=(),
                      first_seq=0, pvcs=(), order="tree", image_nodes=None):
    """scheduleOne loop: each placed pod is assumed (NodeInfo.AddPod) before the next one.

    Returns a list of Result (or FitError/ScheduleError instances for unschedulable pods)."""
    snap = NI.Snapshot(nodes, existing_pods, order=order, image_nodes=image_nodes)
    fw = Framework(profile, Handle(snap, services, rcs, rss, sss, pvcs))
    gs = GenericScheduler(fw)
    out = []
    for i, pod in enumerate(pods):
        try:
            r = gs.schedule(pod, first_seq + i)
        except ScheduleError as e:
            out.append(e)
            continue
        placed = dict(pod)
        placed["spec"] = dict(pod.get("spec") or {})
        placed["spec"]["nodeName"] = r.host
        snap.get(r.host).add_pod(placed)
        out.append(r)
    return out

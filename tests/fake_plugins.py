"""The fake filter/score plugins of pkg/scheduler/core/generic_scheduler_test.go:70-296, restated for
the oracle's framework (oracle/refsched/framework.py Profile.plugin_factories).  Test
infrastructure: they exercise the orchestration (filter early exit, FitError statuses, normalize,
weights, score errors) with plugins whose outcome is known by construction."""
from oracle.refsched import nodeinfo as NI
from oracle.refsched import plugins as P

ERR_REASON_FAKE = "Nodes failed the fake predicate"


def _go_atoi(s):
    t = s[1:] if s[:1] in "+-" else s
    if not t or not t.isdigit() or not t.isascii():
        return None
    return int(s)


class _Filter:
    def __init__(self, name, fn):
        self.name, self._fn = name, fn

    def filter(self, state, pod, ni):
        return self._fn(pod, ni)


def true_filter(_h):            # :72-84
    return _Filter("TrueFilter", lambda pod, ni: None)


def false_filter(_h):           # :86-98
    return _Filter("FalseFilter", lambda pod, ni: P.Status(P.UNSCHEDULABLE, ERR_REASON_FAKE))


def match_filter(_h):           # :100-119
    def fn(pod, ni):
        if ni.node is None:
            return P.Status(P.ERROR, "node not found")
        return None if NI.name(pod) == NI.name(ni.node) else P.Status(P.UNSCHEDULABLE, ERR_REASON_FAKE)
    return _Filter("MatchFilter", fn)


def no_pods_filter(_h):         # :121-135
    return _Filter("NoPodsFilter",
                   lambda pod, ni: None if len(ni.pods) == 0 else P.Status(P.UNSCHEDULABLE, ERR_REASON_FAKE))


def fake_filter(codes):         # :137-164: failedNodeReturnCodeMap
    def make(_h):
        def fn(pod, ni):
            c = codes.get(NI.name(ni.node))
            if c is None:
                return None
            return P.Status(c, "injecting failure for pod %s" % NI.name(pod))
        return _Filter("FakeFilter", fn)
    return make


class _Numeric:
    name = "NumericMap"          # :166-189

    def __init__(self, _h):
        pass

    def score(self, state, pod, node_name):
        v = _go_atoi(node_name)
        if v is None:
            return 0, P.Status(P.ERROR, "Error converting nodename to int: %s" % node_name)
        return v, None


class _ReverseNumeric(_Numeric):
    name = "ReverseNumericMap"   # :191-230

    def normalize(self, state, pod, scores):
        mx, mn = 0.0, 1.7976931348623157e308
        for _, s in scores:
            mx, mn = max(mx, float(s)), min(mn, float(s))
        for sc in scores:
            sc[1] = int(mx + mn - float(sc[1]))
        return None


class _TrueMap:
    name = "TrueMap"             # :232-258

    def __init__(self, _h):
        pass

    def score(self, state, pod, node_name):
        return 1, None

    def normalize(self, state, pod, scores):
        for n, _ in scores:
            if n == "":
                return P.Status(P.ERROR, "unexpected empty host name")
        return None


class _FalseMap:
    name = "FalseMap"            # :260-279

    def __init__(self, _h):
        pass

    def score(self, state, pod, node_name):
        return 0, P.Status(P.ERROR, "priority map encounters an error")


# ---- framework/v1alpha1/framework_test.go:142-170 TestPlugin.Filter and :2007-2039 the injected
# score plugins (TestScorePlugin, TestScoreWithNormalizePlugin): outcomes set by the table's args
class _InjectedFilter:
    def __init__(self, name, code):
        self.name, self.code = name, code

    def filter(self, state, pod, ni):
        return P.Status(self.code, "injected filter status")


class _InjectedScore:
    def __init__(self, name, inj):
        self.name, self.inj = name, inj

    def score(self, state, pod, node_name):   # setScoreRes
        if self.inj.get("scoreStatus", 0) != P.SUCCESS:
            return 0, P.Status(self.inj["scoreStatus"], "injecting failure.")
        return self.inj.get("scoreRes", 0), None


class _InjectedScoreNormalize(_InjectedScore):
    def normalize(self, state, pod, scores):  # injectNormalizeRes
        if self.inj.get("normalizeStatus", 0) != P.SUCCESS:
            return P.Status(self.inj["normalizeStatus"], "injecting failure.")
        for sc in scores:
            sc[1] = self.inj.get("normalizeRes", 0)
        return None


def factories(spec):
    """spec: {"FakeFilter": {node: code}, "injected_filters": {name: code}, "injected_scores":
    {name: {"normalize": bool, injectedResult fields}}} -> Profile.plugin_factories."""
    spec = spec or {}
    out = {"TrueFilter": true_filter, "FalseFilter": false_filter, "MatchFilter": match_filter,
           "NoPodsFilter": no_pods_filter, "NumericMap": _Numeric, "ReverseNumericMap": _ReverseNumeric,
           "TrueMap": _TrueMap, "FalseMap": _FalseMap}
    if "FakeFilter" in spec:
        out["FakeFilter"] = fake_filter(spec["FakeFilter"])
    for name, code in (spec.get("injected_filters") or {}).items():
        out[name] = (lambda n, c: lambda _h: _InjectedFilter(n, c))(name, code)
    for name, inj in (spec.get("injected_scores") or {}).items():
        cls = _InjectedScoreNormalize if inj.get("normalize") else _InjectedScore
        out[name] = (lambda n, i, k: lambda _h: k(n, i))(name, inj, cls)
    return out


# ---- core/extender_test.go:56-80,135-356 FakeExtender (predicates only, no node cache): the
# preemption verb keeps a node when every predicate passes on it (selectVictimsOnNodeByExtender
# without cachedNodeNameToInfo) and adds no victims
class ExtenderError(Exception):
    pass


def _pred_true(pod, node):
    return True


def _pred_false(pod, node):
    return False


def _pred_machine1(pod, node):
    return NI.name(node) == "machine1"


def _pred_error(pod, node):
    raise ExtenderError("Some error")


PREDICATES = {"true": _pred_true, "false": _pred_false, "machine1": _pred_machine1, "error": _pred_error}


class FakeExtender:
    def __init__(self, predicates=(), ignorable=False, uninterested=False):
        self.predicates = [PREDICATES[p] for p in predicates]
        self.ignorable, self.uninterested = ignorable, uninterested

    def supports_preemption(self):
        return True

    def is_ignorable(self):
        return self.ignorable

    def is_interested(self, pod):
        return not self.uninterested

    def run_predicate(self, pod, node):
        for pr in self.predicates:
            if not pr(pod, node):
                return False
        return True

    def process_preemption(self, pod, node_to_victims, node_of):
        """node_to_victims: {node name: (victims, num_pdb_violations)} in iteration order;
        node_of(name) -> v1.Node.  Raises ExtenderError."""
        out = dict(node_to_victims)
        for nn in list(out):
            if not self.run_predicate(pod, node_of(nn)):
                del out[nn]
        return out


def extenders(specs):
    """[{"predicates": [...], "ignorable": bool, "uninterested": bool}] -> FakeExtender list."""
    return [FakeExtender(s.get("predicates", ()), s.get("ignorable", False), s.get("uninterested", False))
            for s in specs or ()]

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


def factories(spec):
    """spec: {"FakeFilter": {node: code}} or plain names -> Profile.plugin_factories."""
    out = {"TrueFilter": true_filter, "FalseFilter": false_filter, "MatchFilter": match_filter,
           "NoPodsFilter": no_pods_filter, "NumericMap": _Numeric, "ReverseNumericMap": _ReverseNumeric,
           "TrueMap": _TrueMap, "FalseMap": _FalseMap}
    if "FakeFilter" in (spec or {}):
        out["FakeFilter"] = fake_filter(spec["FakeFilter"])
    return out

"""ORACLE (test infrastructure only) -- label / field selector restatement.

Follows:
  staging/src/k8s.io/apimachinery/pkg/labels/selector.go:60-80   (Everything / Nothing)
  staging/src/k8s.io/apimachinery/pkg/labels/selector.go:140-242 (NewRequirement, Matches)
  staging/src/k8s.io/apimachinery/pkg/labels/selector.go:346-353 (AND of requirements)
  staging/src/k8s.io/apimachinery/pkg/apis/meta/v1/helpers.go:34-70 (LabelSelectorAsSelector)
  staging/src/k8s.io/apimachinery/pkg/util/validation/validation.go (IsQualifiedName, IsValidLabelValue)
  pkg/apis/core/v1/helper/helpers.go:237-346 (NodeSelectorRequirementsAsSelector,
      NodeSelectorRequirementsAsFieldSelector, MatchNodeSelectorTerms)
"""
import re


class SelectorError(Exception):
    pass


_NAME = r"[A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?"
_NAME_RE = re.compile("^" + _NAME + "$")
_DNS1123_SUB = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")


def is_qualified_name(v):
    parts = v.split("/")
    if len(parts) == 1:
        name = parts[0]
    elif len(parts) == 2:
        prefix, name = parts
        if len(prefix) == 0 or len(prefix) > 253 or not _DNS1123_SUB.match(prefix):
            return False
    else:
        return False
    return 0 < len(name) <= 63 and bool(_NAME_RE.match(name))


def is_valid_label_value(v):
    return len(v) == 0 or (len(v) <= 63 and bool(_NAME_RE.match(v)))


def go_parse_int(s):
    """strconv.ParseInt(s, 10, 64); returns None on error."""
    if not isinstance(s, str) or not re.match(r"^[+-]?[0-9]+$", s):
        return None
    v = int(s)
    if v < -(2 ** 63) or v > 2 ** 63 - 1:
        return None
    return v


IN, NOTIN, EXISTS, DNE, GT, LT, EQ, DEQ, NEQ = "in", "notin", "exists", "!", "gt", "lt", "=", "==", "!="


class Requirement:
    __slots__ = ("key", "op", "vals")

    def __init__(self, key, op, vals):
        # selector.go NewRequirement validation
        if not is_qualified_name(key):
            raise SelectorError("invalid label key %r" % key)
        vals = list(vals or [])
        if op in (IN, NOTIN):
            if len(vals) == 0:
                raise SelectorError("for 'in', 'notin' operators, values set can't be empty")
        elif op in (EQ, DEQ, NEQ):
            if len(vals) != 1:
                raise SelectorError("exact-match compatibility requires one single value")
        elif op in (EXISTS, DNE):
            if len(vals) != 0:
                raise SelectorError("values set must be empty for exists and does not exist")
        elif op in (GT, LT):
            if len(vals) != 1:
                raise SelectorError("for 'Gt', 'Lt' operators, exactly one value is required")
            for v in vals:
                if go_parse_int(v) is None:
                    raise SelectorError("for 'Gt', 'Lt' operators, the value must be an integer")
        else:
            raise SelectorError("operator '%s' is not recognized" % op)
        for v in vals:
            if not is_valid_label_value(v):
                raise SelectorError("invalid label value %r" % v)
        self.key, self.op, self.vals = key, op, vals

    @classmethod
    def raw(cls, key, op, vals):
        r = cls.__new__(cls)
        r.key, r.op, r.vals = key, op, list(vals)
        return r

    def matches(self, ls):
        op, key = self.op, self.key
        if op in (IN, EQ, DEQ):
            return key in ls and ls[key] in self.vals
        if op in (NOTIN, NEQ):
            return key not in ls or ls[key] not in self.vals
        if op == EXISTS:
            return key in ls
        if op == DNE:
            return key not in ls
        if op in (GT, LT):
            if key not in ls:
                return False
            lv = go_parse_int(ls[key])
            if lv is None or len(self.vals) != 1:
                return False
            rv = go_parse_int(self.vals[0])
            if rv is None:
                return False
            return (op == GT and lv > rv) or (op == LT and lv < rv)
        return False


class Selector:
    """internalSelector (AND of requirements) or the Nothing selector."""
    __slots__ = ("reqs", "nothing")

    def __init__(self, reqs=(), nothing=False):
        self.reqs = list(reqs)
        self.nothing = nothing

    def matches(self, ls):
        if self.nothing:
            return False
        ls = ls or {}
        for r in self.reqs:
            if not r.matches(ls):
                return False
        return True

    def empty(self):
        # internalSelector.Empty(): len==0; nothingSelector.Empty() is false
        return (not self.nothing) and len(self.reqs) == 0


NOTHING = Selector(nothing=True)
EVERYTHING = Selector()

_LSEL_OPS = {"In": IN, "NotIn": NOTIN, "Exists": EXISTS, "DoesNotExist": DNE}
_NSEL_OPS = {"In": IN, "NotIn": NOTIN, "Exists": EXISTS, "DoesNotExist": DNE, "Gt": GT, "Lt": LT}


def label_selector_as_selector(ps):
    """metav1.LabelSelectorAsSelector: nil -> Nothing, empty -> Everything."""
    if ps is None:
        return NOTHING
    ml = ps.get("matchLabels") or {}
    me = ps.get("matchExpressions") or []
    if len(ml) + len(me) == 0:
        return Selector()
    reqs = []
    for k in sorted(ml):
        reqs.append(Requirement(k, EQ, [ml[k]]))
    for e in me:
        op = _LSEL_OPS.get(e.get("operator"))
        if op is None:
            raise SelectorError("%r is not a valid pod selector operator" % e.get("operator"))
        reqs.append(Requirement(e.get("key", ""), op, list(e.get("values") or [])))
    return Selector(reqs)


def selector_from_set(m):
    """labels.SelectorFromSet == SelectorFromValidatedSet (selector.go:874-912): no validation."""
    if not m:
        return Selector()
    return Selector([Requirement.raw(k, EQ, [m[k]]) for k in sorted(m)])


def node_selector_requirements_as_selector(nsm):
    if not nsm:
        return NOTHING
    reqs = []
    for e in nsm:
        op = _NSEL_OPS.get(e.get("operator"))
        if op is None:
            raise SelectorError("%r is not a valid node selector operator" % e.get("operator"))
        reqs.append(Requirement(e.get("key", ""), op, list(e.get("values") or [])))
    return Selector(reqs)


def node_field_selector_matches(nsm, fields):
    """NodeSelectorRequirementsAsFieldSelector(...).Matches(fields); raises on error."""
    if not nsm:
        return False  # fields.Nothing()
    for e in nsm:
        op = e.get("operator")
        vals = e.get("values") or []
        if op in ("In", "NotIn"):
            if len(vals) != 1:
                raise SelectorError("unexpected number of value")
            got = fields.get(e.get("key", ""), "")
            if op == "In" and got != vals[0]:
                return False
            if op == "NotIn" and got == vals[0]:
                return False
        else:
            raise SelectorError("%r is not a valid node field selector operator" % op)
    return True


def match_node_selector_terms(terms, node_labels, node_fields):
    """v1helper.MatchNodeSelectorTerms: terms ORed; nil/empty term selects nothing."""
    for t in terms or []:
        me = t.get("matchExpressions") or []
        mf = t.get("matchFields") or []
        if len(me) == 0 and len(mf) == 0:
            continue
        if me:
            try:
                sel = node_selector_requirements_as_selector(me)
            except SelectorError:
                continue
            if not sel.matches(node_labels):
                continue
        if mf:
            try:
                ok = node_field_selector_matches(mf, node_fields)
            except SelectorError:
                continue
            if not ok:
                continue
        return True
    return False

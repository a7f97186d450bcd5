"""ORACLE (test infrastructure only) -- resource.Quantity restatement.

Restates the parts of k8s.io/apimachinery resource.Quantity that the scheduler's
hot path reads:
  staging/src/k8s.io/apimachinery/pkg/api/resource/quantity.go:140-260 (ParseQuantity
  grammar: <signedNumber><suffix>, suffix in binarySI / decimalSI / decimalExponent),
  quantity.go:695-716 (Value / MilliValue = ScaledValue rounded *up*, i.e. away from 0).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package.  Exact arithmetic via fractions.Fraction.
"""
from fractions import Fraction
import re

_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": 1,
        "k": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15, "E": 10 ** 18}
_RE = re.compile(r"^([+-]?)(\d*)(?:\.(\d*))?(.*)$")


def parse(q):
    """Return the exact rational value of a quantity string (or int)."""
    if isinstance(q, int):
        return Fraction(q)
    if isinstance(q, Fraction):
        return q
    s = str(q).strip()
    m = _RE.match(s)
    if not m or (m.group(2) == "" and not m.group(3)):
        raise ValueError("quantities must match the regular expression: %r" % q)
    sign, whole, frac, suffix = m.groups()
    num = Fraction(int(whole or "0"))
    if frac:
        num += Fraction(int(frac), 10 ** len(frac))
    if sign == "-":
        num = -num
    if suffix in _BIN:
        return num * _BIN[suffix]
    if suffix in _DEC:
        return num * _DEC[suffix]
    if suffix[:1] in ("e", "E"):
        return num * Fraction(10) ** int(suffix[1:])
    raise ValueError("unable to parse quantity's suffix: %r" % q)


def _round_away(x):
    if x.denominator == 1:
        return int(x)
    n = x.numerator // x.denominator  # floor
    return n + 1 if x > 0 else n


def value(q):
    """Quantity.Value(): rounded up (away from zero) to an integer."""
    return _round_away(parse(q))


def milli_value(q):
    """Quantity.MilliValue()."""
    return _round_away(parse(q) * 1000)

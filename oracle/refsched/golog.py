"""ORACLE (test infrastructure only) -- Go math.Log restatement.

Go's math.Log (go1.13.9, the reference toolchain: build/root/WORKSPACE:22) is the FreeBSD
e_log.c algorithm (src/math/log.go; the amd64 archLog follows the same sequence of
SSE2 double operations).  It is a Go standard-library dependency absent from
/root/reference; restated here from its published algorithm.  Used by
PodTopologySpread topologyNormalizingWeight (podtopologyspread/scoring.go:286-288).
Parity at the ulp level is pinned only indirectly (PTS scoring golden tables).
"""
import math

LN2HI = 6.93147180369123816490e-01
LN2LO = 1.90821492927058770002e-10
L1 = 6.666666666666735130e-01
L2 = 3.999999999940941908e-01
L3 = 2.857142874366239149e-01
L4 = 2.222219843214978396e-01
L5 = 1.818357216161805012e-01
L6 = 1.531383769920937332e-01
L7 = 1.479819860511658591e-01
SQRT2_HALF = math.sqrt(2) / 2


def go_log(x):
    if math.isnan(x) or x == math.inf:
        return x
    if x < 0:
        return math.nan
    if x == 0:
        return -math.inf
    f1, ki = math.frexp(x)  # same contract as Go Frexp: f1 in [0.5, 1)
    if f1 < SQRT2_HALF:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)))
    t2 = s4 * (L2 + s4 * (L4 + s4 * L6))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * LN2HI - ((hfsq - (s * (hfsq + R) + k * LN2LO)) - f)

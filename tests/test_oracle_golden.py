"""Pin the CPU oracle (oracle/refsched) against the reference's own test tables."""
import pytest

from conftest import golden_groups, load_golden
from golden_runner import check, oracle_eval

CASES = [(g, i, c) for g in golden_groups() for i, c in enumerate(load_golden(g))]


@pytest.mark.parametrize("group,idx,case", CASES, ids=["%s-%d" % (g, i) for g, i, _ in CASES])
def test_oracle_matches_reference_table(group, idx, case):
    got = oracle_eval(case)
    bad = check(case, got)
    assert not bad, "%s (%s): %r" % (case["name"], case["src"], bad)

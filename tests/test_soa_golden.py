"""Golden vectors through the product compile step + the C restatement (CPU) and libkgpu (GPU)."""
import pytest

from conftest import golden_groups, load_golden
from golden_runner import check
from soa_runner import soa_eval, supported

CASES = [(g, i, c) for g in golden_groups() for i, c in enumerate(load_golden(g)) if supported(c)]
IDS = ["%s-%d" % (g, i) for g, i, _ in CASES]


@pytest.mark.parametrize("group,idx,case", CASES, ids=IDS)
def test_compile_and_c_restatement_match_reference_table(group, idx, case):
    got = soa_eval(case, "ref")
    bad = check(case, got)
    assert not bad, "%s (%s): %r" % (case["name"], case["src"], bad)


@pytest.mark.gpu
@pytest.mark.parametrize("group,idx,case", CASES, ids=IDS)
def test_gpu_matches_reference_table(group, idx, case):
    got = soa_eval(case, "gpu")
    bad = check(case, got)
    assert not bad, "%s (%s): %r" % (case["name"], case["src"], bad)

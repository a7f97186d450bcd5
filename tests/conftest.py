import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "kubernetes-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libkgpu.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long CPU test")


def load_golden(group):
    with open(os.path.join(GOLDEN, group + ".json")) as fh:
        return json.load(fh)


def golden_groups():
    return sorted(f[:-5] for f in os.listdir(GOLDEN) if f.endswith(".json"))


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()

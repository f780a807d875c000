import gzip
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP path)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_preset():
    return load_golden("traj_preset.json.gz")


@pytest.fixture(scope="session")
def golden_random():
    return load_golden("traj_random.json.gz")


@pytest.fixture(scope="session")
def golden_rng():
    return load_golden("rng_streams.json.gz")

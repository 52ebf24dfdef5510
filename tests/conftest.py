"""Shared fixtures.  `-m "not gpu"` runs on CPU (oracle vs golden vectors,
host-side library logic, gloo multi-process); `-m gpu` needs an MI355X."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
MAPS = os.path.join(REPO, "f110_gymnasium_ros2_jazzy_amd", "maps")
for p in (REPO, os.path.join(REPO, "oracle"), GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def oracle_scanners(oracle_mod):
    cache = {}

    def get(map_name):
        if map_name not in cache:
            free, res, org = oracle_mod.load_map(os.path.join(MAPS, map_name + ".yaml"))
            cache[map_name] = oracle_mod.OracleScanner(free, res, org)
        return cache[map_name]
    return get


@pytest.fixture(scope="session")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def tracks():
    from f110_gymnasium_ros2_jazzy_amd.maps import load_map
    cache = {}

    def get(map_name):
        if map_name not in cache:
            t = load_map(os.path.join(MAPS, map_name + ".yaml"))
            t.ensure_edt()
            cache[map_name] = t
        return cache[map_name]
    return get

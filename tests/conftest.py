"""Shared test setup: markers, library build-on-demand, fixtures."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: larger inputs")
    lib = os.path.join(ROOT, "sparsecholesky_amd", "libsparsecholesky_amd.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "sparsecholesky_amd", "csrc")], check=True)
    olib = os.path.join(ROOT, "oracle", "liboracle_refchol.so")
    if not os.path.exists(olib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


@pytest.fixture(scope="session")
def known():
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def mtx():
    import sparsecholesky_amd as sc

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = sc.load_matrix_market_to_csc(os.path.join(GOLDEN, name + ".mtx"))
        return cache[name]

    return load


def has_gpu():
    try:
        import sparsecholesky_amd as sc

        return sc.lib().sc_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not has_gpu():
        pytest.fail("GPU test selected but no HIP device is visible (the HIP path has no CPU fallback)")
    return True

import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden", "merkle_golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def oracle_lib():
    """CPU checker (test infrastructure only)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    from oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def ctx():
    """GPU context over device 0 -- only for @pytest.mark.gpu tests."""
    from deoss_amd import MerkleContext, load_library
    load_library()
    c = MerkleContext()
    yield c
    c.close()


def pytest_collection_modifyitems(config, items):
    """DEOSS_TEST_SHUFFLE=<seed>: run the collected tests in a seeded random order (an order-
    dependence check: a context created at a destroyed one's address once read its stale state).
    Unset: the normal order."""
    seed = os.environ.get("DEOSS_TEST_SHUFFLE")
    if seed:
        import random
        random.Random(int(seed)).shuffle(items)

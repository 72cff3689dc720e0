import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "plonk-by-fingers_amd"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpbf.so on cuda:0)")


@pytest.fixture(scope="session")
def kats():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def vectors():
    with open(os.path.join(GOLDEN, "ntt_vectors.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def ctx():
    import pbf

    c = pbf.Context(0)
    yield c
    c.close()

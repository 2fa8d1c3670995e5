import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def ref_vectors():
    import json
    import stream

    with open(os.path.join(GOLDEN, "ref_vectors.json")) as f:
        v = json.load(f)
    blob = stream.golden_blob(v["blob_bytes"])
    return v, blob


@pytest.fixture(scope="session")
def kats():
    import json

    with open(os.path.join(GOLDEN, "kat_reference_tests.json")) as f:
        return json.load(f)

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


# Test infrastructure only: the sanitizer run (tools/asan_cpu.sh) points the
# tests at lib/libforst_checksum_asan.so; the product reads no such variable.
if os.environ.get("FORST_TEST_LIB"):
    from forst_amd import _lib as _forst_lib

    _forst_lib.use_library(os.environ["FORST_TEST_LIB"])


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


@pytest.fixture(scope="session")
def kv_sites():
    """reference-made a15 call-site fixtures (tests/golden/gen_kv_golden.py)"""
    import json

    import numpy as np

    with open(os.path.join(GOLDEN, "kv_sites.json")) as f:
        meta = json.load(f)
    z = np.load(os.path.join(GOLDEN, "kv_sites.npz"), allow_pickle=False)
    return meta, {k: z[k] for k in z.files}

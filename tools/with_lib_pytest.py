#!/usr/bin/env python3
"""tools/with_lib_pytest.py <library.so> [pytest args...] -- run the test suite
against another build of the C ABI (parity of A/B variants before timing)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from forst_amd import _lib  # noqa: E402

_lib.use_library(sys.argv[1])
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[2:]))

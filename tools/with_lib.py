#!/usr/bin/env python3
"""tools/with_lib.py <library.so> <script.py> [args...] -- run a script with
another build of the C ABI loaded (A/B of two builds, tools/ab_libs.sh)."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from forst_amd import _lib  # noqa: E402




class _OlderBuild(_lib.ctypes.CDLL):
    """an older build lacks entry points added since: they raise when CALLED
    (A/B against an earlier round's library), not when the table is bound"""

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            if not name.startswith("forst_"):
                raise

            def missing(*a):
                raise RuntimeError(f"{name} is not in {sys.argv[1]}")
            return missing


_lib.ctypes.CDLL = _OlderBuild  # (tools only: the product binding stays strict)
_lib.use_library(sys.argv[1])
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")

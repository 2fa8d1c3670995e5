#!/usr/bin/env python3
"""tools/ab_kv.py <lib.so> [label] -- the a15_kv bench extra (bench.py run_kv)
through another build of the C ABI (A/B of kv_protect.hip build knobs: one
process per library, tools/build_variant.sh makes them)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from forst_amd import _lib  # noqa: E402

_lib.use_library(sys.argv[1])
import bench  # noqa: E402
from forst_amd import engine  # noqa: E402

engine.init_device()
r = bench.run_kv(20, 3)
r["lib"] = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(sys.argv[1])
print(json.dumps(r), flush=True)

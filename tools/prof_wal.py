#!/usr/bin/env python3
"""tools/prof_wal.py -- the C5 WAL configuration alone (bench.run_wal: writer
CRC, reader verify, a14 record XXH3, fused recovery) for rocprofv3 passes
(profiles/profile.sh <tag> C5)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from forst_amd import engine  # noqa: E402

engine.init_device()
print(json.dumps(bench.run_wal(4, 1)), flush=True)

"""A/B of the WAL writer + verify paths on C5 (bench.run_wal) under env
variants, each in its own process.  Usage: python tools/wal_ab.py [VAR=val ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
variants = sys.argv[1:] or ["FORST_WAL_VARIANT=", "FORST_WAL_VARIANT=wave"]
for v in variants:
    env = dict(os.environ)
    # variants exist only in the diagnostics build (make -C forst_amd/csrc diag)
    k, _, val = v.partition("=")
    env[k] = val
    code = ("import sys, json; sys.path.insert(0, %r); import bench; "
            "from forst_amd import _lib, engine; "
            "_lib.use_library(%r); engine.init_device(); "
            "print(json.dumps(bench.run_wal(5, 1)))" % (ROOT, os.path.join(
                ROOT, "forst_amd", "lib", "libforst_checksum_diag.so")))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=300)
    line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else out.stderr[-2000:]
    print(v, line, flush=True)
    if out.returncode != 0:
        sys.exit(out.returncode)

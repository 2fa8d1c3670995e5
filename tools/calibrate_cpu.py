#!/usr/bin/env python3
"""tools/calibrate_cpu.py -- calibrate bench.py's CPU baseline (the port,
oracle/oracle.c) against the compiled REFERENCE on this host.

The reference's checksum sources (tests/golden/gen_golden.py REF_SRCS) plus
tests/golden/ref_calib.cc (a threaded batch loop over table/format.cc:594
ComputeBuiltinChecksumWithLastByte) are compiled the way the reference's own
CMake build compiles them by default (PORTABLE=0: -march=native, -O2) into a
temporary directory outside the repository and deleted afterwards.  Both
sides checksum the same blocks (C2-shaped 4 KiB and NS16-shaped 16 KiB,
kCRC32c and kXXH3) on 1 thread and on every CPU of this container; the
results must agree bit for bit.  Writes profiles/cpu_calibration_<tag>.json.

    python tools/calibrate_cpu.py r02
"""
import ctypes
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gen_golden  # noqa: E402

from oracle import oracle as O  # noqa: E402

GIB = float(1 << 30)


def build(tmp):
    out = os.path.join(tmp, "libforst_ref_calib.so")
    cmd = (["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-march=native",
            "-ffunction-sections", "-fdata-sections", "-Wl,--gc-sections", "-Wl,--no-undefined",
            "-DROCKSDB_PLATFORM_POSIX", "-DOS_LINUX", "-DNDEBUG", "-DNPERF_CONTEXT",
            "-fvisibility=hidden", "-fvisibility-inlines-hidden", "-w",
            f"-I{gen_golden.REF}", f"-I{gen_golden.REF}/include", "-o", out]
           + [os.path.join(gen_golden.REF, s) for s in gen_golden.REF_SRCS]
           + [os.path.join(gen_golden.HERE, "ref_calib.cc"), "-lpthread"])
    subprocess.check_call(cmd)
    L = ctypes.CDLL(out)
    vp = ctypes.c_void_p
    L.ref_block_checksum_batch.restype = None
    L.ref_block_checksum_batch.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64,
                                           ctypes.c_int, vp]
    return L


def blocks(n, size, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, n * (size + 5), dtype=np.uint8)
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(size + 5))
    sizes = np.full(n, size, np.uint32)
    last = base[(offs + sizes).astype(np.int64)].copy()
    return base, offs, sizes, last


def best_of(fn, budget=6.0, reps=5):
    fn()
    best, spent, k = 1e30, 0.0, 0
    while k < reps and spent < budget:
        t = time.perf_counter()
        fn()
        dt = time.perf_counter() - t
        best, spent, k = min(best, dt), spent + dt, k + 1
    return best


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    ncpu = len(os.sched_getaffinity(0))
    cases = [("C2", 1 << 17, 4096, 1), ("C2-xxh3", 1 << 17, 4096, 4),
             ("NS16", 1 << 15, 16384, 1), ("NS16X", 1 << 15, 16384, 4)]
    tmp = tempfile.mkdtemp(prefix="forst_ref_calib_")
    rows = []
    try:
        L = build(tmp)
        for name, n, size, ct in cases:
            base, offs, sizes, last = blocks(n, size, 0xCA11B + size + ct)
            nbytes = n * (size + 1)
            ref_out = np.zeros(n, np.uint32)
            for nt in sorted({1, ncpu}):
                def ref():
                    L.ref_block_checksum_batch(ct, base.ctypes.data, offs.ctypes.data,
                                               sizes.ctypes.data, last.ctypes.data, n, nt,
                                               ref_out.ctypes.data)
                port_out = [None]

                def port():
                    port_out[0] = O.block_checksum_batch(ct, base, offs, sizes, last_bytes=last,
                                                         nthreads=nt)
                t_ref, t_port = best_of(ref), best_of(port)
                assert np.array_equal(ref_out, port_out[0]), name
                rows.append({"case": name, "blocks": n, "block_size": size, "checksum": ct,
                             "threads": nt, "reference_GiBps": round(nbytes / t_ref / GIB, 3),
                             "port_GiBps": round(nbytes / t_port / GIB, 3),
                             "port_over_reference": round(t_ref / t_port, 3)})
                print(json.dumps(rows[-1]), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    out = {"generator": "tools/calibrate_cpu.py", "host_cpu": cpu, "threads_available": ncpu,
           "reference_build": "g++ -O2 -march=native (the reference CMake default PORTABLE=0) "
                              "of " + ", ".join(gen_golden.REF_SRCS) + " + tests/golden/ref_calib.cc",
           "port_build": "oracle/oracle.c as bench.py's cpu_baseline uses it",
           "what": "ComputeBuiltinChecksumWithLastByte over the same blocks, results equal",
           "rows": rows}
    path = os.path.join(ROOT, "profiles", f"cpu_calibration_{tag}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""profiles/summarize.py <tag> [config]

Turns the raw rocprofv3 output of profiles/profile.sh (gpurun_out/prof_<tag>/)
into committed evidence:
  profiles/<tag>_kernel_stats.csv  -- the --kernel-trace --stats summary
  profiles/pmc_<tag>.json          -- per-kernel HBM traffic per launch

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(FETCH_SIZE/WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reads exactly 1/2 of
the bytes of a wide 16 B/lane streaming read -- MI355X_MICROARCH.md §HBM --
so it is doubled; the per-kernel ratio to the algorithmic byte count is
recorded so the correction stays checkable).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


MODES = {"0": "compute", "1": "trailer", "2": "verify", "3": "raw"}


def short(name):
    """rocprof's demangled name -> the engine's kernel name (forst_last_kernel)"""
    import re
    n = name.replace("forst::(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(forst::")[0].split("(unsigned")[0]
    # <MODE> or <MODE, 0> -> <mode>; probe instantiations keep their numbers
    return re.sub(r"<(\d)(?:, 0)?>", lambda m: "<" + MODES[m.group(1)] + ">", n)


def load_counter(path):
    vals = defaultdict(list)
    if not os.path.exists(path):
        return vals
    for r in csv.DictReader(open(path)):
        vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    config = sys.argv[2] if len(sys.argv) > 2 else "C2"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    avg_ns = {}
    for r in csv.DictReader(open(stats)):
        avg_ns[short(r["Name"])] = float(r["AverageNs"])
    fetch = load_counter(os.path.join(src, "fetch", "fetch_counter_collection.csv"))
    write = load_counter(os.path.join(src, "write", "write_counter_collection.csv"))
    rows = []
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(("crc32c", "xxh3", "wal", "noop", "trailer_scatter")):
            continue
        f = sum(fetch[k]) / len(fetch[k]) if fetch[k] else 0.0
        w = sum(write[k]) / len(write[k]) if write[k] else 0.0
        rows.append({"kernel": k, "config": config,
                     "fetch_size_kib_avg": f, "write_size_kib_avg": w,
                     "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024),
                     "avg_duration_ns_kernel_trace": avg_ns.get(k)})
    out = {"tag": tag, "config": config,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving)",
           "kernels": rows}
    with open(os.path.join(ROOT, "profiles", f"pmc_{tag}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

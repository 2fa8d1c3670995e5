#!/usr/bin/env python3
"""profiles/summarize.py <tag> <config>

Turns the raw rocprofv3 output of profiles/profile.sh
(gpurun_out/prof_<tag>_<config>/) into committed evidence:
  profiles/<tag>_<config>_kernel_stats.csv -- the --kernel-trace --stats summary
  profiles/pmc_<tag>_<config>.json         -- per kernel: average duration from the
                                              kernel trace, HBM bytes per launch

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports exactly 1/2 of
the bytes of a wide 16 B/lane streaming read -- MI355X_MICROARCH.md §HBM --
so it is doubled).  Kernel names are normalised to the engine's
(forst_last_kernel: 'crc32c_rows_kernel<verify>'), which is what bench.py
looks up.
"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = {"0": "compute", "1": "trailer", "2": "verify", "3": "raw"}
KV_MODES = {"0": "hash64", "1": "protect", "2": "verify", "3": "mem_verify", "4": "mem_protect"}
TIMED = 10  # bench.py --steps default (profiles/profile.sh runs the same count)


def short(name):
    """rocprof's demangled name -> the engine's kernel name"""
    n = name.replace("forst::(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(forst::")[0].split("(unsigned")[0].split("(")[0].strip()
    if n.startswith("kv_kernel<"):  # KvMode (engine.h), not the block modes
        return re.sub(r"<(\d)>", lambda m: "<" + KV_MODES[m.group(1)] + ">", n)
    return re.sub(r"<(\d)>", lambda m: "<" + MODES[m.group(1)] + ">", n)


def load_counter(path):
    vals = defaultdict(list)
    if os.path.exists(path):
        for r in csv.DictReader(open(path)):
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def main():
    tag, config = sys.argv[1], sys.argv[2]
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{config}")
    stats = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_{config}_kernel_stats.csv"))
    avg_ns, calls = {}, {}
    for r in csv.DictReader(open(stats)):
        avg_ns[short(r["Name"])] = float(r["AverageNs"])
        calls[short(r["Name"])] = int(r["Calls"])
    # per-launch durations in dispatch order (the spread behind the average:
    # launches of one run differ by up to ~20 % under the profiler)
    launches = defaultdict(list)
    trace = os.path.join(src, "trace", "trace_kernel_trace.csv")
    if os.path.exists(trace):
        for r in sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"])):
            launches[short(r["Kernel_Name"])].append(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    fetch = load_counter(os.path.join(src, "fetch", "fetch_counter_collection.csv"))
    write = load_counter(os.path.join(src, "write", "write_counter_collection.csv"))
    rows = []
    for k in sorted(set(avg_ns) | set(fetch) | set(write)):
        if k.startswith(("fill_stream", "elementwise", "at::", "__amd")) or "native" in k:
            continue
        f = sum(fetch[k]) / len(fetch[k]) if fetch[k] else None
        w = sum(write[k]) / len(write[k]) if write[k] else None
        rows.append({"kernel": k, "config": config, "calls": calls.get(k),
                     "avg_duration_ns_kernel_trace": avg_ns.get(k),
                     "launch_ns": launches.get(k) if len(launches.get(k, [])) <= 64 else None,
                     # the last TIMED launches: a bench config's profiled command is the
                     # default bench run (--steps 10 --warmup 3), whose last 10 launches
                     # of each kernel are the steps its HIP events time
                     "avg_duration_ns_timed_steps": (
                         sum(launches[k][-TIMED:]) / TIMED
                         if config != "C5" and len(launches.get(k, [])) >= TIMED else None),
                     "fetch_size_kib_avg": f, "write_size_kib_avg": w,
                     "hbm_bytes_per_launch": (int(2 * (f or 0) * 1024 + (w or 0) * 1024)
                                              if f is not None or w is not None else None)})
    out = {"tag": tag, "config": config,
           "method": "rocprofv3 --kernel-trace --stats, then --pmc FETCH_SIZE and --pmc "
                     "WRITE_SIZE in separate passes of the same command; "
                     "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving)",
           "kernels": rows}
    with open(os.path.join(ROOT, "profiles", f"pmc_{tag}_{config}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

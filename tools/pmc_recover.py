#!/usr/bin/env python3
"""tools/pmc_recover.py <fetch_dir> <write_dir> -- HBM traffic of one
forst_wal_recover_batch call in a tools/prof_wal.py PMC pass (tools/gpu_wal.sh):
every dispatch from the first rw_count_kernel (the recovery's first kernel; the
recovery calls are the last phase of bench.run_wal) to the end, per call, with
the largest kernels listed.  FETCH_SIZE / WRITE_SIZE are KiB (x1024 bytes)."""
import collections
import csv
import glob
import os
import sys


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def name(r):
    return r["Kernel_Name"].replace("void ", "").replace("forst::(anonymous namespace)::", "").split("(")[0]


out = {}
for d, counter in ((sys.argv[1], "FETCH_SIZE"), (sys.argv[2], "WRITE_SIZE")):
    rows = load(d, counter)
    first = next(i for i, r in enumerate(rows) if name(r).startswith("rw_count_kernel"))
    calls = sum(1 for r in rows[first:] if name(r).startswith("rw_count_kernel"))
    per = collections.defaultdict(float)
    for r in rows[first:]:
        per[name(r)] += float(r["Counter_Value"]) * 1024 / calls
    tot = sum(per.values())
    out[counter] = tot
    print(f"{counter}: {tot / 1e9:.2f} GB per recovery ({calls} calls)")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:6]:
        print(f"   {k[:48]:48s} {v / 1e9:8.2f} GB")
print(f"total {sum(out.values()) / 1e9:.2f} GB")

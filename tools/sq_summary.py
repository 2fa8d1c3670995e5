#!/usr/bin/env python3
"""tools/sq_summary.py <dir>... -- per-kernel averages of the SQ counters
collected by tools/gpu_sq.sh (rocprofv3 --pmc csv), with the derived shares:
VALU busy = ACTIVE_INST_VALU x 4 / (SIMDs x cycles), wait shares of
SQ_WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots)."""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(dict)
    for x in csv.DictReader(open(f[0])):
        k = x["Kernel_Name"].replace("void ", "").replace("forst::(anonymous namespace)::", "")
        k = k.split("(")[0][:48]
        agg[k][x["Counter_Name"]] += float(x["Counter_Value"])
        disp[k][x["Dispatch_Id"]] = (int(x["Start_Timestamp"]), int(x["End_Timestamp"]))
    print(d)
    rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:6]
    for k, v in rows:
        n = len(disp[k])
        ns = sum(e - s for s, e in disp[k].values()) / n
        wc = v["SQ_WAVE_CYCLES"] / n
        valu = v["SQ_INSTS_VALU"] / n
        busy = v["SQ_ACTIVE_INST_VALU"] / n * 4 / (1024 * ns * 2.4)
        print(f"  {k:48s} n={n:2d} {ns/1e6:7.3f} ms  VALU/disp={valu:.3g} valu_busy={busy:.2f} "
              f"wait_mem={v['SQ_WAIT_ANY']/n/wc:.2f} wait_issue={v['SQ_WAIT_INST_ANY']/n/wc:.2f} "
              f"active={v['SQ_ACTIVE_INST_ANY']/n/wc:.2f} LDS/disp={v['SQ_INSTS_LDS']/n:.3g}")

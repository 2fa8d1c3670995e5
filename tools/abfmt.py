"""print an ab_bench.py JSON log as one line per variant"""
import json
import sys

for path in sys.argv[1:]:
    t = open(path).read()
    j = json.loads(t[t.index("{"):])
    for k, v in j.items():
        print(f"{k:50s} {v['median_ms']:8.3f} ms  frac {v['roofline_frac_median']}")

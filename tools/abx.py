"""tools/abx.py <ab_multi output>... -- one line per X:<extra> run of
tools/ab_multi.sh: config, library, verify and trailer fraction of the HBM peak"""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        try:
            cfg, lib, js = line.split(" ", 2)
            d = json.loads(js)
        except ValueError:
            print(line.rstrip())
            continue
        print(cfg, lib, "verify", d.get("verify_roofline_frac"), "trailer", d.get("trailer_roofline_frac"))

#!/bin/bash
# A/B of two builds of the library on one box, alternating processes:
#   tools/ab_libs.sh <tag> <lib A> <lib B> [configs...]   (C5 = tools/prof_wal.py)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; A=$2; B=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in ${*:-C2}; do
  for r in 1 2 3; do
    for L in $A $B; do
      if [ "$c" = C5 ]; then
        timeout -k 10 300 python -u tools/with_lib.py $L tools/prof_wal.py > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
        tail -1 "$OUT/ab.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 $(basename $L)', d['verify_roofline_frac'], d['writer_roofline_frac'], d['record_xxh3_ms'], d['recover_ms'])"
      else
        timeout -k 10 300 python -u tools/with_lib.py $L bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-extras > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
        tail -1 "$OUT/ab.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $(basename $L)', d['value'], {k: v['frac'] for k, v in d['kernels'].items()})"
      fi
    done
  done
done

#!/bin/bash
# A/B/C... of several builds of the library on one box, alternating processes:
#   tools/ab_multi.sh <tag> <config> <lib>...   (X:<extra> = a bench.py extra; config C5 = tools/prof_wal.py, A14 = tools/prof_a14.py, E2E = tools/prof_e2e.py, SW = tools/prof_small_wal.py, B:<cfg> = tools/prof_blocks.py <cfg>)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; c=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in 1 2 3; do
  for L in "$@"; do
    if [ "$c" = C5 ]; then
      timeout -k 10 300 python -u tools/with_lib.py $L tools/prof_wal.py > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
      tail -1 "$OUT/ab.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 $(basename $L)', d['verify_roofline_frac'], d['writer_roofline_frac'], d['record_xxh3_ms'], d['recover_ms'])"
    elif [ "${c#B:}" != "$c" ]; then
      timeout -k 10 300 python -u tools/with_lib.py $L tools/prof_blocks.py ${c#B:} > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
      echo "$c $(basename $L) $(tail -1 "$OUT/ab.log")"
    elif [ "${c#X:}" != "$c" ]; then  # X:<extra> = one bench.py extra (a15_kv, C5_wal, NS16H32, ...)
      timeout -k 10 300 python -u tools/with_lib.py $L bench.py --extra ${c#X:} > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
      echo "$c $(basename $L) $(tail -1 "$OUT/ab.log")"
    elif [ "$c" = SW ]; then
      timeout -k 10 300 python -u tools/with_lib.py $L tools/prof_small_wal.py > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
      echo "SW $(basename $L) $(tail -1 "$OUT/ab.log")"
    elif [ "$c" = E2E ]; then
      timeout -k 10 300 python -u tools/with_lib.py $L tools/prof_e2e.py > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
      echo "E2E $(basename $L) $(tail -1 "$OUT/ab.log")"
    elif [ "$c" = A14 ]; then
      timeout -k 10 300 python -u tools/with_lib.py $L tools/prof_a14.py > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
      echo "A14 $(basename $L) $(tail -1 "$OUT/ab.log")"
    else
      timeout -k 10 300 python -u tools/with_lib.py $L bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-extras > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
      tail -1 "$OUT/ab.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $(basename $L)', d['value'], {k: v['frac'] for k, v in d['kernels'].items()})"
    fi
  done
done

#!/bin/bash
# profiles/profile.sh -- rocprofv3 evidence for one bench.py config (GPU box):
#   1. --kernel-trace --stats   per-kernel durations (compared with bench.py's HIP events)
#   2. --pmc FETCH_SIZE         HBM read traffic   (separate pass, MI355X_MICROARCH.md §HBM)
#   3. --pmc WRITE_SIZE         HBM write traffic  (separate pass)
# Usage: bash profiles/profile.sh <tag> <config> [program args...]
#   config = C2 | NS16 | NS16X | C3 | C3S | C4 (bench.py --config), C5 (tools/prof_wal.py),
#            C5A14 / C5REC / C5VER / C5WRI (one C5 call site, tools/prof_c5_part.py),
#            KV (bench.py --extra a15_kv), NS16H32 / NS16H64 (bench.py --config)
# Raw output under gpurun_out/prof_<tag>_<config>/; summarise with
#   python profiles/summarize.py <tag> <config>
set -euo pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02}
CFG=${2:-C2}
shift 2 || true
if [ "$CFG" = "C5" ]; then
  PROG="tools/prof_wal.py ${*:-}"
elif [ "${CFG#C5}" != "$CFG" ]; then  # one C5 call site: C5A14 / C5REC / C5VER / C5WRI
  case "$CFG" in
    C5A14) PART=a14 ;; C5REC) PART=recover ;; C5VER) PART=verify ;; *) PART=writer ;;
  esac
  PROG="tools/prof_c5_part.py $PART"
elif [ "$CFG" = "KV" ]; then  # a15 per-KV protection (bench.py's a15_kv extra)
  PROG="bench.py --extra a15_kv --steps 10 --warmup 3"
else
  PROG="bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline --no-extras ${*:-}"
fi
OUT=gpurun_out/prof_${TAG}_${CFG}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv \
  -- python3 $PROG > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv \
  -- python3 $PROG > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv \
  -- python3 $PROG > "$OUT/write.log" 2>&1
echo "profile $TAG $CFG done"

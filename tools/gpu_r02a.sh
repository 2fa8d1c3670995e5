#!/bin/bash
# round-2 first GPU pass: parity suite on the product library, smoke, the
# rows-vs-v2 A/B (diagnostics library) at C2/NS16/C4, then the default bench.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02a
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -20 "$OUT/smoke.log"; exit 1; }
for m in verify compute; do
  timeout -k 10 400 python -u tools/ab_bench.py --config C2 --config NS16 --config C4 --mode $m \
    --rounds 4 --reps 5 --var FORST_CRC_VARIANT=rows --var FORST_CRC_VARIANT=v2 \
    > "$OUT/ab_$m.log" 2>&1 || { tail -20 "$OUT/ab_$m.log"; exit 1; }
done
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --rounds 3 --reps 5 \
  --var FORST_CRC_VARIANT=rows_probe_load --var FORST_CRC_VARIANT=probe_load \
  > "$OUT/ab_probe.log" 2>&1 || { tail -20 "$OUT/ab_probe.log"; exit 1; }
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"

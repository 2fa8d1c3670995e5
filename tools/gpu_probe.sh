set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/probe
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --config NS16 --config C64 --var FORST_CRC_VARIANT= --var FORST_CRC_VARIANT=probe_load --var FORST_CRC_VARIANT=v1 > gpurun_out/probe/ab.log 2>&1 || { tail -20 gpurun_out/probe/ab.log; exit 1; }
cat gpurun_out/probe/ab.log

set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/v3
FORST_CRC_VARIANT=${PARITY_VARIANT:-} timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v3/pytest.log 2>&1 || { tail -40 gpurun_out/v3/pytest.log; exit 1; }
tail -1 gpurun_out/v3/pytest.log
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --config NS16 --config C3CRC --config DEV4 --config C64 --var FORST_CRC_VARIANT= --var FORST_CRC_VARIANT=v2 --var FORST_CRC_VARIANT=rows > gpurun_out/v3/ab.log 2>&1 || { tail -20 gpurun_out/v3/ab.log; exit 1; }

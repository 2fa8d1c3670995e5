set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/xx
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xx/pytest.log 2>&1 || { tail -40 gpurun_out/xx/pytest.log; exit 1; }
tail -1 gpurun_out/xx/pytest.log
timeout -k 10 300 python -u tools/ab_bench.py --config NS16X --config C3 --config X4 --config X64 --var FORST_XXH3_VARIANT= --var FORST_XXH3_VARIANT=v1 --var FORST_XXH3_VARIANT=probe_load > gpurun_out/xx/ab.log 2>&1 || { tail -20 gpurun_out/xx/ab.log; exit 1; }

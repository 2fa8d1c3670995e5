# C5 A/B of the current build against HEAD's (tools: ab_multi.sh) + kernel traces of both (recovery call site)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wal_recover.py tests/test_wal_golden.py tests/test_gpu_parity.py -m gpu -k "wal or recover or raw or c5" > gpurun_out/t_rec.log 2>&1
bash tools/ab_multi.sh abshort4 C5 forst_amd/lib/libforst_checksum.so forst_amd/lib/libforst_checksum_prev.so > gpurun_out/abshort4.txt 2>&1
export TMPDIR=/tmp
for L in libforst_checksum libforst_checksum_prev; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$L -o trace --output-format csv -- python3 tools/with_lib.py forst_amd/lib/$L.so tools/prof_c5_part.py recover > gpurun_out/tr_$L.log 2>&1
done

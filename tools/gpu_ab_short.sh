# C5 A/B of the current build against the previous commit's (tools: ab_multi.sh) + kernel traces of both (recovery and a14 call sites)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wal_recover.py tests/test_wal_golden.py tests/test_gpu_parity.py -m gpu -k "wal or recover or raw or c5 or xxh3" > gpurun_out/t_rec.log 2>&1
bash tools/ab_multi.sh abshort4 C5 forst_amd/lib/libforst_checksum.so forst_amd/lib/libforst_checksum_prev.so > gpurun_out/abshort4.txt 2>&1
export TMPDIR=/tmp
for L in libforst_checksum libforst_checksum_prev; do
  for P in recover a14; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_${L}_$P -o trace --output-format csv -- python3 tools/with_lib.py forst_amd/lib/$L.so tools/prof_c5_part.py $P > gpurun_out/tr_${L}_$P.log 2>&1
  done
done

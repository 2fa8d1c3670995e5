set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/pmc_sq.sh c2v2 C2 && bash tools/pmc_sq.sh c2v1 C2 FORST_CRC_VARIANT=v1 && bash tools/pmc_sq.sh ns16v2 NS16

set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/pmc_sq.sh c2v2b C2 && bash tools/pmc_sq.sh ns16v2b NS16

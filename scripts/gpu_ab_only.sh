# A/B kernel timing only (no tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
OPS="${OPS:-1 15}" bash scripts/gpu_ab.sh

# round-4 PMC traffic passes on the final build: C2 and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c2 TAG=r4pmcf KERNELS="validate_kernel walk_kernel" bash scripts/gpu_pmc_traffic.sh || exit 1
CFG=c4 TAG=r4pmcf BENCH_ARGS="--full-check 0" KERNELS="ws_lane_kernel validate_kernel walk_kernel" bash scripts/gpu_pmc_traffic.sh

# round-4 PMC traffic passes (FETCH_SIZE, WRITE_SIZE, L2 hits): C2, C3, C5
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c2 TAG=r4pmc KERNELS="validate_kernel walk_kernel" bash scripts/gpu_pmc_traffic.sh || exit 1
CFG=c3 TAG=r4pmc BENCH_ARGS="--full-check 0" bash scripts/gpu_pmc_traffic.sh || exit 1
CFG=c5 TAG=r4pmc BENCH_ARGS="--full-check 0" KERNELS="decomp_lane_kernel ws_lane_kernel decomp_wave_kernel validate_kernel walk_kernel" bash scripts/gpu_pmc_traffic.sh || exit 1

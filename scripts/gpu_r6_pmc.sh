# Round 6 final PMC: FETCH_SIZE / WRITE_SIZE / L2 hits of one step of C1..C5 on the
# round's library (separate passes per counter set, scripts/gpu_pmc_traffic.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
python -c "from redpanda_amd import engine; print('lib', engine.library_hash())"
CFG=c1 TAG=r6pmc KERNELS="validate_kernel walk_kernel" bash scripts/gpu_pmc_traffic.sh > gpurun_out/r6pmc_c1_summary.txt 2>&1 || { tail -5 gpurun_out/r6pmc_c1_summary.txt; exit 1; }
CFG=c2 TAG=r6pmc KERNELS="validate_kernel walk_kernel" bash scripts/gpu_pmc_traffic.sh > gpurun_out/r6pmc_c2_summary.txt 2>&1 || { tail -5 gpurun_out/r6pmc_c2_summary.txt; exit 1; }
CFG=c3 TAG=r6pmc KERNELS="lz_lane_kernel validate_kernel" bash scripts/gpu_pmc_traffic.sh > gpurun_out/r6pmc_c3_summary.txt 2>&1 || { tail -5 gpurun_out/r6pmc_c3_summary.txt; exit 1; }
CFG=c5 TAG=r6pmc BENCH_ARGS="--full-check 0" KERNELS="part_kernel lz_lane_kernel ws_lane_kernel zblk_entropy_g_kernel zblk_exec_kernel" bash scripts/gpu_pmc_traffic.sh > gpurun_out/r6pmc_c5_summary.txt 2>&1 || { tail -5 gpurun_out/r6pmc_c5_summary.txt; exit 1; }
CFG=c4 TAG=r6pmc KERNELS="ws_lane_kernel validate_kernel" bash scripts/gpu_pmc_traffic.sh > gpurun_out/r6pmc_c4_summary.txt 2>&1 || { tail -5 gpurun_out/r6pmc_c4_summary.txt; exit 1; }
for f in gpurun_out/r6pmc_c*_summary.txt; do tail -n 3 $f; done

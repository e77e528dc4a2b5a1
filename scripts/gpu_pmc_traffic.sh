# HBM traffic (FETCH_SIZE, WRITE_SIZE) and L2 hit counts of one bench config, separate passes: CFG, TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}; TAG=${TAG:-pmc}
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/${TAG}_${CFG}/p$i -o pmc -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_${CFG}_p$i.json 2> gpurun_out/${TAG}_${CFG}_p$i.err || { tail -5 gpurun_out/${TAG}_${CFG}_p$i.err; exit 1; }
done
for k in ${KERNELS:-decomp_lane_kernel validate_kernel walk_kernel}; do
  echo "== $k"; python scripts/pmc_summary.py gpurun_out/${TAG}_${CFG} $k 1
done

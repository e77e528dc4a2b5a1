# Every config's bench line; C3/C4/C5 under rocprofv3 kernel trace (stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r08}
STEPS=${STEPS:-10}
for cfg in ${CFGS:-c2 c1}; do
  timeout -k 10 400 python bench.py --config $cfg > gpurun_out/${TAG}_${cfg}_bench.json 2> gpurun_out/${TAG}_${cfg}_bench.err || { tail -20 gpurun_out/${TAG}_${cfg}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_${cfg}_bench.json
done
for cfg in ${PCFGS:-c3 c4 c5}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${cfg}_prof -o run -- python bench.py --config $cfg --steps $STEPS --warmup 2 > gpurun_out/${TAG}_${cfg}_bench.json 2> gpurun_out/${TAG}_${cfg}_bench.err || { tail -20 gpurun_out/${TAG}_${cfg}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_${cfg}_bench.json
  f=$(find gpurun_out/${TAG}_${cfg}_prof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/${TAG}_${cfg}_kernel_stats.csv
done

# full GPU parity suite, then C3/C4/C5 benches under the kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r09}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-c3 c4 c5}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${cfg}_prof -o run -- python bench.py --config $cfg --steps 5 --warmup 1 > gpurun_out/${TAG}_${cfg}_bench.json 2> gpurun_out/${TAG}_${cfg}_bench.err || { tail -20 gpurun_out/${TAG}_${cfg}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_${cfg}_bench.json
  f=$(find gpurun_out/${TAG}_${cfg}_prof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/${TAG}_${cfg}_kernel_stats.csv
done

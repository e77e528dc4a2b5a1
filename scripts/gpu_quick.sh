# GPU tests, then kernel time for ops=1 and ops=15
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for ops in ${OPS:-1 15}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ops $ops $EXTRA > gpurun_out/var_$ops.json 2> gpurun_out/var_$ops.err || { tail -5 gpurun_out/var_$ops.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/var_$ops.json'));print($ops, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['all_verdicts_ok'])"
done

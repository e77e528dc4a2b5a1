# GPU tests, then kernel time for ops=1 and ops=15, then the stamps build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for ops in 1 15; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ops $ops > gpurun_out/var_$ops.json 2> gpurun_out/var_$ops.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/var_$ops.json'));print($ops, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['all_verdicts_ok'])"
done
[ -f build/diag/librpgpu_STAMPS.so ] && OPS="${STAMP_OPS:-1 15}" bash scripts/gpu_stamps.sh

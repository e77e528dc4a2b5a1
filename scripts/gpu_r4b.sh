# round 4: walk-overlap parity, then C2 A/B: side by side (default) vs 16 chunks vs blocks per CU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_configs.py > gpurun_out/r4b_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4b_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in "side:" "chunk16:--walk-chunks 16" "side4:--blocks-per-cu 4" "side6:--blocks-per-cu 6"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $args > gpurun_out/r4b_$name.json 2> gpurun_out/r4b_$name.err || { tail -3 gpurun_out/r4b_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4b_$name.json'));print('$name', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verdicts_rank0'])"
done
done

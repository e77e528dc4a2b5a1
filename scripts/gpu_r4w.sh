# snappy parts on the main stream: decompress GPU tests, C5 A/B (interleaved twice, full check on the first), C3
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_decomp.py tests/test_gpu_bench_configs.py > gpurun_out/r4w_pytest.log 2>&1 || { tail -30 gpurun_out/r4w_pytest.log; exit 1; }
tail -2 gpurun_out/r4w_pytest.log
run() {  # name, lib, args
  if [ -n "$2" ]; then export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/$2; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 400 python bench.py --warmup 1 --no-cpu-baseline $3 > gpurun_out/r4w_$1.json 2> gpurun_out/r4w_$1.err || { tail -3 gpurun_out/r4w_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4w_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'], (d.get('full_check') or {}).get('mismatched_batches'))"
}
run c5_new_1 "" "--config c5 --steps 5" && run c5_prev_1 build/ab/librpgpu_prev.so "--config c5 --steps 5 --full-check 0" || exit 1
run c5_new_2 "" "--config c5 --steps 5 --full-check 0" && run c5_prev_2 build/ab/librpgpu_prev.so "--config c5 --steps 5 --full-check 0" || exit 1
run c3_new "" "--config c3 --steps 5 --full-check 0"

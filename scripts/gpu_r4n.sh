# zstd ring extDict restatement: decompress GPU tests incl. the crafted ring frames, C4 / C5 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_decomp.py tests/test_gpu_bench_configs.py > gpurun_out/r4n_pytest.log 2>&1 || { tail -30 gpurun_out/r4n_pytest.log; exit 1; }
tail -2 gpurun_out/r4n_pytest.log
run() {  # name, args
  timeout -k 10 400 python bench.py --warmup 1 --no-cpu-baseline --full-check 0 $2 > gpurun_out/r4n_$1.json 2> gpurun_out/r4n_$1.err || { tail -3 gpurun_out/r4n_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4n_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
run c4 "--config c4 --steps 3" && run c5 "--config c5 --steps 5"

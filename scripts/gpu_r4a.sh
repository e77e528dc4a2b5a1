# round 4: decompress parity, then a C3 bench step (each bounded)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_decomp.py tests/test_gpu_bench_configs.py tests/test_segment_parse.py > gpurun_out/r4a_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r4a_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4a_c3.json 2> gpurun_out/r4a_c3.err
rc=$?; tail -2 gpurun_out/r4a_c3.err; python -c "import json;d=json.load(open('gpurun_out/r4a_c3.json'));print('c3', d['ms_per_step'], d['roofline']['kernel_ms'], d['decompress_verdicts_rank0'])"
exit $rc

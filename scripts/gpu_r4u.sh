# split fallbacks below the wave size decoded by the LZ wave decoder: decompress GPU tests, C5 full oracle check
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4final
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_decomp.py tests/test_gpu_bench_configs.py > gpurun_out/r4u_pytest.log 2>&1 || { tail -30 gpurun_out/r4u_pytest.log; exit 1; }
tail -2 gpurun_out/r4u_pytest.log
timeout -k 10 400 python bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/r4final/c5.json 2> gpurun_out/r4final/c5.err || { tail -5 gpurun_out/r4final/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4final/c5.json'));print('c5', d['value'], d['ms_per_step'], d['cpu_baseline']['value'], d['full_check']['mismatched_batches'])"
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 1 > gpurun_out/r4final/c3.json 2> gpurun_out/r4final/c3.err || { tail -5 gpurun_out/r4final/c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4final/c3.json'));print('c3', d['value'], d['ms_per_step'], d['cpu_baseline']['value'])"

# after the 80 KiB split threshold: decompress GPU tests, C5 bench line with its CPU baseline and trace, PMC C2 / C4 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4final
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_decomp.py tests/test_gpu_bench_configs.py tests/test_gpu_wave_walk.py > gpurun_out/r4final_e_pytest.log 2>&1 || { tail -30 gpurun_out/r4final_e_pytest.log; exit 1; }
tail -2 gpurun_out/r4final_e_pytest.log
timeout -k 10 400 python bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/r4final/c5.json 2> gpurun_out/r4final/c5.err || { tail -5 gpurun_out/r4final/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4final/c5.json'));print('c5', d['value'], d['ms_per_step'], d['cpu_baseline']['value'])"
CFG=c5 TAG=r4final STEPS=2 LIMIT=400 BENCH_ARGS="--full-check 0" bash scripts/gpu_prof.sh > /dev/null || exit 1
CFG=c2 TAG=r4pmcf KERNELS="validate_kernel walk_kernel" bash scripts/gpu_pmc_traffic.sh > /dev/null || exit 1
CFG=c5 TAG=r4pmcf BENCH_ARGS="--full-check 0" KERNELS="ws_lane_kernel" bash scripts/gpu_pmc_traffic.sh > /dev/null || exit 1
CFG=c4 TAG=r4pmcf BENCH_ARGS="--full-check 0" KERNELS="ws_lane_kernel" bash scripts/gpu_pmc_traffic.sh > /dev/null

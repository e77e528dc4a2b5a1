# stride-guess wave walk: parity, then C5 overlap off / on and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wave_walk.py tests/test_gpu_parity.py tests/test_gpu_bench_configs.py tests/test_gpu_decomp.py > gpurun_out/r4i_pytest.log 2>&1 || { tail -30 gpurun_out/r4i_pytest.log; exit 1; }
tail -2 gpurun_out/r4i_pytest.log
for v in "c5off:--config c5 --overlap off" "c5on:--config c5 --overlap on" "c2:--config c2" "c2b:--config c2"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-check 0 $args > gpurun_out/r4i_$name.json 2> gpurun_out/r4i_$name.err || { tail -3 gpurun_out/r4i_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4i_$name.json'));print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
done

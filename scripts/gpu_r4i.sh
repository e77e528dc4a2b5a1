# stride-guess wave walk: parity, then C5 overlap off / on, C2 chunk rounds A/B and chunk counts
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wave_walk.py tests/test_gpu_parity.py tests/test_gpu_bench_configs.py tests/test_gpu_decomp.py > gpurun_out/r4i_pytest.log 2>&1 || { tail -30 gpurun_out/r4i_pytest.log; exit 1; }
tail -2 gpurun_out/r4i_pytest.log
run() {  # name, args
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-check 0 $2 > gpurun_out/r4i_$1.json 2> gpurun_out/r4i_$1.err || { tail -3 gpurun_out/r4i_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4i_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
run c5off "--config c5 --overlap off" && run c5on "--config c5 --overlap on" || exit 1
for rep in 1 2; do
  unset RPGPU_DIAG_LIB; run c2_rounds_$rep "--config c2" || exit 1
  export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/build/ab/librpgpu_norounds.so; run c2_norounds_$rep "--config c2" || exit 1
done
unset RPGPU_DIAG_LIB
for k in 8 12 24; do run c2_k$k "--config c2 --walk-chunks $k" || exit 1; done

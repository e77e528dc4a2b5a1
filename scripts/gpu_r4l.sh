# index_first written by the walk, the plan beside the first checksum chunk: GPU suite, then C2 A/B against the
# previous library (same bench: plan + run in rpgpu_validate_device), C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4l_pytest.log 2>&1 || { tail -30 gpurun_out/r4l_pytest.log; exit 1; }
tail -2 gpurun_out/r4l_pytest.log
run() {  # name, args
  timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --full-check 0 $2 > gpurun_out/r4l_$1.json 2> gpurun_out/r4l_$1.err || { tail -3 gpurun_out/r4l_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4l_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  unset RPGPU_DIAG_LIB; run c2_new_$rep "--config c2" || exit 1
  export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/build/ab/librpgpu_prev.so; run c2_prev_$rep "--config c2" || exit 1
done
unset RPGPU_DIAG_LIB
STEPS=5 run c5 "--config c5"

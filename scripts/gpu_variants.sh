# C3 step time per library variant (build/var/*.so via RPGPU_DIAG_LIB) and the
# first the parity tests on the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decomp.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_decomp.log 2>&1 || { tail -20 gpurun_out/pytest_decomp.log; exit 1; }
tail -2 gpurun_out/pytest_decomp.log
CFG=${CFG:-c3}
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config $CFG --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/var_$label.json 2> gpurun_out/var_$label.err || { tail -3 gpurun_out/var_$label.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/var_$label.json')); print('$CFG $label', d['ms_per_step'], d['value'], d['roofline']['frac'])"
}
run base
for f in build/var/*.so; do
  run $(basename $f .so) RPGPU_DIAG_LIB=$PWD/$f
done

# full GPU suite with the walk overlap as the default; C4: round-3 library vs this one (same box); C2 default
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4k_pytest.log 2>&1 || { tail -30 gpurun_out/r4k_pytest.log; exit 1; }
tail -2 gpurun_out/r4k_pytest.log
run() {  # name, args
  timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 1 --no-cpu-baseline --full-check 0 $2 > gpurun_out/r4k_$1.json 2> gpurun_out/r4k_$1.err || { tail -3 gpurun_out/r4k_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4k_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
run c2 "--config c2" || exit 1
for rep in 1 2; do
  unset RPGPU_DIAG_LIB; STEPS=3 run c4_r4_$rep "--config c4 --overlap off" || exit 1
  export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/build/ab/librpgpu_r3final.so; STEPS=3 run c4_r3_$rep "--config c4 --overlap off" || exit 1
done

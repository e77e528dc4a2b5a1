# plan beside the single checksum launch of small arenas: full GPU suite, C1 A/B (interleaved twice)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4v_pytest.log 2>&1 || { tail -30 gpurun_out/r4v_pytest.log; exit 1; }
tail -2 gpurun_out/r4v_pytest.log
run() {  # name, lib
  if [ -n "$2" ]; then export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/$2; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r4v_$1.json 2> gpurun_out/r4v_$1.err || { tail -3 gpurun_out/r4v_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4v_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'], d['value'])"
}
for rep in 1 2; do run c1_new_$rep "" && run c1_prev_$rep build/ab/librpgpu_prev.so || exit 1; done

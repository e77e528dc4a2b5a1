# C4: zstd ring variants vs the previous library (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, lib
  if [ -n "$2" ]; then export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/$2; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 400 python bench.py --warmup 1 --no-cpu-baseline --full-check 0 --config c4 --steps 3 > gpurun_out/r4q_$1.json 2> gpurun_out/r4q_$1.err || { tail -3 gpurun_out/r4q_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4q_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
run prev build/ab/librpgpu_prev.so && run cur "" && run prev_b build/ab/librpgpu_prev.so && run cur_b ""

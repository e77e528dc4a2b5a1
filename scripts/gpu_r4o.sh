# C4 / C5: the zstd ring restatement vs the previous library, same box, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, args
  timeout -k 10 400 python bench.py --warmup 1 --no-cpu-baseline --full-check 0 $2 > gpurun_out/r4o_$1.json 2> gpurun_out/r4o_$1.err || { tail -3 gpurun_out/r4o_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4o_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  unset RPGPU_DIAG_LIB; run c4_new_$rep "--config c4 --steps 3" || exit 1
  export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/build/ab/librpgpu_prev.so; run c4_prev_$rep "--config c4 --steps 3" || exit 1
done
unset RPGPU_DIAG_LIB; run c5_new "--config c5 --steps 5" || exit 1
export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/build/ab/librpgpu_prev.so; run c5_prev "--config c5 --steps 5"

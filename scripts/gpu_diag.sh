set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in default NO_LOOKUP NO_COMBINE; do
  for ops in 1 15; do
    if [ $lib = default ]; then unset RPGPU_DIAG_LIB; else export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/build/diag/librpgpu_$lib.so; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ops $ops $EXTRA > gpurun_out/d.json 2> gpurun_out/d.err || { tail -3 gpurun_out/d.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/d.json'));print('$lib', $ops, d['roofline']['kernel_ms'], d['all_verdicts_ok'])"
  done
done

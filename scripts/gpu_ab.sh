# A/B kernel timing: default build vs build/ab/*.so, ops in $OPS, interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for lib in default build/ab/*.so; do
  for ops in ${OPS:-1 15}; do
    if [ $lib = default ]; then unset RPGPU_DIAG_LIB; else export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ops $ops $EXTRA > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$lib', $ops, d['roofline']['kernel_ms'], d['all_verdicts_ok'])"
  done
done
done

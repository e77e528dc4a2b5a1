# Per-phase wave-cycle attribution with the STAMPS diagnostics build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/build/diag/librpgpu_STAMPS.so
for ops in ${OPS:-1 15}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ops $ops > gpurun_out/s.json 2> gpurun_out/s.err || { tail -3 gpurun_out/s.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/s.json'));print($ops, d['roofline']['kernel_ms'], d['all_verdicts_ok'], d.get('diag_cycles_per_batch'))"
done

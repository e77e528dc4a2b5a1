set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for ops in 1 3 15; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --ops $ops > gpurun_out/var_$ops.json 2> gpurun_out/var_$ops.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/var_$ops.json'));print($ops, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done

# C2 step time under the validate / walk launch knobs (env): RUNS="label:ENV=V,ENV=V ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in $RUNS; do
  label=${r%%:*}; envs=${r#*:}
  ev=""; [ "$envs" != - ] && ev="${envs//,/ }"
  env $ev timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/k_$label.json 2> gpurun_out/k_$label.err || { tail -3 gpurun_out/k_$label.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/k_$label.json')); print('$label', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
done

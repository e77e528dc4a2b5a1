# kernel-trace stats of bench configs under library variants / env: RUNS="cfg:lib:ENV=V,ENV2=V ..." (lib "base" = default build, env "-" = none)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in $RUNS; do
  IFS=: read cfg lib envs <<< "$r"
  tag=${cfg}_${lib}_${envs//[=,]/_}
  ev=""
  [ "$lib" != base ] && ev="RPGPU_DIAG_LIB=$PWD/build/vx/librpgpu_$lib.so"
  [ "$envs" != - ] && ev="$ev ${envs//,/ }"
  env $ev timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv_$tag -o run -- python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/pv_$tag.json 2> gpurun_out/pv_$tag.err || { tail -5 gpurun_out/pv_$tag.err; exit 1; }
  f=$(find gpurun_out/pv_$tag -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/pv_${tag}_kernel_stats.csv
  echo "== $tag"
  python - gpurun_out/pv_${tag}_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(" ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e6,3), "ms", r["Percentage"])
PY
  python -c "import json; d=json.load(open('gpurun_out/pv_$tag.json')); print('  step', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done

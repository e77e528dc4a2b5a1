# round-4 final bench lines: every config with its pinned CPU baseline; C3 alnum; C2 without the overlap
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4final
export TMPDIR=/tmp
run() {  # name, limit, args
  timeout -k 10 $2 python bench.py $3 > gpurun_out/r4final/$1.json 2> gpurun_out/r4final/$1.err || { tail -5 gpurun_out/r4final/$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4final/$1.json'));print('$1', d['value'], d['unit'], d['ms_per_step'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
}
run c2 300 "--config c2" && run c1 300 "--config c1" && run c3 400 "--config c3 --steps 5 --warmup 1" \
  && run c5 400 "--config c5 --steps 5 --warmup 1" && run c4 400 "--config c4 --steps 3 --warmup 1" \
  && run c3_alnum 300 "--config c3 --steps 5 --warmup 1 --payload alnum --no-cpu-baseline" \
  && run c2_nooverlap 300 "--config c2 --overlap off --no-cpu-baseline"

# round-5 final (b): bench lines of every config with its pinned CPU baseline (C5: every batch against the oracle)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5final
export TMPDIR=/tmp
run() {  # name, limit, args
  timeout -k 10 $2 python bench.py $3 > gpurun_out/r5final/$1.json 2> gpurun_out/r5final/$1.err || { tail -5 gpurun_out/r5final/$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5final/$1.json'));print('$1', d['value'], d['unit'], d['ms_per_step'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'), d.get('gpu_matches_oracle_on_all_batches', d.get('gpu_matches_oracle_on_sample')))"
}
run c2 300 "--config c2" && run c1 300 "--config c1" && run c3 400 "--config c3 --steps 5 --warmup 2" \
  && run c5 500 "--config c5 --steps 5 --warmup 2" && run c4 400 "--config c4 --steps 3 --warmup 1"

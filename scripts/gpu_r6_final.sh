# Round 6 final: bench lines of every config with its CPU baseline (C5 and C3: every
# batch against the oracle), then kernel traces + stats of each config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUTTAG:-r6final}
mkdir -p $O
python -c "from redpanda_amd import engine; print('lib', engine.library_hash())"
run() {  # name, limit, args
  timeout -k 10 $2 python -u bench.py $3 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));r=d['roofline'];print('$1', d['value'], d['unit'], d['ms_per_step'], r['frac'], r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), d.get('gpu_matches_oracle_on_all_batches', d.get('gpu_matches_oracle_on_sample')))"
}
run c2 300 "--config c2" && run c1 300 "--config c1" && run c3 500 "--config c3 --steps 5 --warmup 2 --full-check 1" \
  && run c5 500 "--config c5 --steps 5 --warmup 2" && run c4 500 "--config c4 --steps 3 --warmup 1" || exit 1
CFG=c2 TAG=${OUTTAG:-r6final}/prof STEPS=10 LIMIT=300 bash scripts/gpu_prof.sh || exit 1
for c in c3 c5 c4; do CFG=$c TAG=${OUTTAG:-r6final}/prof STEPS=2 LIMIT=400 BENCH_ARGS="--full-check 0" bash scripts/gpu_prof.sh || exit 1; done

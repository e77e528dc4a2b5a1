# kernel-trace stats of one bench config (CFG, TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}; TAG=${TAG:-prof}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${CFG}_prof -o run -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_${CFG}.json 2> gpurun_out/${TAG}_${CFG}.err || { tail -5 gpurun_out/${TAG}_${CFG}.err; exit 1; }
f=$(find gpurun_out/${TAG}_${CFG}_prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${TAG}_${CFG}_kernel_stats.csv
python - <<PY
import csv
rows=list(csv.DictReader(open("gpurun_out/${TAG}_${CFG}_kernel_stats.csv")))
for r in rows[:12]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e6,3), "ms", r["Percentage"])
PY
cat gpurun_out/${TAG}_${CFG}.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['value'], d['roofline']['frac'])"

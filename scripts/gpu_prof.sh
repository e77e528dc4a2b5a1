# kernel trace + stats of a short bench run: CFG, TAG, STEPS, BENCH_ARGS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}; TAG=${TAG:-prof}
timeout -k 10 ${LIMIT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${CFG} -o run -- python bench.py --config $CFG --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_${CFG}.json 2> gpurun_out/${TAG}_${CFG}.err
rc=$?
f=$(find gpurun_out/${TAG}_${CFG} -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>6s} avg {float(r["AverageNs"])/1e6:9.3f} ms total {float(r["TotalDurationNs"])/1e6:9.2f} ms')
PY
exit $rc

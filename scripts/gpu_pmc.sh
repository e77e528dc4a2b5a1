# HBM traffic per kernel: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c2}
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${CFG}_$ctr -o pmc -- python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${CFG}_$ctr.json 2> gpurun_out/pmc_${CFG}_$ctr.err || { tail -20 gpurun_out/pmc_${CFG}_$ctr.err; exit 1; }
  f=$(find gpurun_out/pmc_${CFG}_$ctr -name "*counter_collection.csv" | head -1)
  python - "$f" $ctr <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    acc[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if "rpgpu" in k:
        print(sys.argv[2], k, "dispatches", len(v), "avg", sum(v) / len(v))
PY
done

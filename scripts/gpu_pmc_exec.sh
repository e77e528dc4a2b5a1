# SQ counters of the two-phase LZ kernels on a small C3 arena (separate passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmcx}
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python bench.py --config c3 --batches 16384 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_p$i.json 2> gpurun_out/${TAG}_p$i.err || { tail -5 gpurun_out/${TAG}_p$i.err; exit 1; }
done
python - <<PY
import csv, glob, collections
agg = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/${TAG}_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "lz_exec" in k or "decomp_lane" in k:
            agg[k[:40]][r["Counter_Name"]] = agg[k[:40]].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   ", c, int(v))
PY

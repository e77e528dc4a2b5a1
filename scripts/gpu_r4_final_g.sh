# final C5 bench line (CPU baseline, full oracle check) and kernel trace on the final build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4final
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/r4final/c5.json 2> gpurun_out/r4final/c5.err || { tail -5 gpurun_out/r4final/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4final/c5.json'));print('c5', d['value'], d['ms_per_step'], d['cpu_baseline']['value'], d['full_check']['mismatched_batches'])"
CFG=c5 TAG=r4final STEPS=2 LIMIT=400 BENCH_ARGS="--full-check 0" bash scripts/gpu_prof.sh > /dev/null

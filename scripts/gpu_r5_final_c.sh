# round-5 final (c): kernel traces + stats (C2 10 steps; C3 / C5 / C4 2 steps), C3 twice more, PMC traffic of C2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5final
export TMPDIR=/tmp
CFG=c2 TAG=r5final STEPS=10 LIMIT=300 bash scripts/gpu_prof.sh || exit 1
for c in c3 c5 c4; do CFG=$c TAG=r5final STEPS=2 LIMIT=400 BENCH_ARGS="--full-check 0" bash scripts/gpu_prof.sh || exit 1; done
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5final/c3_again_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r5final/c3_again_$i.json'));print('c3 again', d['ms_per_step'], d['value'])"
done
CFG=c2 TAG=r5pmc KERNELS="validate_kernel walk_kernel" bash scripts/gpu_pmc_traffic.sh || exit 1

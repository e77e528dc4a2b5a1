# C2 attribution: validate only (ops 3) vs the full pipeline, plus a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "full:" "ops3:--ops 3" "ops1:--ops 1"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $args > gpurun_out/r4c_$name.json 2> gpurun_out/r4c_$name.err || { tail -3 gpurun_out/r4c_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4c_$name.json'));print('$name', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
STEPS=5 TAG=r4c CFG=c2 LIMIT=300 bash scripts/gpu_prof.sh

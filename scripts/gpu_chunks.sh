# run time vs overlap chunking (RPGPU_RUN_CHUNKS) and grid
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "4 0 1" "8 0 1" "4 1 4" "4 1 16" "4 1 64" "8 1 16" "8 1 64" "2 1 64"; do
  set -- $cfg
  if [ $2 = 1 ]; then export RPGPU_OVERLAP=1; else unset RPGPU_OVERLAP; fi
  RPGPU_BLOCKS_PER_CU=$1 RPGPU_RUN_CHUNKS=$3 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ch.json 2> gpurun_out/ch.err || { tail -5 gpurun_out/ch.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ch.json'));print('bpc $1 overlap $2 chunks $3', d['roofline']['kernel_ms'], d['roofline']['frac'], d['all_verdicts_ok'])"
done

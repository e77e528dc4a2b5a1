# Round 6, call f: C4 / C5 / C3 with the computed zstd baselines (ll_x / ml_x);
# C2 with 4 / 2 / 1 batches per partition per summary workgroup.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6f
mkdir -p $O
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
}
run c4a --config c4 --steps 3 --warmup 1
run c4b --config c4 --steps 3 --warmup 1
run c5 --config c5 --steps 3 --warmup 1 --full-check 0
run c3 --config c3 --steps 5 --warmup 1
for pp in 4 2 1; do
  RPGPU_SUM_PER_PART=$pp run c2_pp$pp --config c2 --steps 20 --warmup 3
done

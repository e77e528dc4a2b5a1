# Round 6, call hh: C2 with both streams at the default priority (RPGPU_MAIN_PRIORITY=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6hh
mkdir -p $O
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --config c2 --steps 20 --warmup 3 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
}
run base
RPGPU_MAIN_PRIORITY=0 run prio0
run base2
RPGPU_MAIN_PRIORITY=0 run prio0b

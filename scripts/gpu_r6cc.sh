# Round 6, call cc: C5 / C3 with fewer walk-overlap chunks for the input validation
# (runtime field; C5's log-uniform batch sizes make each chunk wait for its largest batch).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6cc
mkdir -p $O
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
C5="--config c5 --steps 3 --warmup 1 --full-check 0"
run c5 $C5
for w in 1 2 4 8; do run c5_wc$w $C5 --walk-chunks $w; done
run c5b $C5
run c3 --config c3 --steps 5 --warmup 1
run c3_wc4 --config c3 --steps 5 --warmup 1 --walk-chunks 4

# Round 6, call aa: C2 over the runtime tuning fields (workgroups per CU, walk chunks).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6aa
mkdir -p $O
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --config c2 --steps 20 --warmup 3 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
}
run base
for b in 3 5 6 8; do run bpc$b --blocks-per-cu $b; done
for w in 12 14 18; do run wc$w --walk-chunks $w; done
run base2

# Round 6, call ff: the part kernel on a default-priority stream (RPGPU_PARTS_LOWPRIO=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ff
mkdir -p $O
run() {  # tag, lib ('' = the library), args...
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RPGPU_DIAG_LIB=$lib; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
C5="--config c5 --steps 3 --warmup 1 --full-check 0"
V=build/vx/librpgpu_RPGPU_PARTS_LOWPRIO_1.so
run base "" $C5
run lp $V $C5
run base2 "" $C5
run lp2 $V $C5
run c3_lp $V --config c3 --steps 5 --warmup 1
export RPGPU_DIAG_LIB=$V
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python -u bench.py --no-cpu-baseline $C5 > $O/tl.json 2> $O/tl.err || { tail -5 $O/tl.err; exit 1; }
python scripts/timeline_db.py $(find $O/prof -name "*.db") 2 > $O/timeline.txt

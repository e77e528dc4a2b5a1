# Round 6, call o: the library with HBM entropy workspaces, the LZ4 lanes on the second
# stream and the 64 KiB block-parallel threshold: C5 (and with the snappy lanes on the
# main stream), C3 and C4 for regressions.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6o
mkdir -p $O
run() {  # tag, lib ('' = the library), args...
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RPGPU_DIAG_LIB=$lib; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
C5="--config c5 --steps 3 --warmup 1 --full-check 0"
V=build/vx/librpgpu_RPGPU_SNAPPY_LANE_AUX_0.so
run c5 "" $C5
run c5_snappy_main $V $C5
run c5b "" $C5
run c5_snappy_main_b $V $C5
run c3 "" --config c3 --steps 5 --warmup 1
run c4 "" --config c4 --steps 3 --warmup 1
export RPGPU_DIAG_LIB=$V
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python -u bench.py --no-cpu-baseline $C5 > $O/tl.json 2> $O/tl.err || { tail -5 $O/tl.err; exit 1; }
python scripts/timeline_db.py $(find $O/prof -name "*.db") 2 > $O/timeline.txt

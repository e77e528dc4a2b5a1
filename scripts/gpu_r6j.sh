# Round 6, call j/k: C5 under variant libraries (build/vx, RPGPU_DIAG_LIB):
# the zstd block-parallel threshold, the two-launch part kernels, the third stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUTTAG:-r6j}
mkdir -p $O
run() {  # tag, lib ('' = the library), args...
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RPGPU_DIAG_LIB=$lib; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
C5="--config c5 --steps 3 --warmup 1 --full-check 0"
run base "" $C5
for v in RPGPU_LZ4_LANE_AUX_1 RPGPU_ZSTD_BLK_MIN_65536 RPGPU_LZ4_LANE_AUX_1_RPGPU_ZSTD_BLK_MIN_65536; do
  run $v build/vx/librpgpu_$v.so $C5
done
run base2 "" $C5
if [ -n "$TL_LIB" ]; then
  export RPGPU_DIAG_LIB=$TL_LIB
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python -u bench.py --no-cpu-baseline $C5 > $O/tl.json 2> $O/tl.err || { tail -5 $O/tl.err; exit 1; }
  python scripts/timeline_db.py $(find $O/prof -name "*.db") 2 > $O/timeline.txt
fi

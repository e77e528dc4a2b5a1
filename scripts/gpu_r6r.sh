# Round 6, call r: the zstd lane kernel at 3 / 4 waves per SIMD (VGPRs capped, more
# lanes in flight) on C4 and C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6r
mkdir -p $O
run() {  # tag, lib ('' = the library), args...
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RPGPU_DIAG_LIB=$lib; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
C4="--config c4 --steps 3 --warmup 1"
C5="--config c5 --steps 3 --warmup 1 --full-check 0"
V3=build/vx/librpgpu_RPGPU_WS_WAVES_3_RPZ_LANES_196608.so
V4=build/vx/librpgpu_RPGPU_WS_WAVES_4_RPZ_LANES_262144.so
run c4 "" $C4
run c4_w3 $V3 $C4
run c4_w4 $V4 $C4
run c5 "" $C5
run c5_w3 $V3 $C5
run c5_w4 $V4 $C5

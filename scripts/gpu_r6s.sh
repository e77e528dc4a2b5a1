# Round 6, call s: geometric checksum / walk chunks (RPGPU_CHUNK_RATIO) on C2; decompress
# tests on the library with the block pool scaled by the arena.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_decomp.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, lib ('' = the library), args...
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RPGPU_DIAG_LIB=$lib; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
}
C2="--config c2 --steps 20 --warmup 3"
V=build/vx/librpgpu_RPGPU_CHUNK_RATIO_
run base "" $C2
run r950 ${V}950.so $C2
run r920 ${V}920.so $C2
run r880 ${V}880.so $C2
run base2 "" $C2
run r920_20 ${V}920.so $C2 --walk-chunks 20
run r920_24 ${V}920.so $C2 --walk-chunks 24
run r920b ${V}920.so $C2

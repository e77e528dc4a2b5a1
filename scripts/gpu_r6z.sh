# Round 6, call z: the zstd workspaces' FSE tables in the 16-bit form (RPZ_WS16=1):
# zstd decompress tests on that library, C4 and C5 against the library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6z
mkdir -p $O
V=build/vx/librpgpu_RPZ_WS16_1.so
RPGPU_DIAG_LIB=$V timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_decomp.py -k "zstd or c5_shaped or generated or mutated" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, lib ('' = the library), args...
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RPGPU_DIAG_LIB=$lib; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
C4="--config c4 --steps 3 --warmup 1"
C5="--config c5 --steps 3 --warmup 1 --full-check 0"
run c4 "" $C4
run c4_16 $V $C4
run c4b "" $C4
run c4_16b $V $C4
run c5 "" $C5
run c5_16 $V $C5

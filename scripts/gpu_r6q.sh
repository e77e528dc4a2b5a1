# Round 6, call q: the LZ4 + snappy lane batches from the plan's lists in one launch
# (lz_lane_kernel): decompress tests, C5 and C3 against the per-codec kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6q
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_decomp.py tests/test_gpu_bench_configs.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, lib ('' = the library), args...
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RPGPU_DIAG_LIB=$lib; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
C5="--config c5 --steps 3 --warmup 1 --full-check 0"
V=build/vx/librpgpu_RPGPU_LZ_LANE_LIST_0.so
run c5 "" $C5
run c5_old $V $C5
run c5b "" $C5
run c5_old_b $V $C5
run c3 "" --config c3 --steps 5 --warmup 1
run c3_old $V --config c3 --steps 5 --warmup 1
unset RPGPU_DIAG_LIB
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python -u bench.py --no-cpu-baseline $C5 > $O/tl.json 2> $O/tl.err || { tail -5 $O/tl.err; exit 1; }
python scripts/timeline_db.py $(find $O/prof -name "*.db") 2 > $O/timeline.txt

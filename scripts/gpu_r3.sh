# GPU tests, then the C2 bench and the C3 (LZ4 decompress) bench, text and alnum
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -20 gpurun_out/c2.err; exit 1; }
cat gpurun_out/c2.json
timeout -k 10 600 python bench.py --config c3 --steps 5 --warmup 1 > gpurun_out/c3_text.json 2> gpurun_out/c3_text.err || { tail -20 gpurun_out/c3_text.err; exit 1; }
cat gpurun_out/c3_text.json
timeout -k 10 600 python bench.py --config c3 --payload alnum --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c3_alnum.json 2> gpurun_out/c3_alnum.err || { tail -20 gpurun_out/c3_alnum.err; exit 1; }
cat gpurun_out/c3_alnum.json

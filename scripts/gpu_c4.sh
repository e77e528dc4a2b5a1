# GPU decompress parity tests, then the C4 (zstd) bench and its kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_decomp.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_decomp.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_decomp.log | head -40; exit $rc; }
timeout -k 10 500 python -u bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
cat gpurun_out/c4.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c4.json 2> gpurun_out/prof_c4.err || { tail -20 gpurun_out/prof_c4.err; exit 1; }
cut -d, -f1-4 gpurun_out/prof_c4/c4_kernel_stats.csv | sed 's/(.*)//' | head -6

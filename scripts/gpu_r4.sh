# GPU suite, smoke, C2/C3/C4 benches and rocprofv3 kernel stats of C2 and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -40; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -20 gpurun_out/c2.err; exit 1; }
cat gpurun_out/c2.json
timeout -k 10 500 python -u bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
cat gpurun_out/c4.json
timeout -k 10 500 python -u bench.py --config c3 --steps 5 --warmup 1 > gpurun_out/c3_text.json 2> gpurun_out/c3_text.err || { tail -20 gpurun_out/c3_text.err; exit 1; }
cat gpurun_out/c3_text.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c2.json 2> gpurun_out/prof_c2.err || { tail -20 gpurun_out/prof_c2.err; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c4.json 2> gpurun_out/prof_c4.err || { tail -20 gpurun_out/prof_c4.err; exit 1; }
for f in $(find gpurun_out/prof_c2 gpurun_out/prof_c4 -name "*kernel_stats.csv"); do echo $f; cut -d, -f1-6 "$f" | head -10; done

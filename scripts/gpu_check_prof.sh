# decompress parity tests on the default build, then kernel stats of RUNS (scripts/gpu_prof_var.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_decomp.py} -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_chk.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_chk.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_chk.log | head -20; exit $rc; }
bash scripts/gpu_prof_var.sh

# zstd change check: GPU decompress parity tests, then C4 A/B vs build/ab/*.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decomp.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_decomp.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_decomp.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_decomp.log | head -40; exit $rc; }
bash scripts/gpu_ab_c4.sh

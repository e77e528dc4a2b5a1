# ring matches decoded by a second pass over the block: decompress GPU tests, then C4 / C5 A/B against the previous library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_decomp.py > gpurun_out/r4p_pytest.log 2>&1 || { tail -30 gpurun_out/r4p_pytest.log; exit 1; }
tail -2 gpurun_out/r4p_pytest.log
bash scripts/gpu_r4o.sh

# round-4 final: full GPU suite, bench lines for every config with CPU baselines, kernel traces
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4final_pytest.log 2>&1 || { tail -30 gpurun_out/r4final_pytest.log; exit 1; }
tail -2 gpurun_out/r4final_pytest.log
bash scripts/gpu_r4_final_a.sh && bash scripts/gpu_r4_final_b.sh

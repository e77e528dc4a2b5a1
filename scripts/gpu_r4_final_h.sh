# the final build: full GPU suite and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4final_pytest.log 2>&1 || { tail -30 gpurun_out/r4final_pytest.log; exit 1; }
tail -2 gpurun_out/r4final_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final_smoke.log 2>&1 || { tail -5 gpurun_out/r4final_smoke.log; exit 1; }
tail -1 gpurun_out/r4final_smoke.log

# round-5 final (a): the full GPU suite and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5final
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5final/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5final/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r5final/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5final/smoke.log 2>&1 || { tail -10 gpurun_out/r5final/smoke.log; exit 1; }
tail -1 gpurun_out/r5final/smoke.log

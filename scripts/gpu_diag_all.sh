# Attribution run: microbenchmark stream rates, diag variants, PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 bash tools/microbench/run.sh > gpurun_out/mb.log 2>&1 || { echo mb failed; tail gpurun_out/mb.log; exit 1; }
cat gpurun_out/mb.log
bash scripts/gpu_diag.sh || exit 1
bash scripts/gpu_pmc.sh || exit 1
python scripts/pmc_summary.py gpurun_out/pmc

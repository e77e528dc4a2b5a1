# GPU tests, then run time with / without the walk overlap for several grids
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
for bpc in ${BPCS:-4 6 8}; do
  for ov in 0 1; do
    if [ $ov = 0 ]; then export RPGPU_NO_OVERLAP=1; else unset RPGPU_NO_OVERLAP; fi
    RPGPU_BLOCKS_PER_CU=$bpc timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ovl.json 2> gpurun_out/ovl.err || { tail -5 gpurun_out/ovl.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ovl.json'));print('bpc', $bpc, 'overlap', $ov, d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['all_verdicts_ok'])"
  done
done

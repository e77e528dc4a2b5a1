# GPU tests, then validate-kernel time vs workgroups per CU (RPGPU_BLOCKS_PER_CU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
for bpc in ${BPCS:-4 6 8}; do
  for ops in 1 15; do
    RPGPU_BLOCKS_PER_CU=$bpc timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ops $ops > gpurun_out/bpc.json 2> gpurun_out/bpc.err || { tail -5 gpurun_out/bpc.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bpc.json'));print('bpc', $bpc, 'ops', $ops, d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['all_verdicts_ok'])"
  done
done

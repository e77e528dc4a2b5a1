# decompress parity tests, then the C3 / C5 benches (two-phase LZ decode checks)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decomp.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_decomp.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_decomp.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-c3}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/chk_$cfg.json 2> gpurun_out/chk_$cfg.err || { tail -5 gpurun_out/chk_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/chk_$cfg.json')); print('$cfg', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('gpu_matches_oracle_on_sample'))"
done

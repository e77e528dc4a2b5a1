# decompress parity tests, then the C3 bench (text, alnum)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decomp.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_decomp.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_decomp.log
[ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_decomp.log; exit $rc; }
for pl in text alnum; do
timeout -k 10 600 python bench.py --config c3 --payload $pl --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c3_$pl.json 2> gpurun_out/c3_$pl.err || { tail -20 gpurun_out/c3_$pl.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3_$pl.json'));print('$pl', d['value'], d['logical_gbps'], d['ms_per_step'], d['roofline']['frac'], d['all_verdicts_ok'])"
done

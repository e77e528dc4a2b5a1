# wave walk parity + parity suite, then C5 / C2 with and without the walk overlap
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_wave_walk.py tests/test_gpu_parity.py tests/test_segment_parse.py tests/test_record_sets.py > gpurun_out/r4f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4f_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in "c5off:--config c5 --overlap off" "c5on:--config c5 --overlap on" "c2:--config c2"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --full-check 0 $args > gpurun_out/r4f_$name.json 2> gpurun_out/r4f_$name.err || { tail -3 gpurun_out/r4f_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4f_$name.json'));print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
done

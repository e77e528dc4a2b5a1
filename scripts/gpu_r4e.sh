# C3: window literals (default build) vs reloaded literals (variant), plus ABI/parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_abi.py tests/test_gpu_decomp.py > gpurun_out/r4e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4e_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for lib in default build/var/librpgpu_RPGPU_LZ4_WINLIT_0.so; do
  if [ $lib = default ]; then unset RPGPU_DIAG_LIB; else export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/$lib; fi
  timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r4e.json 2> gpurun_out/r4e.err || { tail -3 gpurun_out/r4e.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4e.json'));print('$lib', d['ms_per_step'], d['roofline']['kernel_ms'], d['decompress_verdicts_rank0'])"
done
done

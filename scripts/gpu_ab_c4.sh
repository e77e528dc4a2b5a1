# A/B of zstd_kernel builds on C4: default librpgpu.so vs build/ab/*.so, interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for lib in default build/ab/*.so; do
  if [ $lib = default ]; then unset RPGPU_DIAG_LIB; else export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/$lib; fi
  timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_c4.json 2> gpurun_out/ab_c4.err || { tail -5 gpurun_out/ab_c4.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_c4.json'));print('$lib', d['roofline']['kernel_ms'], d['all_verdicts_ok'])"
done
done

# C4 step time vs zstd lanes in flight (RPGPU_ZSTD_LANES)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in ${LANES:-0 65536 98304}; do
  if [ $L -eq 0 ]; then unset RPGPU_ZSTD_LANES; else export RPGPU_ZSTD_LANES=$L; fi
  timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/zl_$L.json 2> gpurun_out/zl_$L.err || { tail -3 gpurun_out/zl_$L.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/zl_$L.json')); print('c4 zstd lanes=$L', d['ms_per_step'], d['value'])"
done

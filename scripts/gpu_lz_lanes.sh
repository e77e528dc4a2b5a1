# C3 step time vs LZ4 lanes in flight (RPGPU_LZ_LANES)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in ${LANES:-0 32768 65536 131072}; do
  if [ $L -eq 0 ]; then unset RPGPU_LZ_LANES; else export RPGPU_LZ_LANES=$L; fi
  timeout -k 10 240 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lz_$L.json 2> gpurun_out/lz_$L.err || { tail -3 gpurun_out/lz_$L.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lz_$L.json')); print('c3 lanes=$L', d['ms_per_step'], d['value'])"
done

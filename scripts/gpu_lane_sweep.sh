# C3 / C4 step time vs lanes in flight of the lane decoders (RPGPU_LZ_LANES,
# RPGPU_ZSTD_LANES): does fewer concurrent lanes (less L2 thrash) help?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/lane_sweep.txt
: > $out
for L in 0 16384 32768 65536 131072; do
  if [ $L -eq 0 ]; then unset RPGPU_LZ_LANES; else export RPGPU_LZ_LANES=$L; fi
  timeout -k 10 240 python bench.py --config c3 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/sw_c3_$L.json 2> gpurun_out/sw_c3_$L.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/sw_c3_$L.json')); print('c3 lanes=$L', d['ms_per_step'], d['value'])" | tee -a $out
done
unset RPGPU_LZ_LANES
for L in 0 8192 16384 32768 65536; do
  if [ $L -eq 0 ]; then unset RPGPU_ZSTD_LANES; else export RPGPU_ZSTD_LANES=$L; fi
  timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sw_c4_$L.json 2> gpurun_out/sw_c4_$L.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/sw_c4_$L.json')); print('c4 lanes=$L', d['ms_per_step'], d['value'])" | tee -a $out
done

# Variant builds of librpgpu.so with extra compile definitions (tuning
# experiments; selected at run time with RPGPU_DIAG_LIB).  Output: $OUT (default build/vx, which travels with a gpurun snapshot)
set -e
cd "$(dirname "$0")/.."
OUT=${OUT:-build/vx}
mkdir -p $OUT
SRCS=$(python3 -c "from redpanda_amd import _build as b; print(' '.join('redpanda_amd/csrc/'+s for s in b.RPGPU_SRCS))")
for v in $VARIANTS; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -D${v//,/ -D} -Iinclude -Iredpanda_amd/csrc $SRCS \
    -o $OUT/librpgpu_${v//[=,]/_}.so &
done
wait
ls -la $OUT

# Variant builds of librpgpu.so with extra compile definitions (tuning
# experiments; selected at run time with RPGPU_DIAG_LIB).  Output: build/var/
set -e
cd "$(dirname "$0")/.."
mkdir -p build/var
SRCS=$(python3 -c "from redpanda_amd import _build as b; print(' '.join('redpanda_amd/csrc/'+s for s in b.RPGPU_SRCS))")
for v in $VARIANTS; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -D${v//,/ -D} -Iinclude -Iredpanda_amd/csrc $SRCS \
    -o build/var/librpgpu_${v//[=,]/_}.so &
done
wait
ls -la build/var

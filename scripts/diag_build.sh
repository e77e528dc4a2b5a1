# Diagnostics builds of librpgpu.so with parts of the validate kernel compiled
# out (timing attribution only; results are not valid).  Output: build/diag/
set -e
cd "$(dirname "$0")/.."
mkdir -p build/diag
SRCS=$(python3 -c "from redpanda_amd import _build as b; print(' '.join('redpanda_amd/csrc/'+s for s in b.RPGPU_SRCS))")
for v in ${DIAG_VARIANTS:-NO_LOOKUP NO_COMBINE STAMPS}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DRPGPU_DIAG_$v -Iinclude -Iredpanda_amd/csrc $SRCS \
    -o build/diag/librpgpu_$v.so &
done
wait

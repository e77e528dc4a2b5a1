# Build librpgpu.so from a git revision into build/ab/librpgpu_<name>.so (A/B timing).
# usage: scripts/ab_build.sh <rev> <name> [extra hipcc flags, e.g. -DRPGPU_CRC_WAVES=3]
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; shift 2
tmp=$(mktemp -d)
git archive "$rev" include redpanda_amd/csrc | tar -x -C "$tmp"
mkdir -p build/ab
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" -I"$tmp/include" -I"$tmp/redpanda_amd/csrc" \
  "$tmp"/redpanda_amd/csrc/rpgpu_*.hip "$tmp/redpanda_amd/csrc/rpgpu_abi.cpp" "$tmp/redpanda_amd/csrc/rpgpu_tables.cpp" \
  -o build/ab/librpgpu_$name.so
rm -rf "$tmp"
echo built build/ab/librpgpu_$name.so

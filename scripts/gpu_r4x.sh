# zstd lane / wave boundary with the round-4 stream layout: 256 KiB (default) / 192 / 160 on C5, interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, lib
  if [ -n "$2" ]; then export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/$2; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 400 python bench.py --warmup 1 --no-cpu-baseline --full-check 0 --config c5 --steps 5 > gpurun_out/r4x_$1.json 2> gpurun_out/r4x_$1.err || { tail -3 gpurun_out/r4x_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4x_$1.json'));print('$1', d['ms_per_step'])"
}
for rep in 1 2; do run z256_$rep "" && run z192_$rep abtmp/librpgpu_z192.so && run z160_$rep abtmp/librpgpu_z160.so || exit 1; done

# C2: partition-summary workgroups (64 default / 128 / 256), interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, lib
  if [ -n "$2" ]; then export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/$2; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --config c2 > gpurun_out/r4r_$1.json 2> gpurun_out/r4r_$1.err || { tail -3 gpurun_out/r4r_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4r_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do run g64_$rep "" && run g128_$rep build/ab/librpgpu_g128.so && run g256_$rep build/ab/librpgpu_g256.so || exit 1; done

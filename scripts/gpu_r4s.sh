# LZ4 / snappy split threshold: 256 KiB (default) / 128 KiB / 80 KiB on C5 (interleaved twice) and C3
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, lib, args
  if [ -n "$2" ]; then export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/$2; else unset RPGPU_DIAG_LIB; fi
  timeout -k 10 400 python bench.py --warmup 1 --no-cpu-baseline --full-check 0 $3 > gpurun_out/r4s_$1.json 2> gpurun_out/r4s_$1.err || { tail -3 gpurun_out/r4s_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4s_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  run c5_s256_$rep "" "--config c5 --steps 5" && run c5_s128_$rep build/ab/librpgpu_s128.so "--config c5 --steps 5" && run c5_s80_$rep build/ab/librpgpu_s80.so "--config c5 --steps 5" || exit 1
done
run c3_s256 "" "--config c3 --steps 5" && run c3_s80 build/ab/librpgpu_s80.so "--config c3 --steps 5"

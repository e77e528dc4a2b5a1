# zstd_kernel phase clocks (diagnostics build with -DRPZ_PROF=1: clock64 around the
# literals section and the sequence loop of each block, printed by 4 workgroups)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
export RPGPU_DIAG_LIB=$GRAFT_REPO_ROOT/build/ab/librpgpu_prof.so
timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/zprof.out 2> gpurun_out/zprof.err || { tail -5 gpurun_out/zprof.err; exit 1; }
grep RPZ_PROF gpurun_out/zprof.out | head -8

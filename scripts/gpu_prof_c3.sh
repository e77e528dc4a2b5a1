# rocprofv3 kernel statistics of the C3 pipeline (text payload)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 -- python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3.json 2> gpurun_out/prof_c3.err || { tail -20 gpurun_out/prof_c3.err; exit 1; }
find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -12

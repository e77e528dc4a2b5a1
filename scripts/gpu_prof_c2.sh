# rocprofv3 kernel statistics of the C2 bench (csv summary)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c2.json 2> gpurun_out/prof_c2.err || { tail -20 gpurun_out/prof_c2.err; exit 1; }
f=$(find gpurun_out/prof_c2 -name "*kernel_stats.csv" | head -1)
cut -d, -f1-6 "$f" | head -8

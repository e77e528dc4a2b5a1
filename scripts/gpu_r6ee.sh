# Round 6, call ee: the final C5 step's kernel timeline (rocpd trace) and kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ee
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python -u bench.py --no-cpu-baseline --config c5 --steps 3 --warmup 1 --full-check 0 > $O/tl.json 2> $O/tl.err || { tail -5 $O/tl.err; exit 1; }
python scripts/timeline_db.py $(find $O/prof -name "*.db") 2 > $O/timeline.txt
CFG=c5 TAG=r6ee/stats STEPS=3 LIMIT=300 BENCH_ARGS="--full-check 0" bash scripts/gpu_prof.sh || exit 1

# Round 6, call i: C5's concurrent kernel timeline (rocpd kernel trace) on the
# library with the one-launch part kernel and split fallbacks decided from the parts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/prof -o run -- python -u bench.py --no-cpu-baseline --config c5 --steps 3 --warmup 1 --full-check 0 > $O/c5_prof.json 2> $O/c5_prof.err || { tail -5 $O/c5_prof.err; exit 1; }
python scripts/timeline_db.py $(find $O/prof -name "*.db" | head -1) 2 | head -30

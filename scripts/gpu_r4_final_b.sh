# round-4 kernel traces + stats: C2 (10 steps), C3 / C4 / C5 (2 steps each)
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c2 TAG=r4final STEPS=10 LIMIT=300 bash scripts/gpu_prof.sh || exit 1
for c in c3 c5 c4; do CFG=$c TAG=r4final STEPS=2 LIMIT=400 BENCH_ARGS="--full-check 0" bash scripts/gpu_prof.sh || exit 1; done

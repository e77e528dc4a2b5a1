# Round 6: PMC passes of C1..C5, then the bench lines and kernel stats, on one library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r6_pmc.sh || exit 1
OUTTAG=${OUTTAG:-r6final4} bash scripts/gpu_r6_final.sh || exit 1

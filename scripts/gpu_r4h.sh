# kernel traces: C5 with the walk overlap off / 16 chunks; C3 and C4 on the round-4 build
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "c5:off:--overlap off" "c5:on:--overlap on" "c3:r4:" "c4:r4:"; do
  IFS=: read cfg tag args <<< "$v"
  CFG=$cfg TAG=r4h_$tag STEPS=2 LIMIT=400 BENCH_ARGS="--full-check 0 $args" bash scripts/gpu_prof.sh || exit 1
done

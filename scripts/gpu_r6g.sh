# Round 6, call g: C5's plan counts and LZ wave list (RPGPU_PLAN_TRACE), one step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
RPGPU_PLAN_TRACE=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --config c5 --steps 2 --warmup 1 --full-check 0 > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
grep "rpgpu plan" $O/c5.err | tail -3

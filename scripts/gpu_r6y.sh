# Round 6, call y: the C5-shaped arena gated and ungated (every decoder launched).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6y
mkdir -p $O
RPGPU_PLAN_TRACE=1 timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_decomp.py -k "c5_shaped" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "rpgpu plan|passed|PASSED" $O/pytest.log | tail -8

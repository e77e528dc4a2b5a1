# GPU parity tests in one process, each bounded: TESTS (default: tests), K (pytest -k)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
LOG=gpurun_out/${LOG:-pytest_gpu}.log
timeout -k 10 ${LIMIT:-1000} python -u -m pytest -x -v --timeout ${PER_TEST:-240} --timeout-method thread -m gpu ${TESTS:-tests} ${K:+-k "$K"} > $LOG 2>&1
rc=$?
tail -5 $LOG
exit $rc

# Round 6, call w: the full GPU suite and smoke on the final library; C5, C4 and C3 with
# every batch checked against the oracle.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUTTAG:-r6w}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --config c5 --steps 3 --warmup 1 --full-check 1 > $O/c5_full.json 2> $O/c5_full.err || { tail -5 $O/c5_full.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5_full.json')); print('c5', d['ms_per_step'], d['full_check']['mismatched_batches'], d['full_check']['batches'])"
timeout -k 10 900 python -u bench.py --no-cpu-baseline --config c4 --steps 3 --warmup 1 --full-check 1 > $O/c4_full.json 2> $O/c4_full.err || { tail -5 $O/c4_full.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4_full.json')); print('c4', d['ms_per_step'], d['full_check']['mismatched_batches'], d['full_check']['batches'])"
timeout -k 10 600 python -u bench.py --no-cpu-baseline --config c3 --steps 3 --warmup 1 --full-check 1 > $O/c3_full.json 2> $O/c3_full.err || { tail -5 $O/c3_full.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3_full.json')); print('c3', d['ms_per_step'], d['full_check']['mismatched_batches'], d['full_check']['batches'])"

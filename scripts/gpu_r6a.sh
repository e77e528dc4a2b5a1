# Round 6, call a: the split zstd executor's miscompare out of line (VERDICT r5
# item 1) under three builds -- inlined (the library), out of line, out of line
# with every s_waitcnt forced to zero -- then one full oracle check of C3 and
# of C4 on the production decoders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_append_time.py > $O/pytest_append.log 2>&1 || { tail -30 $O/pytest_append.log; exit 1; }
tail -2 $O/pytest_append.log
for v in default ool ool_wz; do
  if [ $v = default ]; then unset RPGPU_DIAG_LIB; else export RPGPU_DIAG_LIB=$PWD/build/vx/librpgpu_$v.so; fi
  timeout -k 10 400 python -u scripts/zseq_repro.py --iters 4 > $O/repro_$v.log 2>&1 || { tail -5 $O/repro_$v.log; exit 1; }
  echo "== $v"; grep -E "^iter|distinct" $O/repro_$v.log
done
unset RPGPU_DIAG_LIB
for c in c3 c4; do
  timeout -k 10 900 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --full-check 1 > $O/${c}_full.json 2> $O/${c}_full.err || { tail -5 $O/${c}_full.err; exit 1; }
  python -c "import json; d=json.load(open('$O/${c}_full.json')); print('$c', d['ms_per_step'], d['full_check']['batches'], d['full_check']['mismatched_batches'], d['full_check']['mismatches_by_kind'])"
done

# Round 6, call b: bisect the split zstd executor's miscompare (VERDICT r5
# item 1).  exec_lane built four ways -- inlined with global accesses (the
# library), out of line with flat accesses, out of line with global accesses,
# inlined with flat accesses -- each decodes test_many_tiny_zstd_gzip's arena 4
# times against the oracle (scripts/zseq_repro.py).  Then one full oracle check
# of C3 and of C4 on the production decoders (bench.py --full-check 1, with the
# plan-wait step of round 6).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6b
mkdir -p $O
for v in default ool oolg inlf; do
  if [ $v = default ]; then unset RPGPU_DIAG_LIB; else export RPGPU_DIAG_LIB=$PWD/build/vx/librpgpu_$v.so; fi
  timeout -k 10 300 python -u scripts/zseq_repro.py --iters 4 > $O/repro_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -E "^iter|distinct|Error" $O/repro_$v.log
  # a miscompare or assertion (rc 1) is data; anything else (fault, abort, timeout) ends the call
  [ $rc -le 1 ] || exit 1
done
unset RPGPU_DIAG_LIB
for c in c3 c4; do
  timeout -k 10 900 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --full-check 1 > $O/${c}_full.json 2> $O/${c}_full.err || { tail -5 $O/${c}_full.err; exit 1; }
  python -c "import json; d=json.load(open('$O/${c}_full.json')); print('$c', d['ms_per_step'], d['full_check']['batches'], d['full_check']['mismatched_batches'], d['full_check']['mismatches_by_kind'])"
done

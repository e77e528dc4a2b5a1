# Round 6, call c: (1) two probes of the out-of-line exec_lane miscompare --
# wait states before every funnel shift (RPZS_NOP_SHIFT), wait states at the
# function's entry and exit (RPZS_NOP_EDGES); (2) the library with the
# write-combined zstd lane sequences (rpgpu_zstd.h wc_seq): the decompress GPU
# tests, two full oracle checks of C4 and one of C5, and C4 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
for v in oolnopsh oolent; do
  export RPGPU_DIAG_LIB=$PWD/build/vx/librpgpu_$v.so
  timeout -k 10 300 python -u scripts/zseq_repro.py --iters 4 > $O/repro_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -E "^iter|distinct|Error" $O/repro_$v.log
  [ $rc -le 1 ] || exit 1
done
unset RPGPU_DIAG_LIB
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_decomp.py tests/test_gpu_bench_configs.py tests/test_gpu_append_time.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  timeout -k 10 900 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --full-check 1 > $O/c4_full$r.json 2> $O/c4_full$r.err || { tail -5 $O/c4_full$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_full$r.json')); print('c4', d['ms_per_step'], d['roofline']['kernel_ms'], d['full_check']['batches'], d['full_check']['mismatched_batches'])"
done
timeout -k 10 900 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --full-check 1 > $O/c5_full.json 2> $O/c5_full.err || { tail -5 $O/c5_full.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5_full.json')); print('c5', d['ms_per_step'], d['full_check']['batches'], d['full_check']['mismatched_batches'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c4.json 2> $O/prof_c4.err || { tail -5 $O/prof_c4.err; exit 1; }
f=$(find $O/prof_c4 -name "*kernel_stats.csv" | head -1); cp "$f" $O/c4_kernel_stats.csv
python - $O/c4_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print(" ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e6,3), "ms", r["Percentage"])
PY

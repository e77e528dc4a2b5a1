# Round 6, call d: (1) the out-of-line exec_lane with a check of the caller's
# loop index across the call (RPZS_CHECK_K: printf when it changed); (2) kernel
# statistics of C3 / C5 in the plan-wait flow (idle launches); (3) C4 PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6d
mkdir -p $O
export RPGPU_DIAG_LIB=$PWD/build/vx/librpgpu_oolchk.so
timeout -k 10 300 python -u scripts/zseq_repro.py --iters 3 > $O/repro_oolchk.log 2>&1
rc=$?
echo "== oolchk rc=$rc"; grep -E "^iter|distinct|Error" $O/repro_oolchk.log; grep -c "k .* ->" $O/repro_oolchk.log; grep "k .* ->" $O/repro_oolchk.log | head -5
[ $rc -le 1 ] || exit 1
unset RPGPU_DIAG_LIB
for c in c3 c5; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --full-check 0 > $O/prof_$c.json 2> $O/prof_$c.err || { tail -5 $O/prof_$c.err; exit 1; }
  f=$(find $O/prof_$c -name "*kernel_stats.csv" | head -1); cp "$f" $O/${c}_kernel_stats.csv
  echo "== $c"; python -c "import json; d=json.load(open('$O/prof_$c.json')); print('  step', d['ms_per_step'], d['value'], d['roofline']['frac'])"
  python - $O/${c}_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print("  ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e6,3), "ms", r["Percentage"])
PY
done
CFG=c4 TAG=r6d bash scripts/gpu_pmc_traffic.sh > $O/pmc_c4.log 2>&1 || { tail -5 $O/pmc_c4.log; exit 1; }
tail -12 $O/pmc_c4.log

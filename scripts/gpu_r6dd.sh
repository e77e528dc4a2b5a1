# Round 6, call dd: the C5 bench line (CPU baseline, every batch against the oracle) with
# its walk-overlap chunks at 8 (bench.py's c5 config), twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6dd
mkdir -p $O
for k in 1 2; do
  timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 2 > $O/c5_$k.json 2> $O/c5_$k.err || { tail -5 $O/c5_$k.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c5_$k.json'));r=d['roofline'];print('c5', d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), d['config'].get('walk_chunks'), d['full_check']['mismatched_batches'])"
done

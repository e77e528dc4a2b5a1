# Round 6, call gg: the full GPU suite and smoke on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6gg
mkdir -p $O
python -c "from redpanda_amd import engine; print('lib', engine.library_hash())"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/default_bench.json 2> $O/default_bench.err || { tail -5 $O/default_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/default_bench.json'));r=d['roofline'];print('default', d['metric'][:40], d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'))"

# Round 6, call e: the full GPU suite on the library without the split zstd
# decoder; C4 at fewer zstd lanes (their tables L2 / MALL-resident?); C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for wl in 0 65536 32768 16384; do
  timeout -k 10 600 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --ws-lanes $wl > $O/c4_wl$wl.json 2> $O/c4_wl$wl.err || { tail -5 $O/c4_wl$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_wl$wl.json')); print('c4 ws_lanes $wl', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
timeout -k 10 600 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/c2.json')); print('c2', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"

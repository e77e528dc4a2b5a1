# Full GPU parity suite + smoke, then C2..C5 bench lines (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r11}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
run() {  # cfg label env...
  local cfg=$1 label=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_${cfg}_$label.json 2> gpurun_out/${TAG}_${cfg}_$label.err || { tail -3 gpurun_out/${TAG}_${cfg}_$label.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${cfg}_$label.json')); print('$cfg $label', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('gpu_matches_oracle_on_sample'))"
}
run c2 base && run c3 base && run c4 base && run c5 base

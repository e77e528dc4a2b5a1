# step time of library variants (build/var/*.so, RPGPU_DIAG_LIB) per config: VARS="cfg:name ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # cfg label env...
  local cfg=$1 label=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/var_${cfg}_$label.json 2> gpurun_out/var_${cfg}_$label.err || { tail -3 gpurun_out/var_${cfg}_$label.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/var_${cfg}_$label.json')); print('$cfg $label', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('gpu_matches_oracle_on_sample'))"
}
for v in $VARS; do
  cfg=${v%%:*}; name=${v#*:}
  if [ "$name" = base ]; then run $cfg base || exit 1; else run $cfg $name RPGPU_DIAG_LIB=$PWD/build/var/librpgpu_$name.so || exit 1; fi
done

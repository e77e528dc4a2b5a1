# C2 chunk counts (interleaved twice); C3 / C4 with the overlap on and off
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, args
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-check 0 $2 > gpurun_out/r4j_$1.json 2> gpurun_out/r4j_$1.err || { tail -3 gpurun_out/r4j_$1.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4j_$1.json'));print('$1', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  for k in 16 20 24 32; do run c2_k${k}_$rep "--config c2 --walk-chunks $k" || exit 1; done
done
run c3off "--config c3 --steps 5 --overlap off" && run c3on "--config c3 --steps 5 --overlap on" || exit 1
run c4off "--config c4 --steps 3 --overlap off" && run c4on "--config c4 --steps 3 --overlap on" || exit 1

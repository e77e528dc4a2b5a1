# C5: overlap off / chunked / side by side; C2 default twice (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "c5off:--config c5 --overlap off" "c5side:--config c5 --overlap on --walk-chunks 1" "c2:--config c2" "c2side6:--config c2 --walk-chunks 1 --blocks-per-cu 6" "c2b:--config c2"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --full-check 0 $args > gpurun_out/r4g_$name.json 2> gpurun_out/r4g_$name.err || { tail -3 gpurun_out/r4g_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4g_$name.json'));print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
done

export TMPDIR=/tmp; mkdir -p gpurun_out/r5o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_decomp.py -k "block_parallel or large_bodies or ring_extdict or mixed_codecs or split_decoder" > gpurun_out/r5o/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5o/pytest.log; [ $rc -eq 0 ] || exit 1
run() { # tag args
  tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5o/$tag -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/r5o/$tag.json 2> gpurun_out/r5o/$tag.err || { tail -3 gpurun_out/r5o/$tag.err; exit 1; }
  f=$(find gpurun_out/r5o/$tag -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r5o/${tag}_kernel_stats.csv
  echo "== $tag $(python -c "import json;d=json.load(open('gpurun_out/r5o/$tag.json'));print(d['ms_per_step'], d['value'])")"
  python - $f <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:9]:
    print("  ", r["Name"][:50], r["Calls"], round(float(r["AverageNs"])/1e6,2), "ms")
PY
}
run c5_blk --config c5 --full-check 0 && run c5_wave --config c5 --full-check 0 --zstd-blocks off && run c4_off --config c4 && run c4_fused --config c4 --zstd-split fused

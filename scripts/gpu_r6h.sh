# Round 6, call h: the new decompress tests (segment-span zstd frames, short
# LZ4 blocks); C5 with split fallbacks decided from the parts; C5's kernels
# one after the other on one stream (each one's duration alone).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_decomp.py -k "span or short_block or fallback or band or ring" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
RPGPU_PLAN_TRACE=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --config c5 --steps 3 --warmup 1 --full-check 0 > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
grep "rpgpu plan" $O/c5.err | tail -1
python -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['ms_per_step'], d['roofline']['kernel_ms'])"
RPGPU_SERIAL_STREAMS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_serial -o run -- python -u bench.py --no-cpu-baseline --config c5 --steps 2 --warmup 1 --full-check 0 > $O/c5_serial.json 2> $O/c5_serial.err || { tail -5 $O/c5_serial.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5_serial.json')); print('c5 serial', d['ms_per_step'], d['roofline']['kernel_ms'])"
find $O/prof_serial -name "*kernel_stats.csv" | head -3

#!/bin/bash
# GPU suite + a first C4 (zstd) measurement.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --config c4 --batches 32768 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4_small.json 2> gpurun_out/c4_small.log || exit 1
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/c4_bench.json 2> gpurun_out/c4_bench.log

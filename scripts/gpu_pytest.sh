set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import torch;print(torch.cuda.get_device_name(0))" > gpurun_out/dev.txt 2>&1
ls /opt/conda/lib/liblz4* /opt/conda/lib/libzstd* /opt/conda/lib/libsnappy* >> gpurun_out/dev.txt 2>&1
nproc >> gpurun_out/dev.txt
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log

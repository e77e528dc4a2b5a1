# SQ counters of the decode kernels (separate passes), small C3/C4 arenas
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r09pmc}
for cfg in c3 c4; do
  i=0
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/${TAG}_${cfg}_p$i -o pmc -- python bench.py --config $cfg --batches 16384 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_${cfg}_p$i.json 2> gpurun_out/${TAG}_${cfg}_p$i.err || { tail -5 gpurun_out/${TAG}_${cfg}_p$i.err; exit 1; }
  done
done

# PMC passes over bench.py (one rocprofv3 --pmc pass per counter set, kernel
# trace only).  BENCH_ARGS selects the workload/ops; PMC_SETS overrides sets
# (';'-separated).  Output: gpurun_out/pmc/p<i>/
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
SETS=${PMC_SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS;SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD;TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES;FETCH_SIZE;WRITE_SIZE"}
i=0
IFS=';' read -ra ARR <<< "$SETS"
for set in "${ARR[@]}"; do
  i=$((i+1))
  rm -rf $R/gpurun_out/pmc/p$i
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc/p$i.log; exit 1; }
done
echo pmc done

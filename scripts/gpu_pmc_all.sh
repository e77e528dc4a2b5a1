# PMC traffic passes for the decompress configs (CFGS), one pass per counter group
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in ${CFGS:-c3 c4 c5}; do
  CFG=$c TAG=${TAG:-r11pmc} KERNELS="validate_kernel" bash scripts/gpu_pmc_traffic.sh || exit 1
done

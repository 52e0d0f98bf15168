#!/bin/bash
# Round-6 PMC breakdown of the wide kernels: where the wave cycles go (parked at s_waitcnt/barrier,
# issue-stalled, issuing) and what the VMEM / LDS paths report, for the p = 32 encode (A-resident),
# the 6-tile tile-major GEMM without and with 104 fused copies, and the 7-tile one with 102 copies.
#   usage: r6_pmc2.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6r}; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
cases=("enc128:--k 128 --m 32 --engine mfma" "tm6:--k 128 --m 24 --engine mfma" "tm6c:--k 128 --m 24 --copies 104 --engine mfma" "tm7c:--k 128 --m 26 --copies 102 --engine mfma")
for cfg in "${cases[@]}"; do
  name=${cfg%%:*}; args=${cfg#*:}; i=0
  for ctr in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    echo "[$(date +%T)] ${name}_$i"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr -d $O/${name}_$i -o run --output-format csv -- \
      python3 scripts/prof_case.py --iters 3 $args > $O/${name}_$i.log 2>&1 || { echo "rc=$? ${name}_$i"; tail -5 $O/${name}_$i.log; exit 1; }
  done
done
echo PMC2-OK

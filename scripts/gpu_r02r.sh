#!/bin/bash
# Round-2 session R: PMC passes of the A-resident FP4 kernel vs the default (sk) kernel, k=128 m=32.
O=gpurun_out/r02r
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for kern in ar sk; do
  for p in 1 2; do
    eval CTR=\$P$p
    GFRS_FP4_KERNEL=$kern step pmc_${kern}_$p 120 rocprofv3 --kernel-trace --pmc $CTR -d $O/pmc_${kern}_$p -o run --output-format csv -- \
      python3 scripts/prof_case.py --iters 5 --k 128 --m 32 --engine mfma || exit 1
  done
done
echo SESSION-OK | tee -a $O/progress.log

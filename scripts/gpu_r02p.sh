#!/bin/bash
# Round-2 session P: clock / cycle counters of the FP4 ablation builds (is the wide stripe
# power-bound?): one PMC pass per build, kernel trace for the wall time.
O=gpurun_out/r02p
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
CTR="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for a in 0 1 2 4; do
  GFRS_FP4_ABL=$a step pmc_abl$a 120 rocprofv3 --kernel-trace --pmc $CTR -d $O/pmc_abl$a -o run --output-format csv -- \
    python3 scripts/prof_case.py --iters 5 --k 128 --m 32 --engine mfma || exit 1
done
echo SESSION-OK | tee -a $O/progress.log

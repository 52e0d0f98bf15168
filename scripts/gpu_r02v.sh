#!/bin/bash
# Round-2 session V: HBM bytes fetched by the A-resident kernel with / without fused copies (is the
# second row-half wave's duplicate DMA an L2 hit?), vs the default kernels.
O=gpurun_out/r02v
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
CTR="FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES"
GFRS_FP4_KERNEL=ar step ar_plain 120 rocprofv3 --kernel-trace --pmc $CTR -d $O/ar_plain -o run --output-format csv -- python3 scripts/prof_case.py --iters 3 --k 128 --m 24 --engine mfma &&
GFRS_FP4_KERNEL=ar step ar_copy 120 rocprofv3 --kernel-trace --pmc $CTR -d $O/ar_copy -o run --output-format csv -- python3 scripts/prof_case.py --iters 3 --k 128 --m 24 --copies 104 --engine mfma &&
step def_copy 120 rocprofv3 --kernel-trace --pmc $CTR -d $O/def_copy -o run --output-format csv -- python3 scripts/prof_case.py --iters 3 --k 128 --m 24 --copies 104 --engine mfma &&
echo SESSION-OK | tee -a $O/progress.log

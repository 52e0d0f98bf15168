#!/bin/bash
# Round-2 session O: FP4 sk-kernel ablations (k=128, m=32 encode, 1 GiB): which part bounds it.
O=gpurun_out/r02o
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step abl0 120 env GFRS_FP4_ABL=0 python scripts/fp4_ablate.py &&
step abl1 120 env GFRS_FP4_ABL=1 python scripts/fp4_ablate.py &&
step abl2 120 env GFRS_FP4_ABL=2 python scripts/fp4_ablate.py &&
step abl3 120 env GFRS_FP4_ABL=3 python scripts/fp4_ablate.py &&
step abl4 120 env GFRS_FP4_ABL=4 python scripts/fp4_ablate.py &&
step abl7 120 env GFRS_FP4_ABL=7 python scripts/fp4_ablate.py &&
step abl0b 120 env GFRS_FP4_ABL=0 python scripts/fp4_ablate.py &&
echo SESSION-OK | tee -a $O/progress.log

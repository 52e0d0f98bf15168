#!/bin/bash
# Round-2 session S: A-resident vs default FP4 kernels over M-tile counts (k=128; m = 8..32 plain
# and with fused copies), alternating runs.
O=gpurun_out/r02s
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step def1 300 python scripts/fp4_shapes.py 4,8,12,16,24,32 &&
step ar1 300 env GFRS_FP4_KERNEL=ar python scripts/fp4_shapes.py 4,8,12,16,24,32 &&
step def2 300 python scripts/fp4_shapes.py 4,8,12,16,24,32 &&
step ar2 300 env GFRS_FP4_KERNEL=ar python scripts/fp4_shapes.py 4,8,12,16,24,32 &&
echo SESSION-OK | tee -a $O/progress.log

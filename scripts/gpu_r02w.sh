#!/bin/bash
# Round-2 session W: A-resident kernel on scattered inputs (row-pointer table, no copy) at two row
# halves — is the fused-copy slowdown the copy or the pointer-table path?
O=gpurun_out/r02w
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step def 300 python scripts/fp4_shapes.py 24,32 --scattered &&
step ar 300 env GFRS_FP4_KERNEL=ar python scripts/fp4_shapes.py 24,32 --scattered &&
echo SESSION-OK | tee -a $O/progress.log

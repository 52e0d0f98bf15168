#!/bin/bash
# Round-2 session J: ring depth 8 vs 4 for the exact-MG (5..7) static FP4 kernels.
O=gpurun_out/r02j
source "$(dirname "$0")/gpustep.sh"
step shapes_r8 300 python scripts/fp4_shapes.py &&
step shapes_r4 300 env GFRS_FP4_RING=4 python scripts/fp4_shapes.py &&
step shapes_pad 300 env GFRS_FP4_EXACT_MG=0 python scripts/fp4_shapes.py &&
step shapes_r4b 300 env GFRS_FP4_RING=4 python scripts/fp4_shapes.py &&
step shapes_r8b 300 python scripts/fp4_shapes.py &&
echo SESSION-OK | tee -a $O/progress.log

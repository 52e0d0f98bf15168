#!/bin/bash
# Round-2 session T: A-resident kernel with both row-half waves storing the fused copies.
O=gpurun_out/r02t
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step pytest_ar 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "a_resident" --timeout 120 --timeout-method thread &&
step def1 300 python scripts/fp4_shapes.py 20,24,28,32 &&
step ar1 300 env GFRS_FP4_KERNEL=ar python scripts/fp4_shapes.py 20,24,28,32 &&
step def2 300 python scripts/fp4_shapes.py 20,24,28,32 &&
step ar2 300 env GFRS_FP4_KERNEL=ar python scripts/fp4_shapes.py 20,24,28,32 &&
echo SESSION-OK | tee -a $O/progress.log

#!/bin/bash
# Round-2 session X: the hybrid FP4 kernel (5..8 M-tiles per wave, tiles 4+ from LDS): correctness,
# then shapes against the default LDS kernels and the two-row-halves form.
O=gpurun_out/r02x
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step pytest_ar 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "a_resident or staggered" --timeout 120 --timeout-method thread &&
step def1 300 env GFRS_FP4_KERNEL=v1 python scripts/fp4_shapes.py 20,24,28,32 &&
step hy1 300 env GFRS_FP4_KERNEL=ar python scripts/fp4_shapes.py 20,24,28,32 &&
step def2 300 env GFRS_FP4_KERNEL=v1 python scripts/fp4_shapes.py 20,24,28,32 &&
step hy2 300 env GFRS_FP4_KERNEL=ar python scripts/fp4_shapes.py 20,24,28,32 &&
step sk 300 env GFRS_FP4_KERNEL=sk python scripts/fp4_shapes.py 24,32 &&
echo SESSION-OK | tee -a $O/progress.log

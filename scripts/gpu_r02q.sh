#!/bin/bash
# Round-2 session Q: the A-resident FP4 kernel (gf_mfma_fp4ar.hip): correctness, then encode and
# decode-shape timings against the default kernels.
O=gpurun_out/r02q
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step pytest_fp4 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "fp4" --timeout 120 --timeout-method thread &&
step enc_default 120 python scripts/fp4_ablate.py &&
step enc_ar 120 env GFRS_FP4_KERNEL=ar python scripts/fp4_ablate.py &&
step shapes_default 300 python scripts/fp4_shapes.py 20,26,32 &&
step shapes_ar 300 env GFRS_FP4_KERNEL=ar python scripts/fp4_shapes.py 20,26,32 &&
step enc_ar2 120 env GFRS_FP4_KERNEL=ar python scripts/fp4_ablate.py &&
step enc_default2 120 python scripts/fp4_ablate.py &&
echo SESSION-OK | tee -a $O/progress.log

#!/bin/bash
# Round-2 session I: exact M-tile counts (MG 5..7) for the static wide-stripe chunk — FP4 tests,
# shape A/B (padded 8 vs exact), k128n160 bench A/B.
O=gpurun_out/r02i
source "$(dirname "$0")/gpustep.sh"
step test_fp4 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread -k "fp4 or mfma or auto_engine or decode" &&
step shapes_exact 300 python scripts/fp4_shapes.py &&
step shapes_pad 300 env GFRS_FP4_EXACT_MG=0 python scripts/fp4_shapes.py &&
step bench_exact 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step bench_pad 300 env GFRS_FP4_EXACT_MG=0 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step bench_exact2 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

#!/bin/bash
# Round-2 session K: exact-MG kernels at ring 4 (the new default), ring 4 vs 8 for m <= 16,
# k128n160 bench.
O=gpurun_out/r02k
source "$(dirname "$0")/gpustep.sh"
step test_fp4 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_codec.py tests/test_properties.py -x -q --timeout 120 --timeout-method thread -k "fp4 or mfma or auto_engine or decode" &&
step shapes 300 python scripts/fp4_shapes.py 8,12,16,20,24,28,32 &&
step shapes_r4 300 env GFRS_FP4_RING=4 python scripts/fp4_shapes.py 8,12,16 &&
step shapes_b 300 python scripts/fp4_shapes.py 8,12,16 &&
step bench1 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step bench2 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --preset k128n160 --steps 10 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

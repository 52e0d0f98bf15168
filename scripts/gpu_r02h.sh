#!/bin/bash
# Round-2 session H: sk kernel with the refill DMA one step earlier — FP4 tests, wide-stripe bench,
# kernel stats and one PMC pass set.
O=gpurun_out/r02h
source "$(dirname "$0")/gpustep.sh"
step test_fp4 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "fp4 or mfma or auto_engine" &&
step bench_k128 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step prof_k128 300 rocprofv3 --kernel-trace --stats -d $O/prof_k128 -o run --output-format csv -- python3 bench.py --preset k128n160 --steps 10 --no-e2e &&
step prof_case 300 rocprofv3 --kernel-trace --stats -d $O/prof_case -o run --output-format csv -- python3 scripts/prof_case.py --k 128 --m 32 --engine mfma --iters 5 &&
step pmc_sk 600 env PMC_DIR=$O/pmc bash scripts/pmc_one.sh fp4sk_k128_m32 "--k 128 --m 32 --engine mfma" &&
echo SESSION-OK | tee -a $O/progress.log

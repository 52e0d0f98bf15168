#!/bin/bash
# Round-2 session E: the double-buffered FP4 kernel — correctness (new + existing FP4 tests), then
# wide-stripe bench db vs v1, kernel stats and PMC of the db kernel.
O=gpurun_out/r02e
source "$(dirname "$0")/gpustep.sh"
step test_db 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "fp4 or mfma or auto_engine or decode_system" &&
step test_codec 600 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread -k "wide" &&
step bench_k128_sk 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step bench_k128_v1 300 env GFRS_FP4_KERNEL=v1 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step prof_k128 300 rocprofv3 --kernel-trace --stats -d $O/prof_k128 -o run --output-format csv -- python3 bench.py --preset k128n160 --steps 10 --no-e2e &&
step pmc_sk 600 env PMC_DIR=$O/pmc bash scripts/pmc_one.sh fp4sk_k128_m32 "--k 128 --m 32 --engine mfma" &&
echo SESSION-OK | tee -a $O/progress.log

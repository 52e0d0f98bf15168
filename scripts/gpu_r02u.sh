#!/bin/bash
# Round-2 session U: A-resident FP4 kernel as the default where it wins — full GPU suite, wide and
# headline benches.
O=gpurun_out/r02u
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step bench_k128_a 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step bench_k128_sk 300 env GFRS_FP4_KERNEL=sk python bench.py --preset k128n160 --steps 20 --no-e2e &&
step bench_k128_b 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step prof_k128 300 rocprofv3 --kernel-trace --stats -d $O/prof_k128 -o run --output-format csv -- python3 bench.py --preset k128n160 --steps 20 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

#!/bin/bash
# Round-2 session F: staggered FP4 encode + v1 fused-copy decode, decode solve pipelined one step
# ahead beside the previous decode GEMM; headline and wide-stripe benches, graph mode, kernel stats.
O=gpurun_out/r02f
source "$(dirname "$0")/gpustep.sh"
step test_fp4 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "fp4 or mfma or auto_engine or decode_system" &&
step bench_k10 300 python bench.py --steps 20 --warmup 5 --no-e2e &&
step bench_k10_graph 300 python bench.py --steps 20 --warmup 5 --no-e2e --graph &&
step bench_k128 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step bench_k128_v1 300 env GFRS_FP4_KERNEL=v1 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step prof_k128 300 rocprofv3 --kernel-trace --stats -d $O/prof_k128 -o run --output-format csv -- python3 bench.py --preset k128n160 --steps 10 --no-e2e &&
step prof_k10 300 rocprofv3 --kernel-trace --stats -d $O/prof_k10 -o run --output-format csv -- python3 bench.py --steps 10 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

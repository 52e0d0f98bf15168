#!/bin/bash
# Round-2 session L: two-lane step pipelining in bench.py (A/B vs --lanes 1), trace.
O=gpurun_out/r02l
source "$(dirname "$0")/gpustep.sh"
step b2a 300 python bench.py --steps 50 --no-e2e &&
step b1a 300 python bench.py --steps 50 --no-e2e --lanes 1 &&
step b2b 300 python bench.py --steps 50 --no-e2e &&
step b1b 300 python bench.py --steps 50 --no-e2e --lanes 1 &&
step k128_2 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step k128_1 300 python bench.py --preset k128n160 --steps 20 --no-e2e --lanes 1 &&
step k16_2 300 python bench.py --preset k16n20_8g --steps 10 --no-e2e &&
step k16_1 300 python bench.py --preset k16n20_8g --steps 10 --no-e2e --lanes 1 &&
step trace 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --no-e2e &&
step full 300 python bench.py --steps 20 --warmup 5 &&
echo SESSION-OK | tee -a $O/progress.log

#!/bin/bash
# Round-2 session AI: sustained throughput (~1 minute of back-to-back steps per config) after the
# packaging change, plus the full GPU suite once more.
O=gpurun_out/r02ai
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
step short_k10 300 python bench.py --steps 20 --warmup 5 --no-e2e &&
step sustained_k10 300 python bench.py --steps 90000 --warmup 100 --no-e2e &&
step short_k128 300 python bench.py --preset k128n160 --steps 20 --warmup 5 --no-e2e &&
step sustained_k128 300 python bench.py --preset k128n160 --steps 40000 --warmup 100 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

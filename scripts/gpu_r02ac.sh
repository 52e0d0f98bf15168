#!/bin/bash
# Round-2 session AC: kernel timeline of the k=128, n=160 bench step (where does the 1.52 ms go).
O=gpurun_out/r02ac
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step prof_k128 300 rocprofv3 --kernel-trace -d $O/prof_k128 -o run --output-format csv -- python3 bench.py --preset k128n160 --steps 20 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

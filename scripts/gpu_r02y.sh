#!/bin/bash
O=gpurun_out/r02y
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step dbg32 300 env GFRS_FP4_KERNEL=ar python scripts/fp4_debug.py 128 32 262144 ident &&
step dbg20 120 env GFRS_FP4_KERNEL=ar python scripts/fp4_debug.py 128 20 262144 &&
echo SESSION-OK | tee -a $O/progress.log

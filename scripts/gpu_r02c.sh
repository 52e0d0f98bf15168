#!/bin/bash
# Round-2 session C: cold (first-call, fresh pinned buffers) vs warm host pipeline.
O=gpurun_out/r02c
source "$(dirname "$0")/gpustep.sh"
step pipe_cold 300 python scripts/pipe_bench.py --cold 0,2147483648,1073741824 --streams 1,4 --split 0,1 --rect 1 --slices 16777216 &&
echo SESSION-OK | tee -a $O/progress.log

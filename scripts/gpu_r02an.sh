#!/bin/bash
# Round-2 session AN: rocprofv3 kernel statistics of the final tree, headline and wide-stripe presets.
O=gpurun_out/r02an
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step prof_k10 300 rocprofv3 --kernel-trace --stats -d $O/prof_k10 -o run --output-format csv -- python3 bench.py --steps 20 --no-e2e &&
step prof_k128 300 rocprofv3 --kernel-trace --stats -d $O/prof_k128 -o run --output-format csv -- python3 bench.py --preset k128n160 --steps 20 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

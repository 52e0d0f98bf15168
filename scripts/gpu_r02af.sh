#!/bin/bash
# Round-2 session AF: every BASELINE preset on the final tree (device step + e2e block).
O=gpurun_out/r02af
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step k10n14 300 python bench.py --steps 20 --warmup 5 &&
step k4n6 300 python bench.py --preset k4n6 --steps 20 --warmup 5 &&
step k16n20_8g 400 python bench.py --preset k16n20_8g --steps 10 --warmup 3 &&
step k128n160 300 python bench.py --preset k128n160 --steps 20 --warmup 5 &&
echo SESSION-OK | tee -a $O/progress.log

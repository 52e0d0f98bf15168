#!/bin/bash
# Round-2 session AH: k=128, n=160 bench step with 1 / 2 / 3 / 4 lanes (co-running FP4 GEMMs), twice.
O=gpurun_out/r02ah
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step l2a 300 python bench.py --preset k128n160 --steps 20 --no-e2e --lanes 2 &&
step l3a 300 python bench.py --preset k128n160 --steps 20 --no-e2e --lanes 3 &&
step l4a 300 python bench.py --preset k128n160 --steps 20 --no-e2e --lanes 4 &&
step l1a 300 python bench.py --preset k128n160 --steps 20 --no-e2e --lanes 1 &&
step l2b 300 python bench.py --preset k128n160 --steps 20 --no-e2e --lanes 2 &&
step l3b 300 python bench.py --preset k128n160 --steps 20 --no-e2e --lanes 3 &&
step l4b 300 python bench.py --preset k128n160 --steps 20 --no-e2e --lanes 4 &&
echo SESSION-OK | tee -a $O/progress.log

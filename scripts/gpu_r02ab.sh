#!/bin/bash
# Round-2 session AB: the new GPU bench-record tests, and the GPU-side cost of the per-step parity
# exchange (scripts/exchange_cost.py: the owners all-to-all's local HBM traffic replayed on one GPU).
O=gpurun_out/r02ab
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step pytest_bench 400 python -u -m pytest tests/test_bench.py -m gpu -x -v --timeout 300 --timeout-method thread &&
step exchange_cost 300 python scripts/exchange_cost.py --steps 30 --rounds 3 &&
echo SESSION-OK | tee -a $O/progress.log

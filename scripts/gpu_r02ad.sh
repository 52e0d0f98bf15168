#!/bin/bash
# Round-2 session AD: the final tree as the driver runs it (full GPU suite, smoke, default bench).
O=gpurun_out/r02ad
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE-OK')" &&
step bench 300 python bench.py --steps 20 --warmup 5 &&
step bench_lanes3 300 python bench.py --steps 20 --warmup 5 --lanes 3 --no-e2e &&
step bench_lanes2 300 python bench.py --steps 20 --warmup 5 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

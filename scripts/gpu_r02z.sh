#!/bin/bash
# Round-2 session Z (restored container): full GPU suite + smoke + default bench as the driver runs
# them, the wide-stripe preset, and kernel stats of the headline bench.
O=gpurun_out/r02z
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE-OK')" &&
step bench 300 python bench.py --steps 20 --warmup 5 &&
step bench_k128n160 300 python bench.py --preset k128n160 --steps 20 &&
step prof_bench 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python3 bench.py --steps 20 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

#!/bin/bash
# Round-2 session N: the restored tree (fresh container, rebuilt extensions): full GPU suite,
# smoke, default bench and the wide-stripe preset.
O=gpurun_out/r02n
source "$(dirname "$0")/gpustep.sh"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE-OK')" &&
step bench 300 python bench.py --steps 20 --warmup 5 &&
step bench_k128 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

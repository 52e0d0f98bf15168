#!/bin/bash
# Round-2 session G: full GPU suite + smoke on the current tree, headline bench (default flags, as
# the driver runs it), BASELINE presets, the reference k-sweep, streaming file codec, kernel stats.
O=gpurun_out/r02g
source "$(dirname "$0")/gpustep.sh"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench 300 python bench.py --steps 20 --warmup 5 &&
step bench_k16n20 300 python bench.py --preset k16n20_8g --steps 10 --no-e2e &&
step bench_k4n6 300 python bench.py --preset k4n6 --steps 20 &&
step sweep_gpu 600 python scripts/sweep.py --part gpu --out $O/sweep_gpu.json &&
step mkfile 120 python -c "import os; open('/tmp/rs_in.bin','wb').write(os.urandom((1<<30)+12345))" &&
step stream_encode 300 bin/RS -k 10 -n 14 -e /tmp/rs_in.bin --window 0 --no-sync -s 4 &&
step stream_decode 300 bash -c "printf '/tmp/_%d_rs_in.bin\n' 0 2 3 5 6 8 10 11 12 13 > /tmp/rs_conf && bin/RS -d -i /tmp/rs_in.bin -c /tmp/rs_conf -o /tmp/rs_out.bin --window 0 --no-sync -s 4 && cmp /tmp/rs_in.bin /tmp/rs_out.bin && echo IDENTICAL" &&
step prof_bench 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python3 bench.py --steps 20 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

#!/bin/bash
# Round-2 session A: GPU tests (incl. the new multi-device paths), smoke, headline bench with the
# default e2e block, -s 1 vs -s 4 host pipeline through bin/RS, rocprofv3 kernel stats.
O=gpurun_out/r02a
source "$(dirname "$0")/gpustep.sh"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench 300 python bench.py --steps 20 --warmup 5 &&
step mkfile 120 python -c "import os; open('/tmp/rs_in.bin','wb').write(os.urandom((1<<30)+12345))" &&
step rs_encode_s1 120 bin/RS -k 10 -n 14 -e /tmp/rs_in.bin -s 1 &&
step rs_encode_s4 120 bin/RS -k 10 -n 14 -e /tmp/rs_in.bin -s 4 &&
step rs_decode_s4 120 bash -c "printf '/tmp/_%d_rs_in.bin\n' 0 2 3 5 6 8 10 11 12 13 > /tmp/rs_conf && bin/RS -d -i /tmp/rs_in.bin -c /tmp/rs_conf -o /tmp/rs_out.bin -s 4 && cmp /tmp/rs_in.bin /tmp/rs_out.bin && echo IDENTICAL" &&
step rs_decode_s1 120 bash -c "bin/RS -d -i /tmp/rs_in.bin -c /tmp/rs_conf -o /tmp/rs_out.bin -s 1 && cmp /tmp/rs_in.bin /tmp/rs_out.bin && echo IDENTICAL" &&
step prof_bench 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python3 bench.py --steps 20 --no-e2e &&
echo SESSION-OK | tee -a $O/progress.log

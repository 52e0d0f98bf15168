#!/bin/bash
# Round-2 session B: host pipeline sweep (streams x copy-in split x 2-D copies x slice), the
# reference's k-sweep on the GPU, bin/RS 1 GiB encode/decode at -s 1 and -s 4.
O=gpurun_out/r02b
source "$(dirname "$0")/gpustep.sh"
step pipe_bench 300 python scripts/pipe_bench.py &&
step pipe_bench_dec 300 python scripts/pipe_bench.py --m 1 --streams 1,4 --slices 33554432 &&
step sweep_gpu 600 python scripts/sweep.py --part gpu --out $O/sweep_gpu.json &&
step mkfile 120 python -c "import os; open('/tmp/rs_in.bin','wb').write(os.urandom((1<<30)+12345))" &&
step rs_encode_s1 120 bin/RS -k 10 -n 14 -e /tmp/rs_in.bin -s 1 &&
step rs_encode_s4 120 bin/RS -k 10 -n 14 -e /tmp/rs_in.bin -s 4 &&
step rs_decode_s4 120 bash -c "printf '/tmp/_%d_rs_in.bin\n' 0 2 3 5 6 8 10 11 12 13 > /tmp/rs_conf && bin/RS -d -i /tmp/rs_in.bin -c /tmp/rs_conf -o /tmp/rs_out.bin -s 4 && cmp /tmp/rs_in.bin /tmp/rs_out.bin && echo IDENTICAL" &&
step rs_decode_s1 120 bash -c "bin/RS -d -i /tmp/rs_in.bin -c /tmp/rs_conf -o /tmp/rs_out.bin -s 1 && cmp /tmp/rs_in.bin /tmp/rs_out.bin && echo IDENTICAL" &&
echo SESSION-OK | tee -a $O/progress.log

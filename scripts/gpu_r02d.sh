#!/bin/bash
# Round-2 session D: GPU tests after the pipeline changes, bin/RS 1 GiB cold encode/decode at -s 1
# and -s 4, headline bench (+e2e), wide-stripe bench + PMC passes of the FP4 kernel (k=128, p=32).
O=gpurun_out/r02d
source "$(dirname "$0")/gpustep.sh"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step mkfile 120 python -c "import os; open('/tmp/rs_in.bin','wb').write(os.urandom((1<<30)+12345))" &&
step rs_encode_s1 120 bin/RS -k 10 -n 14 -e /tmp/rs_in.bin -s 1 &&
step rs_encode_s4 120 bin/RS -k 10 -n 14 -e /tmp/rs_in.bin -s 4 &&
step rs_decode_s4 120 bash -c "printf '/tmp/_%d_rs_in.bin\n' 0 2 3 5 6 8 10 11 12 13 > /tmp/rs_conf && bin/RS -d -i /tmp/rs_in.bin -c /tmp/rs_conf -o /tmp/rs_out.bin -s 4 && cmp /tmp/rs_in.bin /tmp/rs_out.bin && echo IDENTICAL" &&
step rs_decode_s1 120 bash -c "bin/RS -d -i /tmp/rs_in.bin -c /tmp/rs_conf -o /tmp/rs_out.bin -s 1 && cmp /tmp/rs_in.bin /tmp/rs_out.bin && echo IDENTICAL" &&
step bench 300 python bench.py --steps 20 --warmup 5 &&
step bench_k128n160 300 python bench.py --preset k128n160 --steps 20 --no-e2e &&
step prof_k128n160 300 rocprofv3 --kernel-trace --stats -d $O/prof_k128n160 -o run --output-format csv -- python3 bench.py --preset k128n160 --steps 10 --no-e2e &&
step pmc_fp4 600 env PMC_DIR=$O/pmc bash scripts/pmc_one.sh fp4_k128_m32 "--k 128 --m 32 --engine mfma" &&
echo SESSION-OK | tee -a $O/progress.log

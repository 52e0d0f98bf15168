#!/bin/bash
# Round-2 session AA: default bench (e2e decode now erases the first e natives), the wide-stripe
# preset, and HBM-byte PMC passes (FETCH_SIZE / WRITE_SIZE / SQ issue counters, each its own run,
# kernel-trace beside for durations) of the headline encode and decode kernels.
O=gpurun_out/r02aa
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
P=$O/pmc
mkdir -p $P
step bench 300 python bench.py --steps 20 --warmup 5 &&
step bench_k128n160 300 python bench.py --preset k128n160 --steps 20 &&
step pmc_enc_fetch 90 timeout -s KILL 80 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $P/enc_fetch -o run --output-format csv -- python3 scripts/prof_case.py --k 10 --m 4 --iters 3 &&
step pmc_enc_write 90 timeout -s KILL 80 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $P/enc_write -o run --output-format csv -- python3 scripts/prof_case.py --k 10 --m 4 --iters 3 &&
step pmc_enc_sq 90 timeout -s KILL 80 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $P/enc_sq -o run --output-format csv -- python3 scripts/prof_case.py --k 10 --m 4 --iters 3 &&
step pmc_dec_fetch 90 timeout -s KILL 80 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $P/dec_fetch -o run --output-format csv -- python3 scripts/prof_case.py --k 10 --m 4 --copies 6 --iters 3 &&
step pmc_dec_write 90 timeout -s KILL 80 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $P/dec_write -o run --output-format csv -- python3 scripts/prof_case.py --k 10 --m 4 --copies 6 --iters 3 &&
step pmc_dec_sq 90 timeout -s KILL 80 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $P/dec_sq -o run --output-format csv -- python3 scripts/prof_case.py --k 10 --m 4 --copies 6 --iters 3 &&
echo SESSION-OK | tee -a $O/progress.log

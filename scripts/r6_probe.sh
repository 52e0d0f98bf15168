#!/bin/bash
# Round-6 probes: FP4 MFMA rate by shape, config #4's (k = 16) pattern ceiling and kernel variants,
# and the wide-stripe step with one lane against two. Each step under its own time limit, && chained.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6c}; mkdir -p $O
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; return $rc; }
st mfma_rate 120 bin/mfma_rate 20000 &&
st membench_k16 240 bin/membench k16 5 &&
st kbench_k16 500 python3 -u scripts/kbench.py --bytes 8589934592 --cases enc_k16_p4,dec_k16_e4_copy12 \
   --variants "None;1,0,1;1,2,1;1,4,1;2,2,1" --rounds 3 --reps 3 &&
st k128_l2_a 200 python3 -u bench.py --preset k128n160 --steps 20 --warmup 5 &&
st k128_l1_a 200 python3 -u bench.py --preset k128n160 --steps 20 --warmup 5 --lanes 1 &&
st k128_l2_b 200 python3 -u bench.py --preset k128n160 --steps 20 --warmup 5 &&
st k128_l1_b 200 python3 -u bench.py --preset k128n160 --steps 20 --warmup 5 --lanes 1 &&
st k16_l2 200 python3 -u bench.py --preset k16n20_8g --steps 10 --warmup 3 &&
st k16_l1 200 python3 -u bench.py --preset k16n20_8g --steps 10 --warmup 3 --lanes 1

#!/bin/bash
# Round-6 probe 2: config #4's rows at power-of-two pitch vs padded pitches (no-math ceiling), and
# the k16n20_8g step with one lane against two, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6d}; mkdir -p $O
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; return $rc; }
st membench_k16_pitch 300 bin/membench k16 5 512 514 516 520 544 576 640 &&
st k16_l2_a 200 python3 -u bench.py --preset k16n20_8g --steps 10 --warmup 3 &&
st k16_l1_a 200 python3 -u bench.py --preset k16n20_8g --steps 10 --warmup 3 --lanes 1 &&
st k16_l2_b 200 python3 -u bench.py --preset k16n20_8g --steps 10 --warmup 3 &&
st k16_l1_b 200 python3 -u bench.py --preset k16n20_8g --steps 10 --warmup 3 --lanes 1 &&
st k16_l2_c 200 python3 -u bench.py --preset k16n20_8g --steps 10 --warmup 3 &&
st k16_l1_c 200 python3 -u bench.py --preset k16n20_8g --steps 10 --warmup 3 --lanes 1

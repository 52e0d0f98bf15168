#!/bin/bash
# Round-6 probe 3: HBM placement of large rows — no-math ceilings of the k = 16 patterns over row
# pitches at three row lengths, then the k16n20_8g step (one lane) with alloc_rows' pitch skewed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6e}; mkdir -p $O
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; return $rc; }
st mb512 300 bin/membench k16 5 512 512 516 520 528 544 576 608 640 &&
st mb128 200 bin/membench k16 5 128 128 130 136 144 160 192 &&
st mb1024 300 bin/membench k16 3 1024 1024 1032 1088 1152 1280 &&
for r in a b; do
  for sk in 0 8388608 67108864 134217728; do
    st k16_s${sk}_$r 200 env GFRS_TUNE=row_skew=$sk python3 -u bench.py --preset k16n20_8g --steps 10 --warmup 3 --lanes 1 || exit 1
  done
done

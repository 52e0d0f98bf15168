#!/bin/bash
# Round-6 probe 4: the k16n20_8g config child's exact command (20 steps, 5 warmup) with the new
# quarter pitch skew against none, and one lane against two, alternating on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6g}; mkdir -p $O
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; return $rc; }
for r in a b c; do
  st k16_def_$r 200 python3 -u bench.py --preset k16n20_8g --steps 20 --warmup 5 &&
  st k16_noskew_$r 200 env GFRS_TUNE=row_skew=0 python3 -u bench.py --preset k16n20_8g --steps 20 --warmup 5 &&
  st k16_l2_$r 200 python3 -u bench.py --preset k16n20_8g --steps 20 --warmup 5 --lanes 2 || exit 1
done

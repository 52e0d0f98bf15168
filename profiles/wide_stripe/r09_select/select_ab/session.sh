#!/bin/bash
# Round-6 probe 11: same-box A/B of the tile-major fused-copy address as a select (default) against
# the branchy form (GFRS_TUNE=tm_old=1): kernel medians and the k128n160 step, interleaved.
#   usage: r6_probe11.sh OUT [ROUNDS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6t}; mkdir -p $O
R=${2:-3}
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -ne 0 ] && tail -5 $O/$n.log; return $rc; }
for r in $(seq 1 $R); do
  st shapes_new_$r 200 python3 -u scripts/fp4_shapes.py 20,22,24,26 || exit 1
  st shapes_old_$r 200 env GFRS_TUNE=tm_old=1 python3 -u scripts/fp4_shapes.py 20,22,24,26 || exit 1
done
for r in $(seq 1 $R); do
  st k128_new_$r 200 python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
  st k128_old_$r 200 env GFRS_TUNE=tm_old=1 python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
done
echo PROBE11-OK

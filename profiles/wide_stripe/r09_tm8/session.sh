#!/bin/bash
# Round-6 probe 8: the tile-major FP4 kernel at 8 tiles (uniform inputs, no copies: the k = 128,
# p = 32 encode) against the A-resident kernel: bit-exact checks, kernel medians, k128n160 step.
#   usage: r6_probe8.sh OUT [ROUNDS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6m}; mkdir -p $O
R=${2:-3}
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -ne 0 ] && tail -5 $O/$n.log; return $rc; }
st check_tm 300 env GFRS_TUNE=fp4=tm python3 -u scripts/fp4_check.py || exit 1
st check_def 300 python3 -u scripts/fp4_check.py || exit 1
for r in $(seq 1 $R); do
  st shapes_ar_$r 200 env GFRS_TUNE=fp4=ar python3 -u scripts/fp4_shapes.py 29,32 || exit 1
  st shapes_tm_$r 200 env GFRS_TUNE=fp4=tm python3 -u scripts/fp4_shapes.py 29,32 || exit 1
done
for r in $(seq 1 $R); do
  st k128_def_$r 200 python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
  st k128_tm_$r 200 env GFRS_TUNE=fp4=tm python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
done

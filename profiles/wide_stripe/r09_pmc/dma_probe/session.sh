#!/bin/bash
# Round-6 probe 9: the tile-major kernel issuing the next chunk's 8 LDS-DMAs 1 / 2 / 4 per
# super-step of group 0 (GFRS_TUNE=tm_dps=N): checks, kernel medians, k128n160 step.
#   usage: r6_probe9.sh OUT [ROUNDS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6o}; mkdir -p $O
R=${2:-2}
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -ne 0 ] && tail -5 $O/$n.log; return $rc; }
st check_2 300 env GFRS_TUNE=tm_dps=2 python3 -u scripts/fp4_check.py || exit 1
st check_4 300 env GFRS_TUNE=tm_dps=4 python3 -u scripts/fp4_check.py || exit 1
for r in $(seq 1 $R); do
  for d in 1 2 4; do
    st shapes_d${d}_$r 200 env GFRS_TUNE=tm_dps=$d python3 -u scripts/fp4_shapes.py 20,22,24,26 || exit 1
  done
done
for r in $(seq 1 $R); do
  for d in 1 2; do
    st k128_d${d}_$r 200 env GFRS_TUNE=tm_dps=$d python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
  done
done

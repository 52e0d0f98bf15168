#!/bin/bash
# Round-6 probe 7: the tile-major FP4 kernel at 6 tiles with fused copies, without the scratch
# spills (row indices laundered so the per-slot LDS addresses are not hoisted), with and without the
# early pack of the second-to-last group (GFRS_TUNE=tm_early=1), against v1.
#   usage: r6_probe7.sh OUT [ROUNDS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6k}; mkdir -p $O
R=${2:-2}
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; return $rc; }
st check_tm 240 env GFRS_TUNE=fp4=tm python3 -u scripts/fp4_check.py || exit 1
st check_tm_early 240 env GFRS_TUNE=fp4=tm,tm_early=1 python3 -u scripts/fp4_check.py || exit 1
st check_def 240 python3 -u scripts/fp4_check.py || exit 1
for r in $(seq 1 $R); do
  st shapes_v1_$r 200 env GFRS_TUNE=fp4=v1 python3 -u scripts/fp4_shapes.py 20,22,24,26 || exit 1
  st shapes_tm_$r 200 env GFRS_TUNE=fp4=tm python3 -u scripts/fp4_shapes.py 20,22,24,26 || exit 1
  st shapes_tme_$r 200 env GFRS_TUNE=fp4=tm,tm_early=1 python3 -u scripts/fp4_shapes.py 20,22,24,26 || exit 1
done
for r in $(seq 1 $R); do
  st k128_def_$r 200 python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
  st k128_tm_$r 200 env GFRS_TUNE=fp4=tm python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
  st k128_tme_$r 200 env GFRS_TUNE=fp4=tm,tm_early=1 python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
done

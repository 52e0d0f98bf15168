#!/bin/bash
# Round-6 probe 10: the tile-major decode with its fused-copy address as a select instead of a
# divergent branch: checks, kernel medians (tm and v1 forced), k128n160 step, PMC pass.
#   usage: r6_probe10.sh OUT [ROUNDS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6s}; mkdir -p $O
R=${2:-2}
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -ne 0 ] && tail -5 $O/$n.log; return $rc; }
st check 300 python3 -u scripts/fp4_check.py || exit 1
for r in $(seq 1 $R); do
  st shapes_tm_$r 200 python3 -u scripts/fp4_shapes.py 20,22,24,26 || exit 1
  st shapes_v1_$r 200 env GFRS_TUNE=fp4=v1 python3 -u scripts/fp4_shapes.py 20,22,24 || exit 1
done
for r in $(seq 1 $R); do
  st k128_$r 200 python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
done
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
for cfg in "tm6c:--k 128 --m 24 --copies 104 --engine mfma" "tm7c:--k 128 --m 26 --copies 102 --engine mfma"; do
  name=${cfg%%:*}; args=${cfg#*:}
  echo "[$(date +%T)] pmc_$name"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P1 -d $O/pmc_$name -o run --output-format csv -- \
    python3 scripts/prof_case.py --iters 3 $args > $O/pmc_$name.log 2>&1 || exit 1
done
echo PROBE10-OK

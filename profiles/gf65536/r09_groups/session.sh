#!/bin/bash
# Round-6 probe 6: GF(2^16) vector kernel with four 16-byte groups per lane (GFRS_TUNE=gf16_vec_g=4)
# against two (the default): correctness under the forced setting, then the k10n14_w16 preset
# interleaved over rounds.   usage: r6_probe6.sh OUT [ROUNDS] [STEPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6j}; mkdir -p $O
R=${2:-3}; S=${3:-200}
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; return $rc; }
st tests_g4 300 env GFRS_TUNE=gf16_vec_g=4 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gf16w.py || exit 1
for r in $(seq 1 $R); do
  for g in 2 4; do
    st w16_g${g}_$r 200 env GFRS_TUNE=gf16_vec_g=$g python3 -u bench.py --preset k10n14_w16 --steps $S --warmup 10 || exit 1
  done
done

#!/bin/bash
# Round-6 probe 5: does the wide stripe's row placement matter? k128n160 (8 MiB rows at an 8 MiB
# pitch) with 2 / 4 / 6 MiB added to every large row's pitch, interleaved with the default.
# usage: r6_probe5.sh OUT [ROUNDS] [STEPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6h}; mkdir -p $O
R=${2:-2}; S=${3:-20}
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; return $rc; }
for r in $(seq 1 $R); do
  for x in 0 2097152 4194304 6291456; do
    st k128_x${x}_$r 200 env GFRS_TUNE=row_extra=$x python3 -u bench.py --preset k128n160 --steps $S --warmup 10 || exit 1
  done
done

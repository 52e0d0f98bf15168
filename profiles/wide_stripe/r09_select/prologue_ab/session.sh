#!/bin/bash
# Round-6 probe 12: the A-resident kernel's prologue with its 64 A loads issued back to back
# (default) against the conditional load + tie per fragment (GFRS_TUNE=ar_oldpro=1): the ar GPU
# tests, batched serving launches (RS(128,160), 16 / 256 objects of 64 KiB / 1 MiB) and the
# k128n160 step, interleaved.   usage: r6_probe12.sh OUT [ROUNDS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6u}; mkdir -p $O
R=${2:-2}
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -ne 0 ] && tail -5 $O/$n.log; return $rc; }
st tests 400 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "a_resident or fp4" || exit 1
st check 300 python3 -u scripts/fp4_check.py || exit 1
for r in $(seq 1 $R); do
  st serve_new_$r 300 python3 -u scripts/serve_bench.py --code 128:160 --sizes 65536,1048576 --batches 16,256 --reps 10 --out $O/serve_new_$r.jsonl || exit 1
  st serve_old_$r 300 env GFRS_TUNE=ar_oldpro=1 python3 -u scripts/serve_bench.py --code 128:160 --sizes 65536,1048576 --batches 16,256 --reps 10 --out $O/serve_old_$r.jsonl || exit 1
done
for r in $(seq 1 $R); do
  st k128_new_$r 200 python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
  st k128_old_$r 200 env GFRS_TUNE=ar_oldpro=1 python3 -u bench.py --preset k128n160 --steps 200 --warmup 10 || exit 1
done
echo PROBE12-OK

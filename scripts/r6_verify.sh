#!/bin/bash
# Round-6 verification on the current tree: the GPU suite + smoke, the driver's bench command (twice),
# the GF(2^16) solve bench, and the 64 GiB one-stripe preset (its rows' pitch changed this round).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6f}; mkdir -p $O
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -ne 0 ] && tail -20 $O/$n.log; return $rc; }
st pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread &&
st smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" &&
st bench1 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 &&
st decsys16 300 python3 -u scripts/decsys16_bench.py &&
st k16n20_64g 600 python3 -u bench.py --preset k16n20_64g --steps 5 --warmup 1 &&
st bench2 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5

#!/bin/bash
# Round-6 final verification on the current tree: the GPU suite + smoke, the driver's bench command
# twice, and a kernel trace of the k128n160 preset (which FP4 forms its steps dispatch).
#   usage: r6_final.sh OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/${1:-r6l}; mkdir -p $O
st() { local n=$1 s=$2; shift 2; echo "[$(date +%T)] $n"; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc"; [ $rc -ne 0 ] && tail -20 $O/$n.log; return $rc; }
st pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread &&
st smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" &&
st bench1 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 &&
st prof_k128 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_k128 -o run -- python3 -u bench.py --preset k128n160 --steps 40 --warmup 5 &&
st bench2 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5

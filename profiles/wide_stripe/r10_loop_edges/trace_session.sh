set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/r7c; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/k128 -o run -- python3 bench.py --preset k128n160 --steps 20 --warmup 5 --no-e2e --configs none > $O/k128.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/k10 -o run -- python3 bench.py --preset k10n14 --steps 20 --warmup 5 --no-e2e --configs none > $O/k10.log 2>&1 &&
echo DONE

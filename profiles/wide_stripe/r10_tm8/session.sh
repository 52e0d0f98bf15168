# 8-tile tile-major FP4 kernel (tile 7's A in registers): GPU tests, shape A/B, k128n160 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/r7e; mkdir -p $O
echo "[$(date +%T)] tests"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "tile_major or router or forced_forms" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for kk in v1 tm ar; do
    echo "[$(date +%T)] shapes $kk $r"
    GFRS_TUNE=fp4=$kk timeout -k 10 150 python3 -u scripts/fp4_shapes.py 29,30,32 > $O/shapes_${kk}_$r.json 2> $O/shapes_${kk}_$r.err || exit 1
  done
done
for r in 1 2; do
  for kk in tm8=0 tm8=1; do
    echo "[$(date +%T)] k128 $kk $r"
    GFRS_TUNE=$kk timeout -k 10 200 python3 -u bench.py --preset k128n160 --steps 100 --warmup 5 --no-e2e --configs none > $O/k128_${kk}_$r.json 2> $O/k128_${kk}_$r.err || exit 1
  done
done
echo DONE

set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/r6a; mkdir -p $O
for r in 1 2; do
  for kk in v1 tm; do
    echo "[$(date +%T)] shapes $kk $r"
    GFRS_TUNE=fp4=$kk timeout -k 10 150 python3 -u scripts/fp4_shapes.py 20,22,24,26 > $O/shapes_${kk}_$r.json 2> $O/shapes_${kk}_$r.err || exit 1
  done
done
for r in 1 2; do
  for kk in "" tm; do
    echo "[$(date +%T)] k128 '$kk' $r"
    GFRS_TUNE=fp4=$kk timeout -k 10 200 python3 -u bench.py --preset k128n160 --steps 20 --warmup 5 > $O/k128_${kk:-def}_$r.json 2> $O/k128_${kk:-def}_$r.err || exit 1
  done
done
echo "[$(date +%T)] bench"
timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err

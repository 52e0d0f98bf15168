set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/r7h; mkdir -p $O
for r in 1 2; do
  for v in "--lanes 2" "--lanes 3" "--lanes 2 --side-priority" "--lanes 1"; do
    t=$(echo $v | tr -d ' -')
    timeout -k 10 200 python3 -u bench.py --preset k128n160 --steps 100 --warmup 5 --no-e2e --configs none $v > $O/k128_${t}_$r.log 2>&1 || { echo FAIL $v; exit 1; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open('$O/k128_${t}_$r.log') if l.startswith('{')][-1]; print('$v', $r, d['ms_per_step'], d.get('verified'))" | tee -a $O/summary.txt
  done
done

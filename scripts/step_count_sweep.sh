#!/bin/bash
# ms/step against the number of timed steps (startup cost of a timed loop = intercept of
# total time vs K). Usage: scripts/step_count_sweep.sh OUTDIR "PRESETS" "STEPS" [extra bench args]
# Every run is its own process under its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=${1:?outdir}; PRESETS=${2:-"k10n14 k128n160"}; STEPS=${3:-"10 20 40 200"}; shift 3
mkdir -p "$O"
for rep in 1 2; do
  for p in $PRESETS; do
    for s in $STEPS; do
      f="$O/${p}_s${s}_r${rep}.log"
      timeout -k 10 120 python3 -u bench.py --preset "$p" --steps "$s" --warmup 5 --no-e2e --configs none "$@" > "$f" 2>&1 || {
        echo "FAILED $p $s rc=$?"; tail -5 "$f"; exit 1; }
      python3 - "$f" "$p" "$s" <<'EOF' | tee -a "$O/summary.txt"
import json, sys
rec = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(f"{sys.argv[2]} steps={sys.argv[3]} ms_per_step={rec['ms_per_step']} verified={rec.get('verified')}")
EOF
    done
  done
done

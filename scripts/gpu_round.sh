#!/bin/bash
# One GPU-box session: tests, headline bench (+graph, +e2e), BASELINE presets, streaming file codec
# and a rocprofv3 kernel/marker trace. Every GPU step has its own time limit; the first failure ends
# the script (pool rules: no further GPU work after a fault / timeout).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/round
mkdir -p $O
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a $O/progress.log
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/progress.log
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -x &&
step bench 180 python bench.py &&
step bench_graph 180 python bench.py --graph &&
step bench_e2e 300 python bench.py --e2e --steps 20 &&
step bench_k128n160 300 python bench.py --preset k128n160 --steps 20 &&
step bench_k128n160_valu 300 python bench.py --preset k128n160 --steps 20 --engine valu &&
step bench_k16n20 300 python bench.py --preset k16n20_8g --steps 10 &&
step bench_k4n6 180 python bench.py --preset k4n6 &&
step mkfile 120 python -c "import os; open('/tmp/rs_in.bin','wb').write(os.urandom((1<<30)+12345))" &&
step stream_encode 300 bin/RS -k 10 -n 14 -e /tmp/rs_in.bin --window 0 --no-sync -s 4 &&
step stream_decode 300 bash -c "printf '/tmp/_%d_rs_in.bin\n' 0 2 3 5 6 8 10 11 12 13 > /tmp/rs_conf && bin/RS -d -i /tmp/rs_in.bin -c /tmp/rs_conf -o /tmp/rs_out.bin --window 0 --no-sync -s 4 && cmp /tmp/rs_in.bin /tmp/rs_out.bin && echo IDENTICAL" &&
step inmem_encode 300 bin/RS -k 10 -n 14 -e /tmp/rs_in.bin -s 4 &&
step prof_stream 300 rocprofv3 --kernel-trace --marker-trace --stats -d $O/prof_stream -o run --output-format csv -- bin/RS -k 10 -n 14 -e /tmp/rs_in.bin --window 0 --no-sync -s 4 &&
step prof_bench 300 rocprofv3 --kernel-trace --marker-trace --stats -d $O/prof_bench -o run --output-format csv -- python3 bench.py --steps 20 &&
step prof_k128n160 300 rocprofv3 --kernel-trace --stats -d $O/prof_k128n160 -o run --output-format csv -- python3 bench.py --preset k128n160 --steps 20 &&
echo ROUND-OK | tee -a $O/progress.log

#!/bin/bash
# One GPU-box session: build, kernel tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit and the steps are chained with &&: after a failure,
# timeout or fault nothing else touches the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== build" && timeout -k 10 600 make -C csrc -j16 > gpurun_out/build.log 2>&1 \
&& echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 \
&& tail -3 gpurun_out/pytest_gpu.log \
&& echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& cat gpurun_out/smoke.log \
&& echo "== bench" && timeout -k 10 600 python bench.py --steps 50 --warmup 5 --e2e > gpurun_out/bench.log 2>&1 \
&& cat gpurun_out/bench.log \
&& echo "== rocprof" && cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}" \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/prof.log 2>&1 \
&& echo "done"

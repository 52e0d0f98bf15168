set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GPURS_NO_BUILD=1
O=gpurun_out/r7p; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_gf16w.py -m gpu -x -q --timeout 200 --timeout-method thread -k "w16 or gf16 or blocked or system16 or decode" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/decsys16_bench.py 1000:2000:1000,4000:4500:500,2000:2100:100 > $O/ds.log 2>&1

#!/bin/bash
# Round-2 session AJ: final tree after the CPU-codec change (rebuilt _cpu.so, bin/RS): GPU suite,
# smoke, default bench.
O=${O:-gpurun_out/r02aj}
source "$(dirname "$0")/gpustep.sh"
export GPURS_NO_BUILD=1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE-OK')" &&
step bench 300 python bench.py --steps 20 --warmup 5 &&
step cpu_avx2 60 python -c "import torch; from gpu_rscode_amd import ReedSolomon; import time; d=torch.randint(0,256,(10,1<<24),dtype=torch.uint8); rs=ReedSolomon(10,14); p=rs.encode(d); t=time.perf_counter(); rs.encode(d,p); print('cpu simd 1-thread GB/s', round(10*(1<<24)/(time.perf_counter()-t)/1e9,2)); print(open('/proc/cpuinfo').read().count('avx2')>0)" &&
echo SESSION-OK | tee -a $O/progress.log

#!/bin/bash
# PMC counter passes (kernel-trace only, no sys/runtime trace — see the pool rules) for the
# headline encode, the 4-erasure decode and the wide-stripe kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
P="python3 scripts/prof_case.py --iters 3"
run() {  # name, counters, args...
  local name=$1; shift; local ctr=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pmc/$name -o run --output-format csv -- $P "$@" \
    > gpurun_out/pmc/$name.log 2>&1
}
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_MFMA"
C2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
C3="FETCH_SIZE"
C4="WRITE_SIZE"
for cfg in "enc10:--k 10 --m 4" "dec10:--k 10 --m 4 --copies 6" "wide_valu:--k 128 --m 32" "wide_mfma:--k 128 --m 32 --engine mfma"; do
  name=${cfg%%:*}; args=${cfg#*:}
  run ${name}_c1 "$C1" $args && run ${name}_c2 "$C2" $args && run ${name}_c3 "$C3" $args && run ${name}_c4 "$C4" $args || exit 1
done
echo counters-done

#!/bin/bash
# One-case PMC passes: scripts/pmc_one.sh NAME "prof_case args" — kernel-trace + counters only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PMC_DIR=${PMC_DIR:-gpurun_out/pmc}; mkdir -p $PMC_DIR
export TMPDIR=/tmp
name=$1; shift
args=$1
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $PMC_DIR/${name}_$i -o run --output-format csv -- \
    python3 scripts/prof_case.py --iters 3 $args > $PMC_DIR/${name}_$i.log 2>&1 || exit 1
done
echo pmc-done

# rocprofv3 passes over the k = 10, m = 4 encode on the v_perm kernels, GF(2^16) (valu16) against
# GF(2^8) (valu), 1 GiB: is the w = 16 kernel VALU-bound? Run from the repo root on the GPU box;
# summarise with  python scripts/rocpd_summary.py gemm gpurun_out/pk10/*/run_results.db
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for case in w16 w8; do
  if [ $case = w16 ]; then X="--field 16 --engine valu16"; else X="--field 8 --engine valu"; fi
  P="python3 scripts/prof_case.py --k 10 --m 4 $X --iters 5"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pk10/${case}_trace -o run -- $P > gpurun_out/pk10_${case}_trace.log 2>&1 &&
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU -d gpurun_out/pk10/${case}_pmc1 -o run -- $P > gpurun_out/pk10_${case}_pmc1.log 2>&1 &&
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY -d gpurun_out/pk10/${case}_pmc2 -o run -- $P > gpurun_out/pk10_${case}_pmc2.log 2>&1 || exit 1
done

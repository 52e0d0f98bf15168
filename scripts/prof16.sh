# rocprofv3 passes over the GF(2^16) FP4 matrix-core kernel (gf_mfma16.hip): kernel trace and PMC
# counters for a k=300, m=40 encode and a decode-shaped plan (m=40 outputs plus fused survivor
# copies), 1 GiB. Run from the repo root on the GPU box; summarise with
#   python scripts/rocpd_summary.py gemm16 gpurun_out/p16/*/run_results.db
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for case in enc dec; do
  if [ $case = enc ]; then X=""; else X="--copies 260"; fi
  P="python3 scripts/prof_case.py --k 300 --m 40 $X --field 16 --engine mfma --iters 3"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p16/${case}_trace -o run -- $P > gpurun_out/p16_${case}_trace.log 2>&1 &&
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU -d gpurun_out/p16/${case}_pmc1 -o run -- $P > gpurun_out/p16_${case}_pmc1.log 2>&1 &&
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/p16/${case}_pmc2 -o run -- $P > gpurun_out/p16_${case}_pmc2.log 2>&1 &&
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/p16/${case}_pmc3 -o run -- $P > gpurun_out/p16_${case}_pmc3.log 2>&1 || exit 1
done

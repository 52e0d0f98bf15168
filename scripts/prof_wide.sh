# rocprofv3 passes (kernel trace + 3 PMC passes) over the k=128 FP4 GEMM of one case:
#   M=32 CP=0 bash scripts/prof_wide.sh      (encode, m=32)
#   M=26 CP=102 bash scripts/prof_wide.sh    (decode: 26 rebuilt, 102 fused copies)
# Run from the repo root on the GPU box; summaries land in gpurun_out/pw<M>_summary.json.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 scripts/prof_case.py --k 128 --m ${M:-26} --copies ${CP:-102} --engine mfma --iters 3"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pw${M:-26}/trace -o run -- $P > gpurun_out/pw${M:-26}_trace.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM -d gpurun_out/pw${M:-26}/pmc1 -o run -- $P > gpurun_out/pw${M:-26}_pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/pw${M:-26}/pmc2 -o run -- $P > gpurun_out/pw${M:-26}_pmc2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_FLAT -d gpurun_out/pw${M:-26}/pmc3 -o run -- $P > gpurun_out/pw${M:-26}_pmc3.log 2>&1
python scripts/rocpd_summary.py gemm gpurun_out/pw${M:-26}/*/run_results.db > gpurun_out/pw${M:-26}_summary.json
